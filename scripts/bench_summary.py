"""Summarize bench.py JSON lines (files given on the command line): headline, passes, roofline,
per-kernel table."""
import json
import sys

for f in sys.argv[1:]:
    try:
        d = json.loads([l for l in open(f).read().splitlines() if l.startswith("{")][-1])
    except Exception as e:  # noqa: BLE001
        print(f, "no json", e)
        continue
    print(f"== {f}: {d['config']['workload'][:40]}")
    print("  value %.2fM txns/s  ms/step %.4f  resident %s  total %s" % (
        d["value"] / 1e6, d["ms_per_step"],
        d["device_resident_txns_per_s"] and "%.2fM" % (d["device_resident_txns_per_s"] / 1e6),
        d["total_txns_per_s"] and "%.2fM" % (d["total_txns_per_s"] / 1e6)))
    if d.get("sync"):
        s = d["sync"]
        print("  sync %.2fM txns/s  p50 %.3f ms  p99 %.3f ms" % (s["txns_per_s"] / 1e6, s["latency_ms_p50"], s["latency_ms_p99"]))
    if d.get("device_bound"):
        print("  device-bound %.2fM txns/s  %.4f ms/batch" % (d["device_bound"]["txns_per_s"] / 1e6, d["device_bound"]["ms_per_batch"]))
    print("  host ms/batch", {k: round(v, 4) for k, v in d["host_ms_per_batch"].items()})
    cb = d.get("cpu_baseline")
    if cb:
        print("  cpu %.0f txns/s cores %s  phases %s" % (cb["value"] or 0, cb["cores"],
              {k: round(v, 2) for k, v in cb.get("phase_ms_per_batch", {}).items()}))
    p = d.get("parity")
    if p:
        print("  parity %d/%d mismatched %d" % (p["batches_checked"], p["batches_total"], p["mismatched_batches"]))
    r = d.get("roofline")
    if r:
        print("  roofline %s achieved %.1f GB/s frac %.4f avg %.4f ms (profile %s) bytes %.3g" % (
            r["kernel"], r["achieved"] or 0, r["frac"] or 0, r["avg_launch_ms"], r["profile_avg_launch_ms"],
            r["algorithmic_bytes_per_launch"] or 0))
    print("  sort phase", d.get("sort_phase"))
    if d.get("phase_ms_per_batch"):
        print("  phases", {k: round(v, 4) for k, v in d["phase_ms_per_batch"].items()})
    for k, v in list(d["kernels"].items())[:24]:
        print("    %-52s n=%4d avg=%.4f ms tot=%.3f frac=%s" % (k[:52], v["launches"], v["avg_launch_ms"], v["total_ms"],
                                                            v["frac"] and round(v["frac"], 3)))
