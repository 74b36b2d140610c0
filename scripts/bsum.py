"""One-screen summary of bench JSON lines (value, passes, parity, host split, roofline)."""
import json
import sys

for f in sys.argv[1:]:
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(f, "unreadable", e)
        continue
    g = lambda k: (d.get(k) or 0) / 1e6  # noqa: E731
    print(f"{f}: value {d['value']/1e6:.2f}M total {g('total_txns_per_s'):.2f}M h2d {g('h2d_inclusive_txns_per_s'):.2f}M "
          f"sync {g('sync_txns_per_s'):.2f}M devbound {(d.get('device_bound') or {}).get('txns_per_s', 0)/1e6:.2f}M")
    p = d.get("parity") or {}
    print(f"  parity {p.get('batches_checked')}/{p.get('batches_total')} bad {p.get('mismatched_batches')} mix {d.get('verdict_mix')}")
    print("  host", {k: round(v, 4) for k, v in (d.get("host_ms_per_batch") or {}).items()})
    print("  total_host", {k: round(v, 4) for k, v in (d.get("total_host_ms_per_batch") or {}).items()})
    r = d.get("roofline") or {}
    print(f"  roof {r.get('kernel')} frac {r.get('frac')} rocprof {r.get('frac_rocprof')} avg_ms {r.get('avg_launch_ms')} "
          f"alg {r.get('algorithmic_bytes_per_launch')} traffic {r.get('traffic')}")
    ks = d.get("kernels") or {}
    print("  top kernels:", ", ".join(f"{k} {v['avg_launch_ms']*1e3:.1f}us x{v['launches']}" for k, v in list(ks.items())[:8]))
    print("  x_launches_skipped", d.get("x_launches_skipped"), "compactions", d.get("compactions"))
    cb = d.get("cpu_baseline") or {}
    print(f"  cpu {cb.get('value')}")
