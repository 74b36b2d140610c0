#!/usr/bin/env python3
"""Where a pipelined batch waits: per-batch kernel starts and ends from a rocprofv3 kernel trace of
bench.py's timed loop, with each cross-stream hand-off's latency (the consumer's start minus the
producer's end) and each chain's busy time.  The n-th launch of a kernel name is batch n's (every
per-batch kernel runs once per batch; compaction / GC kernels are listed apart).

    python3 scripts/crit_path.py run_kernel_trace.csv [--skip 20]
"""
import argparse
import csv
import statistics
from collections import defaultdict

A = ["k_sort_partition", "k_sort_bucket", "EdgePairScan", "k_edge_fill"]
X = ["k_check_lanes", "k_resolve_pre", "k_resolve<", "k_combine"]
Y = ["k_seg_prep", "BatchIns", "k_epilogue"]


def key(name):
    for k in A + X + Y:
        if k in name:
            return k
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--skip", type=int, default=20)
    ap.add_argument("--copies", help="memory_copy_trace.csv of the same run: the batches' H2D uploads")
    a = ap.parse_args()
    occ = defaultdict(list)
    other = defaultdict(list)
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            k = key(r["Kernel_Name"])
            (occ[k] if k else other[r["Kernel_Name"].split("(")[0][:50]]).append((s, e, r["Queue_Id"]))
    for k in occ:
        occ[k].sort()
    # the check may be two kernels per batch (split): keep the later-ending one per batch as "check"
    n = min(len(v) for k, v in occ.items() if k != "k_check_lanes")
    # extra launches before the first batch (the history's initial index build runs k_epilogue)
    for k in occ:
        if k != "k_check_lanes" and len(occ[k]) > n:
            print(f"{k}: {len(occ[k]) - n} launches before the first batch dropped")
            occ[k] = occ[k][len(occ[k]) - n:]
    checks = occ.get("k_check_lanes", [])
    per = len(checks) // n if n else 1
    if per > 1:
        print(f"{per} check launches per batch: grouped")
        grp = [checks[i * per:(i + 1) * per] for i in range(n)]
        occ["k_check_lanes"] = [(min(x[0] for x in g), max(x[1] for x in g), g[0][2]) for g in grp]
    B = range(a.skip, n - 4)
    if a.copies:  # one H2D per batch, the largest ones (the packed batches), in order
        cp = []
        with open(a.copies) as f:
            for r in csv.DictReader(f):
                if "HOST_TO_DEVICE" in r.get("Direction", "") or "HOST_TO_DEVICE" in str(r):
                    cp.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r.get("Size", 0) or 0)))
        cp.sort()
        if cp:
            big = max(c[2] for c in cp)
            up = [c for c in cp if c[2] >= big // 2]
            print(f"uploads: {len(up)} H2D copies >= {big // 2} bytes (largest {big})")
            occ["upload"] = [(s_, e_, "dma") for s_, e_, _ in up[len(up) - n:]] if len(up) >= n else []

    def st(k, i):
        return occ[k][i][0]

    def en(k, i):
        return occ[k][i][1]

    us = lambda v: v / 1e3
    ends = [en("k_epilogue", i) for i in range(n)]
    iv = [us(ends[i + 1] - ends[i]) for i in B]
    print(f"batches {n}, steady {len(B)}: epilogue-to-epilogue median {statistics.median(iv):.1f} us, mean {statistics.mean(iv):.1f}")
    rows = {
        "A busy (partition start..edge_fill end)": lambda i: en("k_edge_fill", i) - st("k_sort_partition", i),
        "A kernels sum": lambda i: sum(en(k, i) - st(k, i) for k in A),
        "X busy (check start..combine end)": lambda i: en("k_combine", i) - st("k_check_lanes", i),
        "X kernels sum": lambda i: sum(en(k, i) - st(k, i) for k in X),
        "Y busy (seg_prep start..epilogue end)": lambda i: en("k_epilogue", i) - st("k_seg_prep", i),
        "Y kernels sum": lambda i: sum(en(k, i) - st(k, i) for k in Y),
        "hand-off A(i) -> pre(i)": lambda i: st("k_resolve_pre", i) - max(en("k_edge_fill", i), en("k_check_lanes", i)),
        "  pre(i) waits for A (edge_fill end - check end)": lambda i: en("k_edge_fill", i) - en("k_check_lanes", i),
        "hand-off combine(i) -> seg_prep(i)": lambda i: st("k_seg_prep", i) - en("k_combine", i),
        "check(i+1) start - combine(i) end": lambda i: st("k_check_lanes", i + 1) - en("k_combine", i),
        "check(i+1) start - epilogue(i-1) end": lambda i: st("k_check_lanes", i + 1) - en("k_epilogue", i - 1),
        "partition(i+1) start - edge_fill(i) end": lambda i: st("k_sort_partition", i + 1) - en("k_edge_fill", i),
        "partition(i+3) start - epilogue(i) end": lambda i: st("k_sort_partition", i + 3) - en("k_epilogue", i),
        "seg_prep(i+1) start - epilogue(i) end": lambda i: st("k_seg_prep", i + 1) - en("k_epilogue", i),
        "latency partition(i) start -> epilogue(i) end": lambda i: en("k_epilogue", i) - st("k_sort_partition", i),
    }
    if occ.get("upload"):
        rows["upload duration"] = lambda i: en("upload", i) - st("upload", i)
        rows["upload(i+1) start - upload(i) end"] = lambda i: st("upload", i + 1) - en("upload", i)
        rows["partition(i) start - upload(i) end"] = lambda i: st("k_sort_partition", i) - en("upload", i)
        rows["check(i) start - upload(i) end"] = lambda i: st("k_check_lanes", i) - en("upload", i)
    for name, f in rows.items():
        v = [us(f(i)) for i in B]
        print(f"  {name:52s} median {statistics.median(v):8.1f}  p10 {sorted(v)[len(v) // 10]:8.1f}  p90 {sorted(v)[9 * len(v) // 10]:8.1f}")
    print("per kernel (median duration, us):")
    for k in A + X + Y:
        v = [us(en(k, i) - st(k, i)) for i in B]
        print(f"  {k:20s} {statistics.median(v):7.1f}   queue {occ[k][a.skip][2]}")
    for k, v in sorted(other.items(), key=lambda kv: -sum(e - s for s, e, _ in kv[1]))[:6]:
        print(f"  other {k:44s} calls {len(v):4d} avg {us(sum(e - s for s, e, _ in v) / len(v)):8.1f}")


if __name__ == "__main__":
    main()
