#!/usr/bin/env python3
"""Per-batch GPU timeline from a rocprofv3 kernel trace (run_kernel_trace.csv).

Splits the trace into batches at each k_epilogue, then reports, over the steady-state batches:
the epilogue-to-epilogue interval, each queue's busy time, the union busy time, the idle gaps
between consecutive kernels on each queue, and the kernel sequence of one median batch.

    python3 scripts/timeline.py gpurun_out/prof/run_kernel_trace.csv [--skip 10] [--show 1]
"""
import argparse
import csv
import statistics


def short(name):
    n = name.split("(")[0]
    for p in ("void ", "fdbcs::"):
        n = n.replace(p, "")
    return n[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--skip", type=int, default=10, help="batches skipped at the start (warm-up)")
    ap.add_argument("--show", type=int, default=1, help="batches whose kernel sequence is listed")
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], short(r["Kernel_Name"])))
    rows.sort()
    ep = [i for i, r in enumerate(rows) if "k_epilogue" in r[3]]
    if len(ep) < a.skip + 3:
        print("too few batches:", len(ep))
        return
    ep = ep[a.skip:]
    intervals, busy_union, per_q, gaps = [], [], {}, {}
    seqs = []
    for k in range(1, len(ep)):
        t0, t1 = rows[ep[k - 1]][1], rows[ep[k]][1]
        intervals.append((t1 - t0) / 1e3)
        seg = [r for r in rows if r[1] > t0 and r[0] < t1]
        # union of intervals clipped to the batch window
        iv = sorted((max(s, t0), min(e, t1)) for s, e, _, _ in seg)
        u, cs, ce = 0, None, None
        for s, e in iv:
            if ce is None or s > ce:
                if ce is not None:
                    u += ce - cs
                cs, ce = s, e
            else:
                ce = max(ce, e)
        if ce is not None:
            u += ce - cs
        busy_union.append(u / 1e3)
        byq = {}
        for s, e, q, n in seg:
            byq.setdefault(q, []).append((s, e, n))
        for q, ks in byq.items():
            per_q.setdefault(q, []).append(sum(min(e, t1) - max(s, t0) for s, e, _ in ks) / 1e3)
            g = [max(0, ks[i][0] - ks[i - 1][1]) / 1e3 for i in range(1, len(ks))]
            gaps.setdefault(q, []).extend(g)
        seqs.append((t0, seg))
    med = statistics.median
    print(f"batches {len(intervals)}: interval median {med(intervals):.1f} us, mean {statistics.mean(intervals):.1f} us")
    print(f"union busy median {med(busy_union):.1f} us ({med(busy_union) / med(intervals):.0%} of the interval)")
    for q in sorted(per_q):
        g = gaps[q]
        print(f"queue {q}: busy median {med(per_q[q]):.1f} us/batch, {len(g) / len(intervals):.1f} gaps/batch, "
              f"gap median {med(g) if g else 0:.1f} us, gap sum/batch {sum(g) / len(intervals):.1f} us")
    order = sorted(range(len(intervals)), key=lambda i: intervals[i])
    for i in order[len(order) // 2: len(order) // 2 + a.show]:
        t0, seg = seqs[i]
        print(f"-- batch interval {intervals[i]:.1f} us (times relative to the previous epilogue end)")
        for s, e, q, n in seg:
            print(f"  q{q} {(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f}  {n}")


if __name__ == "__main__":
    main()
