#!/usr/bin/env python3
"""Steady-state pipeline view from a rocprofv3 kernel trace of a bench run with only the timed
region (--resident-steps 0 --breakdown-steps 0 --total-steps 0 --no-cpu-baseline).

For the last N batches: the epilogue-to-epilogue interval, each queue's busy share, every kernel's
mean duration, and per batch the span of stage A (k_sample start .. k_edge_fill end), of stage B
(delta check start .. epilogue end) and the idle time inside each stage's chain.

    python3 scripts/pipeline_trace.py gpurun_out/tl/.../run_kernel_trace.csv [--last 80]
"""
import argparse
import csv
import statistics
from collections import defaultdict


def short(name):
    n = name.split("(")[0]
    for p in ("void ", "fdbcs::"):
        n = n.replace(p, "")
    return n[:48]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last", type=int, default=80)
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], short(r["Kernel_Name"])))
    rows.sort()
    ep = [i for i, r in enumerate(rows) if r[3].startswith("k_epilogue")]
    ep = ep[-(a.last + 1):]
    t0, t1 = rows[ep[0]][1], rows[ep[-1]][1]
    win = [r for r in rows if r[0] >= t0 and r[1] <= t1]
    n = len(ep) - 1
    print(f"batches {n}: interval mean {(t1 - t0) / n / 1e3:.1f} us")
    busy = defaultdict(int)
    kt = defaultdict(list)
    for s, e, q, k in win:
        busy[q] += e - s
        kt[k].append(e - s)
    for q in sorted(busy):
        qs = sorted({k for s, e, qq, k in win if qq == q})
        print(f"queue {q}: busy {busy[q] / n / 1e3:6.1f} us/batch  ({', '.join(qs)[:150]})")
    print("kernel                                            calls/batch  mean_us  us/batch")
    for k, v in sorted(kt.items(), key=lambda kv: -sum(kv[1])):
        print(f"{k:50s} {len(v) / n:6.2f} {statistics.mean(v) / 1e3:8.1f} {sum(v) / n / 1e3:8.1f}")
    # stage spans: follow each queue's kernels between markers
    byq = defaultdict(list)
    for r in win:
        byq[r[2]].append(r)
    spans = defaultdict(list)
    for q, rs in byq.items():
        cur = None
        for s, e, _, k in rs:
            if k == "k_sample":
                cur = ("A", s, e, 0)
            elif k.startswith("k_check_tier<false"):
                cur = ("B", s, e, 0)
            elif cur is not None:
                cur = (cur[0], cur[1], e, cur[3])
            if cur is not None and ((cur[0] == "A" and k == "k_edge_fill") or (cur[0] == "B" and k.startswith("k_epilogue"))):
                spans[cur[0]].append((cur[1], cur[2]))
                cur = None
    for st, v in sorted(spans.items()):
        d = [(e - s) / 1e3 for s, e in v]
        print(f"stage {st}: span median {statistics.median(d):.1f} us over {len(d)} batches")
    # gaps inside each queue's chain: idle between consecutive kernels on one queue
    for q, rs in sorted(byq.items()):
        g = [rs[i + 1][0] - rs[i][1] for i in range(len(rs) - 1)]
        g = [x for x in g if x > 0]
        if g:
            print(f"queue {q}: gaps/batch {len(g) / n:.1f}, median {statistics.median(g) / 1e3:.1f} us, "
                  f"sum/batch {sum(g) / n / 1e3:.1f} us")


if __name__ == "__main__":
    main()
