#!/usr/bin/env python3
"""Device-bound pass anatomy from a rocprofv3 kernel trace: the kernels that ran after the last
k_hold released its queue (batches queued up front, so no host pacing), grouped into the
pipeline's chains (A: sort + edges, X: check + resolution, Y: merge + compaction + epilogue);
per chain its busy time (union of its kernels' intervals) over the pass span.  A chain near 1.0
bounds the device.  Usage: hold_trace.py kernel_trace.csv"""
import csv
import sys

CH = {"A": ["k_sort_partition", "k_sort_bucket", "EdgePairScan", "k_edge_fill", "k_sample", "k_quant_cold"],
      "X": ["k_check_lanes", "k_check_tier", "k_resolve", "k_combine", "k_intra_report", "k_conflict_output"],
      "Y": ["k_seg_prep", "k_merge_copy", "k_epilogue", "k_compact_search", "CompactSumScan", "GcScan", "k_directory",
            "k_lvl3_reset"]}
rows = []
for r in csv.DictReader(open(sys.argv[1])):
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
holds = [x for x in rows if "k_hold" in x[2]]
if not holds:
    sys.exit("no k_hold in the trace")
t0 = max(e for s, e, n in holds)
after = [x for x in rows if x[0] >= t0 - 1000 and "k_hold" not in x[2]]
nxt = [s for s, e, n in rows if "k_hold" in n and s > t0]
if nxt:
    after = [x for x in after if x[0] < min(nxt)]
span = (max(e for s, e, n in after) - min(s for s, e, n in after)) / 1e3
print(f"device-bound pass: {len(after)} kernels over {span:.1f} us")


def union(iv):
    iv = sorted(iv)
    tot, cs, ce = 0, None, None
    for s, e in iv:
        if cs is None or s > ce:
            if cs is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if cs is not None:
        tot += ce - cs
    return tot / 1e3


allk = []
for c, names in CH.items():
    iv = [(s, e) for s, e, n in after if any(k in n for k in names)]
    allk += iv
    kt = sum(e - s for s, e in iv) / 1e3
    print(f"  chain {c}: busy {union(iv):8.1f} us ({union(iv) / span:5.2f} of the span), kernel time {kt:8.1f} us, {len(iv)} kernels")
print(f"  any kernel running: {union(allk) / span:5.2f} of the span")
per = {}
for s, e, n in after:
    k = n.split("(")[0].replace("void ", "").replace("fdbcs::", "")
    a = per.setdefault(k, [0, 0.0])
    a[0] += 1
    a[1] += (e - s) / 1e3
for k, (c, t) in sorted(per.items(), key=lambda kv: -kv[1][1])[:16]:
    print(f"    {k[:50]:50s} x{c:4d} {t / c:8.1f} us avg {t:9.1f} us total")
