#!/usr/bin/env python3
"""Host issue vs device start of every kernel of a rocprofv3 --hip-runtime-trace --kernel-trace
run: per kernel name, the median time from the launch call's return to the kernel's start
(queueing behind its stream and the chip) and the share of launches that started within 5 us of
the call (the device waited for the host).  Usage: launch_gaps.py api_trace.csv kernel_trace.csv"""
import csv
import statistics
import sys
from collections import defaultdict

api = {}
for r in csv.DictReader(open(sys.argv[1])):
    if "Launch" in r["Function"]:
        api[r["Correlation_Id"]] = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Thread_Id"])
rows = defaultdict(list)
for r in csv.DictReader(open(sys.argv[2])):
    a = api.get(r["Correlation_Id"])
    if not a:
        continue
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("fdbcs::", "")
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    rows[name].append(((s - a[1]) / 1e3, (e - s) / 1e3, (a[1] - a[0]) / 1e3, a[2]))
print(f"{'kernel':42s} {'n':>5s} {'issue->start':>12s} {'p10':>7s} {'p90':>7s} {'<5us':>6s} {'dur':>7s} {'call':>6s} threads")
for k, v in sorted(rows.items(), key=lambda kv: -len(kv[1])):
    g = sorted(x[0] for x in v)
    q = lambda f: g[min(len(g) - 1, int(f * len(g)))]  # noqa: E731
    fast = sum(1 for x in g if x < 5) / len(g)
    th = sorted(set(x[3] for x in v))
    print(f"{k[:42]:42s} {len(v):5d} {statistics.median(g):12.1f} {q(0.1):7.1f} {q(0.9):7.1f} {fast:6.2f} "
          f"{statistics.median(x[1] for x in v):7.1f} {statistics.median(x[2] for x in v):6.1f} {len(th)}")
