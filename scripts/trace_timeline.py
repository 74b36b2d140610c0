#!/usr/bin/env python3
"""Print a window of a rocprofv3 kernel trace as a per-queue timeline (us), for pipelining checks."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
start = int(sys.argv[2]) if len(sys.argv) > 2 else len(rows) // 2
count = int(sys.argv[3]) if len(sys.argv) > 3 else 40
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
win = rows[start:start + count]
t0 = int(win[0]["Start_Timestamp"])
for r in win:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].replace("fdbcs::", "").split("(")[0][:40]
    print(f"q{r['Queue_Id']:>2} {(s - t0) / 1000:8.1f} -> {(e - t0) / 1000:8.1f}  dur={(e - s) / 1000:6.1f}  {name}")
