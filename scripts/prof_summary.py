"""Print a rocprofv3 kernel_stats.csv as a per-kernel table (sorted by total time)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    name = r["Name"].split("(")[0][:72]
    print(f"{name:72s} calls={int(r['Calls']):5d} avg_us={float(r['AverageNs'])/1e3:8.2f} "
          f"total_ms={float(r['TotalDurationNs'])/1e6:8.3f} pct={100*float(r['TotalDurationNs'])/tot:5.1f}")
