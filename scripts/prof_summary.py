"""Print a rocprofv3 kernel_stats.csv as a per-kernel table (sorted by total time).

With --dominant OUT.json, also record which of the kernels bench.py prices against the roofline
(roofline.py: check / sort / merge / compact) has the largest total device time in this profile,
so bench.py reports the roofline of the rocprof-dominant kernel (its own HIP-event timing slightly
inflates kernels on the stage-A stream, which overlap stage B)."""
import csv
import json
import sys

ROOF = {  # bench/roofline.py key -> kernel name fragments (the read check: k_check_reads over
    # both tiers, or the split check's base-tier launch k_check_tier<true, ...>)
    "check": ("k_check_tier<true", "k_check_reads"),
    "sort": ("k_bucket_sort",),
    "merge": ("k_merge_copy<fdbcs::BatchIns",),
    "compact": ("k_merge_copy<fdbcs::CompactIns",),
}

rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    name = r["Name"].split("(")[0][:72]
    print(f"{name:72s} calls={int(r['Calls']):5d} avg_us={float(r['AverageNs'])/1e3:8.2f} "
          f"total_ms={float(r['TotalDurationNs'])/1e6:8.3f} pct={100*float(r['TotalDurationNs'])/tot:5.1f}")
if "--dominant" in sys.argv:
    out = sys.argv[sys.argv.index("--dominant") + 1]
    totals = {}
    for k, frags in ROOF.items():
        for r in rows:
            if any(f in r["Name"] for f in frags):
                totals[k] = totals.get(k, 0.0) + float(r["TotalDurationNs"])
    top = max(totals, key=totals.get) if totals else None
    all_top = max(rows, key=lambda r: float(r["TotalDurationNs"]))["Name"].split("(")[0] if rows else None
    with open(out, "w") as f:
        json.dump({"dominant": top, "total_ns": totals, "top_kernel_overall": all_top,
                   "source": sys.argv[1]}, f, indent=1)
