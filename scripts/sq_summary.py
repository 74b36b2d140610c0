"""Per-kernel SQ counters (rocprofv3 --pmc, one pass of SQ_ counters) averaged per launch: waves,
wave cycles (quad-cycles), waiting / issue-stalled / active fractions, instructions per wave.
Usage: sq_summary.py <dir with *counter_collection.csv>"""
import csv
import glob
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary_names import engine_name  # noqa: E402

vals = defaultdict(lambda: defaultdict(float))
launches = defaultdict(set)
for f in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = engine_name(r.get("Kernel_Name", ""))
        vals[k][r["Counter_Name"]] += float(r["Counter_Value"])
        launches[k].add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
rows = []
for k, v in vals.items():
    n = max(1, len(launches[k]))
    wc = v.get("SQ_WAVE_CYCLES", 0.0)
    waves = v.get("SQ_WAVES", 0.0)
    rows.append((wc / n, k, n, waves / n, wc / n,
                 v.get("SQ_WAIT_ANY", 0) / wc if wc else 0, v.get("SQ_WAIT_INST_ANY", 0) / wc if wc else 0,
                 v.get("SQ_ACTIVE_INST_ANY", 0) / wc if wc else 0,
                 v.get("SQ_INSTS_VALU", 0) / waves if waves else 0, v.get("SQ_INSTS_SALU", 0) / waves if waves else 0,
                 v.get("SQ_INSTS_VMEM_RD", 0) / waves if waves else 0, v.get("SQ_INSTS_LDS", 0) / waves if waves else 0))
print("kernel launches waves/launch wavecyc/launch(quad) wait inst_stall active valu/wave salu/wave vmem_rd/wave lds/wave")
for r in sorted(rows, reverse=True):
    print(f"{r[1][:60]:60s} {r[2]:5d} {r[3]:8.0f} {r[4]:12.0f} {r[5]:.2f} {r[6]:.2f} {r[7]:.2f} {r[8]:7.0f} {r[9]:6.0f} "
          f"{r[10]:6.1f} {r[11]:6.1f} quadcyc/wave {r[4] / max(1, r[3]):.0f}")
