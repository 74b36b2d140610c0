"""A rocprofv3 kernel-trace stats CSV as the per-kernel summary bench.py ranks kernels by:
profiles/rocprof_<workload>_<txns>_<history>.json with the engine build id (roofline.build_id) and
the git head of the tree it was measured on.  Kernel names as the engine reports them.
Usage: rocprof_rank.py <kernel_stats.csv> <workload> <txns> <history> [git_head] > out.json"""
import csv
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))
import roofline  # noqa: E402
from pmc_summary_names import engine_name  # noqa: E402

rows = list(csv.DictReader(open(sys.argv[1])))
kern = {}
for r in rows:
    k = engine_name(r["Name"])
    if k.startswith("k_hold") or k.startswith("__amd"):
        continue
    kern[k] = {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3,
               "total_ms": float(r["TotalDurationNs"]) / 1e6}
out = {"source": "rocprofv3 --kernel-trace --stats (dispatch to completion per kernel)",
       "config": {"workload": sys.argv[2], "txns": int(sys.argv[3]), "history": int(sys.argv[4])},
       "build_id": roofline.build_id(os.path.dirname(HERE)),
       "git_head": sys.argv[5] if len(sys.argv) > 5 else None,
       "kernels": dict(sorted(kern.items(), key=lambda kv: -kv[1]["total_ms"]))}
print(json.dumps(out, indent=1))
