"""Per-launch HBM bytes of every pipeline kernel from rocprofv3 --pmc CSVs (FETCH_SIZE and
WRITE_SIZE, each from its own pass; MI355X_MICROARCH.md: PMC slots, gfx950 corrections).

FETCH_SIZE / WRITE_SIZE are in KiB.  On gfx950 FETCH_SIZE reads exactly half the bytes of a wide
(16 B/lane) coalesced streaming read, so `bytes_per_launch` uses 2 x FETCH_SIZE + WRITE_SIZE and
`bytes_per_launch_raw` the counters as read.  Kernel names are the engine's (fdbcs_kernel_profile:
no `void`, no leading namespace, no parameter list), the key roofline.pmc_traffic reads.
Usage: pmc_summary.py <dir with FETCH_SIZE/ and WRITE_SIZE/> [workload txns history]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def engine_name(n: str) -> str:
    n = n.strip()
    if n.startswith("void "):
        n = n[5:]
    depth = 0
    for i, ch in enumerate(n):  # cut the parameter list: the first '(' outside template brackets
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            n = n[:i]
            break
    return n[len("fdbcs::"):] if n.startswith("fdbcs::") else n


root = sys.argv[1]
per = {c: defaultdict(list) for c in ("FETCH_SIZE", "WRITE_SIZE")}
for c in per:
    for f in glob.glob(os.path.join(root, c, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") == c:
                per[c][engine_name(r.get("Kernel_Name", ""))].append(float(r["Counter_Value"]))
out = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes; bytes = (2 x FETCH + WRITE) x 1024",
       "bytes_per_launch": {}, "bytes_per_launch_raw": {}, "launches": {}}
if len(sys.argv) >= 5:
    out["config"] = {"workload": sys.argv[2], "txns": int(sys.argv[3]), "history": int(sys.argv[4])}
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import roofline  # noqa: E402

out["build_id"] = roofline.build_id(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
out["git_head"] = os.environ.get("GIT_HEAD")
for k in sorted(set(per["FETCH_SIZE"]) & set(per["WRITE_SIZE"])):
    f = sum(per["FETCH_SIZE"][k]) / len(per["FETCH_SIZE"][k])
    w = sum(per["WRITE_SIZE"][k]) / len(per["WRITE_SIZE"][k])
    out["bytes_per_launch"][k] = (2 * f + w) * 1024
    out["bytes_per_launch_raw"][k] = (f + w) * 1024
    out["launches"][k] = len(per["FETCH_SIZE"][k])
# The model of the same run (the FETCH_SIZE pass's bench line prices every kernel at that run's own
# shape: its delta sizes and its share of compacting batches, which set what an average launch of
# the merge copy or the epilogue moves), beside the measured bytes.
try:
    line = [l for l in open(os.path.join(root, "FETCH_SIZE.json")).read().splitlines() if l.startswith("{")][-1]
    kern = json.loads(line).get("kernels", {})
    out["model_bytes_per_launch"] = {}
    out["ratio_to_model"] = {}
    for k, v in out["bytes_per_launch"].items():
        m = (kern.get(k) or {}).get("algorithmic_bytes_per_launch")
        if m:
            out["model_bytes_per_launch"][k] = m
            out["ratio_to_model"][k] = round(v / m, 3)
except (OSError, IndexError, ValueError):
    pass
print(json.dumps(out, indent=1))
