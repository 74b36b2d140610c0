"""Per-kernel rocprof averages of same-box A/B runs (scripts/gpu_ab_lib.sh), one column per build."""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary_names import engine_name  # noqa: E402

root, w, libs, rounds = sys.argv[1], sys.argv[2], sys.argv[3].split(), int(sys.argv[4])
avg = {}
vals = {}
for n in libs:
    for r in range(1, rounds + 1):
        f = glob.glob(os.path.join(root, f"{n}_{w}_{r}", "**", "*kernel_stats.csv"), recursive=True)
        if not f:
            continue
        for row in csv.DictReader(open(f[0])):
            k = engine_name(row["Name"])
            avg.setdefault(k, {}).setdefault(n, []).append(float(row["AverageNs"]) / 1e3)
        try:
            d = json.loads(open(os.path.join(root, f"{n}_{w}_{r}.json")).read().splitlines()[-1])
            vals.setdefault(n, []).append((d["value"] / 1e6, (d.get("device_bound") or {}).get("ms_per_batch")))
        except Exception:  # noqa: BLE001
            pass
print("value (M txns/s, device-bound ms/batch):", {n: vals.get(n) for n in libs})
keys = sorted(avg, key=lambda k: -max(sum(v) / len(v) for v in avg[k].values()))
print(f"{'kernel':58s}" + "".join(f"{n:>12s}" for n in libs))
for k in keys:
    if k.startswith("k_hold"):
        continue
    row = avg[k]
    print(f"{k[:58]:58s}" + "".join(f"{(sum(row[n]) / len(row[n]) if n in row else float('nan')):12.2f}" for n in libs))
