#!/bin/bash
# C4 with the 2^17-slot directory code: rocprof kernel table, bench line; C2 bench line.
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/${TAG:-r05w}
mkdir -p $O
WORKLOAD=c4 OUT=$O/prof_c4 timeout -k 10 700 bash scripts/gpu_profile.sh || exit 1
head -16 $O/prof_c4/summary.txt
for w in c4 c2; do
  timeout -k 10 600 python bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || exit 1
  python3 -c "import json;d=json.load(open('$O/bench_$w.json'));print('$w',d['value'],d.get('h2d_inclusive_txns_per_s'),d['device_bound'],d['parity']['mismatched_batches'])"
done
