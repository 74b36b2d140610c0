#!/bin/bash
# k_seg_prep layout at C2 5000-txn batches: rocprof seg_prep time and bench line.
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/${TAG:-r05ab}
mkdir -p $O
WORKLOAD=c2 OUT=$O/prof_c2 timeout -k 10 600 bash scripts/gpu_profile.sh || exit 1
grep -E "seg_prep" $O/prof_c2/summary.txt
timeout -k 10 600 python bench.py --workload c2 --cpu-seconds 5 > $O/bench.json 2> $O/bench.err || exit 1
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['h2d_inclusive_txns_per_s'],d['device_bound']['ms_per_batch'],d['parity']['mismatched_batches'],d['parity']['batches_checked'])"
