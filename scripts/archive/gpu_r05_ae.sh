#!/bin/bash
# Wave-cooperative delta directory fill in k_epilogue: GPU suite, C4 rocprof + PMC, C4 / C2 bench.
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/${TAG:-r05ae}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 280 --timeout-method thread -p no:cacheprovider tests -m gpu > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
WORKLOAD=c4 OUT=$O/prof_c4 timeout -k 10 600 bash scripts/gpu_profile.sh || exit 1
grep -E "epilogue|merge_copy" $O/prof_c4/summary.txt
WORKLOAD=c4 timeout -k 10 500 bash scripts/gpu_pmc.sh 2>/dev/null || exit 1
python3 -c "
import json;d=json.load(open('gpurun_out/pmc/pmc_c4_5000_50000000.json'))
for k in d['ratio_to_model']:
    if 'epilogue' in k or 'merge' in k: print(k, d['bytes_per_launch'][k], d['model_bytes_per_launch'].get(k), d['ratio_to_model'][k])"
for w in c4 c2; do
  timeout -k 10 600 python bench.py --workload $w --cpu-seconds 5 > $O/bench_$w.json 2> $O/bench_$w.err || exit 1
  python3 -c "import json;d=json.load(open('$O/bench_$w.json'));print('$w',d['value'],d['h2d_inclusive_txns_per_s'],d['device_bound']['ms_per_batch'],d['parity']['mismatched_batches'],d['parity']['batches_checked'])"
done
