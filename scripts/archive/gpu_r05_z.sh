#!/bin/bash
# k_seg_prep layouts by batch size (cooperative narrow tiles under 24576 writes, wide one-lane tiles
# above): GPU suite, rocprof C2 and C2 at 32768, bench lines C2 / C2 at 32768 / C3.
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/${TAG:-r05z}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 280 --timeout-method thread -p no:cacheprovider tests -m gpu > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
WORKLOAD=c2 OUT=$O/prof_c2 timeout -k 10 600 bash scripts/gpu_profile.sh || exit 1
grep -E "seg_prep" $O/prof_c2/summary.txt
WORKLOAD=c2 OUT=$O/prof_c2_32768 STEPS=24 BENCH_ARGS="--txns 32768" timeout -k 10 600 bash scripts/gpu_profile.sh || exit 1
head -8 $O/prof_c2_32768/summary.txt
for a in "--workload c2" "--workload c2 --txns 32768" "--workload c3"; do
  timeout -k 10 600 python bench.py $a --cpu-seconds 5 > $O/bench.json 2> $O/bench.err || exit 1
  python3 -c "import json;d=json.load(open('$O/bench.json'));print('$a',d['value'],d['h2d_inclusive_txns_per_s'],d['device_bound']['ms_per_batch'],d['parity']['mismatched_batches'],d['parity']['batches_checked'])"
done
