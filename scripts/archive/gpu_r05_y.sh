#!/bin/bash
# Wider k_seg_prep tiles (255 segments, one lane per lookup, short keys): GPU suite, rocprof C2 /
# C2 at 32768 / C3, bench lines C2 and C2 at 32768; then the RCCL leg at world 1.
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/${TAG:-r05y}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 280 --timeout-method thread -p no:cacheprovider tests -m gpu > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for w in c2 c3; do
  WORKLOAD=$w OUT=$O/prof_$w timeout -k 10 600 bash scripts/gpu_profile.sh || exit 1
  grep -E "seg_prep|merge_copy<fdbcs::Batch" $O/prof_$w/summary.txt
done
WORKLOAD=c2 OUT=$O/prof_c2_32768 STEPS=24 BENCH_ARGS="--txns 32768" timeout -k 10 600 bash scripts/gpu_profile.sh || exit 1
head -6 $O/prof_c2_32768/summary.txt
for a in "--workload c2" "--workload c2 --txns 32768"; do
  timeout -k 10 600 python bench.py $a --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 1
  python3 -c "import json;d=json.load(open('$O/bench.json'));print('$a',d['value'],d['h2d_inclusive_txns_per_s'],d['device_bound']['ms_per_batch'],d['parity']['mismatched_batches'])"
done
TAG=r05f bash scripts/gpu_r05_rccl.sh
