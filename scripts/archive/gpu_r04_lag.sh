#!/bin/bash
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/r04lag
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
  -p no:cacheprovider -k "async or pipeline_variants or timing_level or c4_window" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for W in c2 c3 c4; do
ROUNDS=2 BENCH_ARGS="--workload $W --steps 300 --warmup 60 --no-cpu-baseline --breakdown-steps 0 --sync-steps 0 --resident-steps 0 --total-steps 0" \
  VARIANTS="base: lag:FDBCS_LAG=1 thr:FDBCS_SUBMIT_THREAD=1" bash scripts/gpu_ab_env.sh 2>&1 | sed "s/^/$W /" | tee -a $O/ab.txt || exit 1
done
