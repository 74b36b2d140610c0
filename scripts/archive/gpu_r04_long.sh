#!/bin/bash
# Round-4 long-key lanes: parity tests of the long-key paths, isolated C4 check A/B, C4 bench A/B,
# and the C3 device trace of the resolution.  Output gpurun_out/long/.
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/long
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider -k "long or c4 or pipeline_variants or random_vs_oracle or radix" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
WORKLOAD=c4 WHICH=0,3,4 timeout -k 10 300 python scripts/kernel_sweep.py "FDBCS_LONG_LANES=0" "FDBCS_LONG_LANES=1" > $O/sweep.txt 2>&1 || exit $?
cat $O/sweep.txt
ROUNDS=1 BENCH_ARGS="--workload c4 --steps 40 --no-cpu-baseline --breakdown-steps 0 --sync-steps 0 --resident-steps 0 --total-steps 0" \
  VARIANTS="coop:FDBCS_LONG_LANES=0 lanes:FDBCS_LONG_LANES=1" bash scripts/gpu_ab_env.sh || exit $?
timeout -k 10 300 python scripts/trace_c2.py 8 5000 c3 > $O/trace_c3.txt 2>&1 || exit $?
tail -12 $O/trace_c3.txt
