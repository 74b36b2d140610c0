#!/bin/bash
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/r04i
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
H=$PWD/foundationdb_amd/variants/libfdbcs_head.so
ROUNDS=2 BENCH_ARGS="--steps 400 --warmup 100 --no-cpu-baseline --breakdown-steps 0 --sync-steps 0 --resident-steps 0 --total-steps 0" \
  VARIANTS="head:FDBCS_LIB=$H cur: headthr:FDBCS_LIB=$H,FDBCS_SUBMIT_THREAD=1 curthr:FDBCS_SUBMIT_THREAD=1" bash scripts/gpu_ab_env.sh 2>&1 | tee $O/ab_c2.txt
