#!/bin/bash
# Round-4: resolution tests, C3 trace, C4 run-probe variant, C3 A/B of the resolver change.
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/r04c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider -k "c3 or chain or 32768 or pipeline_variants or keyspace or report or sort_bucket" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/trace_c2.py 8 5000 c3 > $O/trace_c3.txt 2>&1 || exit $?
grep resolve $O/trace_c3.txt | tail -3
WORKLOAD=c4 WHICH=0,3,4 timeout -k 10 300 python scripts/kernel_sweep.py "X=1" "FDBCS_LIB=$PWD/foundationdb_amd/variants/libfdbcs_p7.so" > $O/sweep.txt 2>&1 || exit $?
cat $O/sweep.txt
WORKLOAD=c3 ROUNDS=2 LIBS="head:head cur:cur" STEPS=40 bash scripts/gpu_ab_lib.sh > $O/ab_c3.txt 2>&1 || exit $?
tail -25 $O/ab_c3.txt
ROUNDS=2 BENCH_ARGS="--workload c4 --steps 60 --no-cpu-baseline --sync-steps 0 --resident-steps 0 --total-steps 0" \
  VARIANTS="n16:FDBCS_DELTA_SQRT=0 sqrt:FDBCS_DELTA_SQRT=1" bash scripts/gpu_ab_env.sh || exit $?
for f in gpurun_out/ab/n16_1.json gpurun_out/ab/sqrt_1.json; do python3 -c "
import json,sys; d=json.loads(open('$f').read().splitlines()[-1]); print('$f', d['amortized_ms_per_batch'], d['phase_ms_per_batch'].get('ms_merge'), d['phase_ms_per_batch'].get('ms_epilogue'))"; done
