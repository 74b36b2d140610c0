#!/bin/bash
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/r04e
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider -k "c3 or chain or 32768 or pipeline_variants or keyspace or report or c2 or c4" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/trace_c2.py 8 5000 c3 > $O/trace_c3.txt 2>&1 || exit $?
grep resolve $O/trace_c3.txt | tail -3
for W in c3 c2; do
WORKLOAD=$W ROUNDS=2 LIBS="head:head cur:cur" STEPS=40 bash scripts/gpu_ab_lib.sh > $O/ab_$W.txt 2>&1 || exit $?
head -16 $O/ab_$W.txt
done
