#!/bin/bash
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/r04f
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for W in c3 c2; do
WORKLOAD=$W ROUNDS=2 LIBS="head:head cur:cur" STEPS=40 bash scripts/gpu_ab_lib.sh > $O/ab_$W.txt 2>&1 || exit $?
head -16 $O/ab_$W.txt
done
