#!/bin/bash
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/r04h
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "long or c4 or sort or pipeline_variants or keyspace or random or radix or kat or frozen" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
WORKLOAD=c4 WHICH=1,2 timeout -k 10 200 python scripts/kernel_sweep.py "FDBCS_LIB=$PWD/foundationdb_amd/variants/libfdbcs_head.so" "X=1" || exit 1
WORKLOAD=c4 ROUNDS=2 LIBS="head:head cur:cur" STEPS=40 bash scripts/gpu_ab_lib.sh > $O/ab_c4.txt 2>&1 || exit $?
head -14 $O/ab_c4.txt
