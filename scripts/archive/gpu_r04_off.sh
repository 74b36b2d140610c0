#!/bin/bash
# Bucket bases computed once by k_sort_partition's last workgroup (working tree) against every
# k_sort_bucket workgroup reducing all counters (HEAD, libfdbcs_base.so): the GPU suite, isolated
# sort times at C2/C3, pipelined kernel tables and lines at C2, C3 and C4.
set -u
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/off
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/off/tests.log 2>&1 || { tail -30 gpurun_out/off/tests.log; exit 1; }
tail -1 gpurun_out/off/tests.log
for W in c2 c3; do
  for L in base cur; do
    lib=foundationdb_amd/variants/libfdbcs_$L.so; [ $L = cur ] && lib=foundationdb_amd/libfdbcs.so
    FDBCS_LIB=$PWD/$lib WORKLOAD=$W WHICH=1,2 timeout -k 10 300 python3 scripts/kernel_sweep.py "$L" || exit 1
  done
done
for W in c2 c3 c4; do
  WORKLOAD=$W ROUNDS=2 LIBS="base:base off:cur" timeout -k 10 900 bash scripts/gpu_ab_lib.sh 2>&1 | grep -E "value|sort_bucket|sort_partition|check_lanes" || exit 1
done
