#!/bin/bash
# k_sort_bucket at 1, 2 and 4 waves per workgroup (variant builds): isolated at C2/C3, pipelined at C2.
set -u
cd "$(dirname "$0")/.." || exit 1
for W in c2 c3; do
  for L in b64 b128 b256; do
    FDBCS_LIB=$PWD/foundationdb_amd/variants/libfdbcs_$L.so WORKLOAD=$W WHICH=1,2 timeout -k 10 300 python3 scripts/kernel_sweep.py "$L" || exit 1
  done
done
WORKLOAD=c2 ROUNDS=2 LIBS="b64:b64 b128:b128 b256:b256" timeout -k 10 900 bash scripts/gpu_ab_lib.sh 2>&1 | grep -E "value|sort_bucket|sort_partition|check_lanes|seg_prep" || exit 1
