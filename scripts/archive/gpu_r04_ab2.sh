#!/bin/bash
# Lane exchanges by DPP / permlane swaps in the bucket sort's network: device check of every J,
# the parity tests that sort, then isolated and pipelined A/B against HEAD's build.
set -u
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/ab2
timeout -k 10 60 tools/bin/xorbench || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 150 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/ab2/tests.log 2>&1 || { tail -30 gpurun_out/ab2/tests.log; exit 1; }
tail -2 gpurun_out/ab2/tests.log
for W in c2 c3; do
  for L in base cur; do
    lib=foundationdb_amd/variants/libfdbcs_$L.so; [ $L = cur ] && lib=foundationdb_amd/libfdbcs.so
    FDBCS_LIB=$PWD/$lib WORKLOAD=$W WHICH=0,1,2 timeout -k 10 300 python3 scripts/kernel_sweep.py "$L" || exit 1
  done
done
WORKLOAD=c2 ROUNDS=2 LIBS="base:base dpp:cur" timeout -k 10 900 bash scripts/gpu_ab_lib.sh || exit 1
