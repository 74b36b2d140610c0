#!/bin/bash
# C4 kernel-trace profiles at 4 and 8 hardware queues: which kernels stretch when every stream has
# a queue of its own.
set -u
cd "$(dirname "$0")/.." || exit 1
for q in 4 8; do
  GPU_MAX_HW_QUEUES=$q WORKLOAD=c4 OUT=gpurun_out/hwq/c4_q$q STEPS=24 timeout -k 10 700 bash scripts/gpu_profile.sh || exit 1
  head -14 gpurun_out/hwq/c4_q$q/summary.txt
done
