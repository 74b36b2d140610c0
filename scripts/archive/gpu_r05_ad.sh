#!/bin/bash
# CU partitions between the chains (FDBCS_CU_MASK), same-box A/B on C2 (and C4 for the best).
set -u
cd "$(dirname "$0")/.." || exit 1
BENCH_ARGS="--workload c2 --steps 60 --no-cpu-baseline --breakdown-steps 0 --sync-steps 0 --h2d-steps 0 --total-steps 0" \
VARIANTS="none:FDBCS_X=0 halfA:FDBCS_CU_MASK=a:0-127,x:128-255,y:128-255 xcdA:FDBCS_CU_MASK=a:%0-3,x:%4-7,y:%4-7 xcd3:FDBCS_CU_MASK=a:%0-2,x:%3-5,y:%6-7 xyA:FDBCS_CU_MASK=a:%0-3,y:%0-3 xOwn:FDBCS_CU_MASK=x:%0-3" \
  ROUNDS=2 timeout -k 10 1000 bash scripts/gpu_ab_env.sh || exit 1
