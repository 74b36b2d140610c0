#!/bin/bash
# Hardware queues per process (GPU_MAX_HW_QUEUES, HIP's default 4 on the box) against the engine's
# five streams plus torch's: A/B on C2 and C4, same box, interleaved.
set -u
cd "$(dirname "$0")/.." || exit 1
for W in c2 c4; do
ROUNDS=2 BENCH_ARGS="--workload $W --steps 300 --warmup 60 --no-cpu-baseline --breakdown-steps 0 --sync-steps 0 --resident-steps 0 --total-steps 0" \
  VARIANTS="q4:GPU_MAX_HW_QUEUES=4 q8:GPU_MAX_HW_QUEUES=8 q6:GPU_MAX_HW_QUEUES=6" bash scripts/gpu_ab_env.sh 2>&1 | sed "s/^/$W /" | tee -a gpurun_out/ab_hwq.txt || exit 1
done
