#!/bin/bash
# Delta floor 0 vs 1.25M with the bench's default window (50 timed batches) and with 400, same box.
set -u
cd "$(dirname "$0")/.." || exit 1
for steps in 50 400; do
  BENCH_ARGS="--workload c2 --steps $steps --no-cpu-baseline --breakdown-steps 0 --sync-steps 0 --h2d-steps 0 --total-steps 0" \
  VARIANTS="f0:FDBCS_DELTA_FLOOR=0 f125:FDBCS_DELTA_FLOOR=1250000" ROUNDS=3 timeout -k 10 900 bash scripts/gpu_ab_env.sh 2>&1 | sed "s/^/steps$steps /" || exit 1
done
