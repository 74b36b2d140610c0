#!/bin/bash
# Second evidence call at the final build: the bench lines (gpu_benches.sh), then C4's isolated
# check with and without the shared-prefix directory and a same-box C4 A/B.
set -u
cd "$(dirname "$0")/.." || exit 1
TAG=${TAG:-r04f} timeout -k 10 900 bash scripts/gpu_benches.sh || exit 1
WORKLOAD=c4 WHICH=0,3,4 timeout -k 10 400 python3 scripts/kernel_sweep.py "FDBCS_DIR_PREFIX=1" "FDBCS_DIR_PREFIX=0" || exit 1
ROUNDS=1 BENCH_ARGS="--workload c4 --steps 200 --warmup 40 --no-cpu-baseline --breakdown-steps 0 --sync-steps 0 --total-steps 0" \
  VARIANTS="dp1:FDBCS_DIR_PREFIX=1 dp0:FDBCS_DIR_PREFIX=0" timeout -k 10 400 bash scripts/gpu_ab_env.sh 2>&1 | sed "s/^/c4 /" || exit 1
