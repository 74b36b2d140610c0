#!/bin/bash
set -u
cd "$(dirname "$0")/.." || exit 1
BENCH_ARGS="--workload c2 --steps 60 --no-cpu-baseline --breakdown-steps 0 --sync-steps 0 --h2d-steps 0 --total-steps 0" \
VARIANTS="none:FDBCS_X=0 force:FDBCS_EXP_FORCE_SKIP=1" ROUNDS=3 timeout -k 10 900 bash scripts/gpu_ab_env.sh || exit 1
