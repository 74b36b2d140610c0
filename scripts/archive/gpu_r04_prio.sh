#!/bin/bash
# Stream priority A/B (FDBCS_PRIO) on C2 and C4.
set -u
cd "$(dirname "$0")/.." || exit 1
for W in c2 c4; do
ROUNDS=2 BENCH_ARGS="--workload $W --steps 300 --warmup 60 --no-cpu-baseline --breakdown-steps 0 --sync-steps 0 --resident-steps 0 --total-steps 0" \
  VARIANTS="none: a:FDBCS_PRIO=a x:FDBCS_PRIO=x ac:FDBCS_PRIO=ac xy:FDBCS_PRIO=xy" bash scripts/gpu_ab_env.sh 2>&1 | sed "s/^/$W /" | tee -a gpurun_out/ab_prio.txt || exit 1
done
