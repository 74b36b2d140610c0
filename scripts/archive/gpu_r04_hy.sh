#!/bin/bash
# Y half of stage B issued by the helper thread (FDBCS_HELPER_Y): the GPU tests, then same-box A/B
# on C2, C3 and C4.
set -u
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/hy
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/hy/tests.log 2>&1 || { tail -30 gpurun_out/hy/tests.log; exit 1; }
tail -2 gpurun_out/hy/tests.log
for W in c2 c3 c4; do
ROUNDS=2 BENCH_ARGS="--workload $W --steps 300 --warmup 60 --no-cpu-baseline --breakdown-steps 0 --sync-steps 0 --total-steps 0" \
  VARIANTS="hy1:FDBCS_HELPER_Y=1 hy0:FDBCS_HELPER_Y=0" bash scripts/gpu_ab_env.sh 2>&1 | sed "s/^/$W /" || exit 1
done
