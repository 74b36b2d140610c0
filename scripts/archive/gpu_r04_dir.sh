#!/bin/bash
# Base-tier directory keyed past the shared key prefix (MaxLevels::dir_p): its parity test, the GPU
# suite, C4's isolated check times and same-box C4 / C2 bench A/B (FDBCS_DIR_PREFIX=0: first two bytes).
set -u
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/dir
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  -k directory_past > gpurun_out/dir/t1.log 2>&1 || { tail -30 gpurun_out/dir/t1.log; exit 1; }
tail -1 gpurun_out/dir/t1.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/dir/tests.log 2>&1 || { tail -30 gpurun_out/dir/tests.log; exit 1; }
tail -1 gpurun_out/dir/tests.log
WORKLOAD=c4 WHICH=0,3,4 timeout -k 10 600 python3 scripts/kernel_sweep.py "FDBCS_DIR_PREFIX=1" "FDBCS_DIR_PREFIX=0" || exit 1
for W in c4 c2; do
ROUNDS=2 BENCH_ARGS="--workload $W --steps 200 --warmup 40 --no-cpu-baseline --breakdown-steps 0 --sync-steps 0 --total-steps 0" \
  VARIANTS="dp1:FDBCS_DIR_PREFIX=1 dp0:FDBCS_DIR_PREFIX=0" bash scripts/gpu_ab_env.sh 2>&1 | sed "s/^/$W /" || exit 1
done
