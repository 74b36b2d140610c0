#!/bin/bash
# Delta bound floor (FDBCS_DELTA_FLOOR, default 1.25M): GPU suite, then same-box A/B of floors
# 0 (N/16) / 1.25M / 2.5M at C2 and C3 over 400-batch windows.
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/${TAG:-r05df}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 280 --timeout-method thread -p no:cacheprovider tests -m gpu > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for w in c2 c3; do
  BENCH_ARGS="--workload $w --steps 400 --warmup 20 --no-cpu-baseline --breakdown-steps 0 --sync-steps 0 --h2d-steps 0 --total-steps 0" \
  VARIANTS="f0:FDBCS_DELTA_FLOOR=0 f125:FDBCS_DELTA_FLOOR=1250000 f250:FDBCS_DELTA_FLOOR=2500000" ROUNDS=1 timeout -k 10 900 bash scripts/gpu_ab_env.sh 2>&1 | sed "s/^/$w /" || exit 1
done
