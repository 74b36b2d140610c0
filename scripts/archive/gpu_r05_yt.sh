#!/bin/bash
# Third submitting thread for the Y half (FDBCS_Y_THREAD=1): the async pipeline tests, then same-box
# A/Bs of the C2 and C4 lines.
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/${TAG:-r05yt}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 280 --timeout-method thread -p no:cacheprovider tests/test_gpu_fullsize.py -m gpu -k "async_pipeline or flag_before" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for w in c2 c4; do
  BENCH_ARGS="--workload $w --steps 60 --no-cpu-baseline --breakdown-steps 0 --sync-steps 0 --h2d-steps 0 --total-steps 0" \
  VARIANTS="two:FDBCS_Y_THREAD=0 three:FDBCS_Y_THREAD=1" ROUNDS=3 timeout -k 10 900 bash scripts/gpu_ab_env.sh 2>&1 | sed "s/^/$w /" || exit 1
done
