#!/bin/bash
# Completed cross-stream waits left unqueued at replay (FDBCS_WAIT_SKIP): issue profile, then a
# same-box A/B of the C2 line, then the GPU suite.
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/${TAG:-r05ws}
mkdir -p $O
FDBCS_ISSUE_PROFILE=1 timeout -k 10 300 python bench.py --workload c2 --steps 200 --warmup 10 --no-cpu-baseline --breakdown-steps 0 \
  --sync-steps 0 --h2d-steps 0 --total-steps 0 --profile-steps 0 --hold-steps 0 > $O/bench.json 2> $O/bench.err || exit 1
grep "issue profile" $O/bench.err
BENCH_ARGS="--workload c2 --steps 60 --no-cpu-baseline --breakdown-steps 0 --sync-steps 0 --h2d-steps 0 --total-steps 0" \
VARIANTS="skip:FDBCS_WAIT_SKIP=1 noskip:FDBCS_WAIT_SKIP=0" ROUNDS=3 timeout -k 10 900 bash scripts/gpu_ab_env.sh || exit 1
timeout -k 10 900 python -u -m pytest -x -q --timeout 280 --timeout-method thread -p no:cacheprovider tests -m gpu > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
