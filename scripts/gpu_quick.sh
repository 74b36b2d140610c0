#!/bin/bash
# Parity tests, then a short bench per workload given in $WORKLOADS (default: c2 c3).
# Stops at the first failing GPU step.
set -u
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -15 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
for wl in ${WORKLOADS:-c2 c3}; do
  timeout -k 10 300 python bench.py --workload $wl --steps ${STEPS:-30} --warmup 3 ${BENCH_ARGS:-} \
    > gpurun_out/bench_$wl.json 2> gpurun_out/bench_$wl.err || { tail -20 gpurun_out/bench_$wl.err; exit 1; }
  cat gpurun_out/bench_$wl.json
done
