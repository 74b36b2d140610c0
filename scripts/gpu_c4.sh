#!/bin/bash
# C4 (tuple keys, 50M-boundary history): parity tests with long keys, bench line, kernel stats.
set -u
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_c4
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 -p no:cacheprovider ${PYTEST_ARGS:-} > gpurun_out/c4_tests.log 2>&1
rc=$?; tail -3 gpurun_out/c4_tests.log >&2; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --workload c4 --steps ${STEPS:-20} --warmup 3 --breakdown-steps 8 ${BENCH_ARGS:-} > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err
rc=$?; cat gpurun_out/bench_c4.json >&2; [ $rc -ne 0 ] && exit $rc
if [ "${PROFILE:-1}" = "1" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4 -o run -- \
    python3 bench.py --workload c4 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof_c4/bench.json 2> gpurun_out/prof_c4/bench.err
  rc=$?; echo "rocprof rc=$rc" >&2; [ $rc -ne 0 ] && exit $rc
  python3 scripts/prof_summary.py gpurun_out/prof_c4/run_kernel_stats.csv >&2
fi
