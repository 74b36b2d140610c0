#!/bin/bash
# rocprofv3 kernel-trace stats of a short bench run; summaries land in gpurun_out/prof/.
set -u
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
  python3 bench.py --steps ${STEPS:-48} --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/prof/bench.json 2> gpurun_out/prof/bench.err
rc=$?
echo "rocprof rc=$rc" >&2
find gpurun_out/prof -name "*stats*" >&2
exit $rc
