#!/bin/bash
# Bench plus a rocprofv3 kernel + memory-copy trace of the same command (diagnosis of the timed loop).
set -u
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/diag
timeout -k 10 300 python3 bench.py ${BENCH_ARGS:---steps 30 --warmup 3} > gpurun_out/diag/bench.json 2> gpurun_out/diag/bench.err || exit $?
cat gpurun_out/diag/bench.json >&2
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/diag/prof -o run -- \
  python3 bench.py --steps 30 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/diag/prof_bench.json 2> gpurun_out/diag/prof_bench.err
