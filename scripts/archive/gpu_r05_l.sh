#!/bin/bash
# Replicated level-3 entries: isolated whole-base rebuild, the GPU suite, C2 / C4 bench lines.
set -u
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05l}
mkdir -p $O
HISTORY=5000000 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/epi -o run -- python3 scripts/epi_bench.py > $O/epi.log 2>&1 || { tail $O/epi.log; exit 1; }
S=$(find $O/epi -name "*kernel_stats.csv" | head -1)
python3 scripts/prof_summary.py $S | grep epilogue >&2
find $O/epi -name "*kernel_trace.csv" -delete
timeout -k 10 900 python -u -m pytest -x -v --timeout 280 --timeout-method thread -p no:cacheprovider tests -m gpu > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log >&2
for w in ${WORKLOADS:-c2 c4}; do
  timeout -k 10 600 python bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || exit 1
done
