#!/bin/bash
# rocprofv3 kernel-trace stats of a short bench run; summaries land in gpurun_out/prof/, plus the
# rocprof-dominant roofline kernel (dominant.json, copy to profiles/dominant_<workload>.json).
set -u
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
  python3 bench.py --steps ${STEPS:-48} --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/prof/bench.json 2> gpurun_out/prof/bench.err
rc=$?
echo "rocprof rc=$rc" >&2
find gpurun_out/prof -name "*stats*" >&2
[ $rc -eq 0 ] && python3 scripts/prof_summary.py $(find gpurun_out/prof -name "*kernel_stats.csv" | head -1) \
  --dominant gpurun_out/prof/dominant.json > gpurun_out/prof/summary.txt
exit $rc
