#!/bin/bash
# rocprofv3 kernel-trace stats of a short bench run; summaries land in $OUT (default
# gpurun_out/prof): summary.txt, the rocprof-dominant roofline kernel (dominant.json, copy to
# profiles/dominant_<workload>.json) and the per-batch timeline (timeline.txt).
set -u
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/prof}
mkdir -p "$OUT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
  python3 bench.py --steps ${STEPS:-48} --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?
echo "rocprof rc=$rc" >&2
[ $rc -ne 0 ] && exit $rc
python3 scripts/prof_summary.py $(find "$OUT" -name "*kernel_stats.csv" | head -1) \
  --dominant "$OUT/dominant.json" > "$OUT/summary.txt"
python3 scripts/timeline.py $(find "$OUT" -name "*kernel_trace.csv" | head -1) > "$OUT/timeline.txt" 2>&1 || true
exit 0
