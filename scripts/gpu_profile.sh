#!/bin/bash
# rocprofv3 kernel-trace stats of a short bench run of WORKLOAD; summaries land in $OUT (default
# gpurun_out/prof_<workload>): summary.txt, the per-batch timeline (timeline.txt) and
# rocprof_<workload>_<txns>_<history>.json (copy to profiles/: bench.py ranks the dominant kernel by
# it when the build id matches).  GIT_HEAD: recorded in the summary (the box has no .git).
set -u
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
W=${WORKLOAD:-c2}
case $W in c1) TX=2500; HI=0 ;; c4) TX=5000; HI=50000000 ;; *) TX=5000; HI=5000000 ;; esac
# a --txns in BENCH_ARGS names the profile (rocprof_c2_32768_5000000.json for the 32768-txn batches)
T2=$(echo " ${BENCH_ARGS:-} " | sed -n 's/.* --txns \([0-9]*\) .*/\1/p'); [ -n "$T2" ] && TX=$T2
OUT=${OUT:-gpurun_out/prof_$W}
mkdir -p "$OUT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
  python3 bench.py --workload $W --steps ${STEPS:-48} --warmup 3 --no-cpu-baseline --breakdown-steps 0 ${BENCH_ARGS:-} \
  > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?
echo "rocprof $W rc=$rc" >&2
[ $rc -ne 0 ] && exit $rc
CSV=$(find "$OUT" -name "*kernel_stats.csv" | head -1)
python3 scripts/prof_summary.py "$CSV" > "$OUT/summary.txt"
python3 scripts/rocprof_rank.py "$CSV" $W $TX $HI ${GIT_HEAD:-} > "$OUT/rocprof_${W}_${TX}_${HI}.json"
python3 scripts/timeline.py $(find "$OUT" -name "*kernel_trace.csv" | head -1) > "$OUT/timeline.txt" 2>&1 || true
find "$OUT" -name "*kernel_trace.csv" -delete
exit 0
