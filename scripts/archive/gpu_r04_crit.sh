#!/bin/bash
# Kernel trace of the pipelined C2 loop only (no side passes), and where its batches wait.
set -u
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
W=${WORKLOAD:-c2}
O=gpurun_out/crit_$W${SUFFIX:-}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace ${COPYTRACE:+--memory-copy-trace} --output-format csv -d $O -o run -- \
  python3 bench.py --workload $W --steps 300 --warmup 20 --no-cpu-baseline --breakdown-steps 0 --sync-steps 0 \
  --resident-steps 0 --total-steps 0 --profile-steps 0 --hold-steps 0 ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err || exit 1
T=$(find $O -name "*kernel_trace.csv" | head -1)
C=$(find $O -name "*memory_copy_trace.csv" | head -1)
head -3 "$C" 2>/dev/null
python3 scripts/crit_path.py $T ${C:+--copies $C} > $O/crit.txt 2>&1; cat $O/crit.txt
[ -n "$C" ] && gzip -f $C
gzip -f $T
