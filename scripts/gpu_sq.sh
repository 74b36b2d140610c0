#!/bin/bash
# SQ counters per kernel (one rocprofv3 --pmc pass of 8 SQ_ counters) on a short bench run.
# Output: gpurun_out/sq_<workload>/summary.txt
set -u
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
W=${WORKLOAD:-c2}
O=gpurun_out/sq_$W
mkdir -p $O
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD --output-format csv -d $O/raw -o run -- \
  python3 bench.py --workload $W --steps ${STEPS:-16} --warmup 2 --no-cpu-baseline --total-steps 0 \
  --breakdown-steps 0 --sync-steps 0 --hold-steps 0 --resident-steps 0 --profile-steps 0 ${BENCH_ARGS:-} \
  > $O/bench.json 2> $O/bench.err
rc=$?
echo "sq $W rc=$rc" >&2
[ $rc -ne 0 ] && exit $rc
python3 scripts/sq_summary.py $O/raw > $O/summary.txt
rm -rf $O/raw
head -12 $O/summary.txt >&2
