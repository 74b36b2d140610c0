#!/bin/bash
# Round-5 evidence at the current build, part 1: GPU tests (junit), smoke, rocprofv3 kernel-trace
# profiles C1-C4 and C2 at 32768-txn batches, PMC traffic passes C2 and C4.  Copy the rocprof_*.json
# and pmc_*.json into profiles/ before part 2 (the bench lines).
set -u
cd "$(dirname "$0")/.." || exit 1
TAG=${TAG:-r05f}
O=gpurun_out/$TAG
mkdir -p $O
step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "== $name $(date +%T)" >&2
  timeout -k 10 "$t" "$@"
  local rc=$?
  echo "== $name rc=$rc" >&2
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >&2; exit $rc; fi
}
step tests 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  --junitxml=$O/junit.xml > $O/gpu_tests.log 2>&1
tail -2 $O/gpu_tests.log >&2
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
for w in c1 c2 c3 c4; do
  WORKLOAD=$w OUT=$O/prof_$w step prof_$w 600 bash scripts/gpu_profile.sh
  head -3 $O/prof_$w/summary.txt >&2
done
WORKLOAD=c2 OUT=$O/prof_c2_32768 STEPS=24 BENCH_ARGS="--txns 32768" step prof_c2_32768 600 bash scripts/gpu_profile.sh
WORKLOAD=c2 step pmc_c2 500 bash scripts/gpu_pmc.sh
WORKLOAD=c4 step pmc_c4 500 bash scripts/gpu_pmc.sh
echo done >&2
