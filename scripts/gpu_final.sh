#!/bin/bash
# Round evidence at the current build, in one GPU call: the GPU tests, smoke, then per workload a
# rocprofv3 kernel-trace profile (rocprof_<w>_<txns>_<history>.json: the ranking bench.py names the
# dominant kernel by), PMC traffic passes for C2 and C4, and the 32768-transaction C2 profile.
# Copy prof_*/rocprof_*.json and pmc/pmc_*.json into profiles/ afterwards, then run the benches.
set -u
cd "$(dirname "$0")/.." || exit 1
TAG=${TAG:-r04e}
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
step tests 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -o log_cli=false \
  --junitxml=$O/junit.xml > $O/gpu_tests.log 2>&1
tail -3 $O/gpu_tests.log >&2
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
for w in c1 c2 c3 c4; do
  WORKLOAD=$w OUT=$O/prof_$w step prof_$w 700 bash scripts/gpu_profile.sh
  head -4 $O/prof_$w/summary.txt >&2
done
WORKLOAD=c2 step pmc_c2 700 bash scripts/gpu_pmc.sh
WORKLOAD=c4 step pmc_c4 700 bash scripts/gpu_pmc.sh
WORKLOAD=c2 OUT=$O/prof_c2_32768 STEPS=24 BENCH_ARGS="--txns 32768" step prof_c2_32768 700 bash scripts/gpu_profile.sh
head -6 $O/prof_c2_32768/summary.txt >&2
