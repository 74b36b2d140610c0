#!/bin/bash
# Round 6 evidence, part A (final build): the GPU suite, smoke, rocprofv3 kernel-trace profiles of
# C1-C4 and C2 at 32768-txn batches (rocprof_<w>_<txns>_<history>.json: bench.py ranks the dominant
# kernel by them; copy into profiles/ before part B).
set -u
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06final}
mkdir -p $O
step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "== $name $(date +%T)" >&2
  timeout -k 10 "$t" "$@"
  local rc=$?
  echo "== $name rc=$rc" >&2
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >&2; exit $rc; fi
}
step tests 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  --junitxml=$O/junit.xml > $O/gpu_tests.log 2>&1
tail -2 $O/gpu_tests.log >&2
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
for w in c1 c2 c3 c4; do
  WORKLOAD=$w OUT=$O/prof_$w GIT_HEAD=${GIT_HEAD:-} step prof_$w 600 bash scripts/gpu_profile.sh
  head -4 $O/prof_$w/summary.txt >&2
done
WORKLOAD=c2 OUT=$O/prof_c2_32768 STEPS=24 BENCH_ARGS="--txns 32768" GIT_HEAD=${GIT_HEAD:-} step prof_c2_32768 600 bash scripts/gpu_profile.sh
head -4 $O/prof_c2_32768/summary.txt >&2
