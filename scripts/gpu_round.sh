#!/bin/bash
# Round evidence in one GPU call: parity tests, smoke, then per workload a bench line (with the
# CPU baseline and parity replay) and a rocprofv3 kernel-trace profile.  Output: gpurun_out/$TAG/.
# Stops at the first step that faults, aborts or times out.
set -u
cd "$(dirname "$0")/.." || exit 1
TAG=${TAG:-r02}
O=gpurun_out/$TAG
mkdir -p $O
step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "== $name $(date +%T)" >&2
  timeout -k 10 "$t" "$@"
  local rc=$?
  echo "== $name rc=$rc" >&2
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)" >&2; exit $rc; fi
  return 0
}
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  step tests 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
  tail -5 $O/gpu_tests.log >&2
  grep -qE "[0-9]+ (failed|error)" $O/gpu_tests.log && { echo "tests failed; stop" >&2; exit 1; }
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
fi
for w in ${WORKLOADS:-c2 c3 c4}; do
  step bench_$w 600 python bench.py --workload $w ${BENCH_ARGS:-} > $O/bench_$w.json 2> $O/bench_$w.err
  cat $O/bench_$w.json >&2
  if [ "${PROFILE:-1}" = "1" ]; then
    WORKLOAD=$w OUT=$O/prof_$w step prof_$w 660 bash scripts/gpu_profile.sh
    head -3 $O/prof_$w/timeline.txt >&2
  fi
done
