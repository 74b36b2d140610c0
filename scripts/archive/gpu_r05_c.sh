#!/bin/bash
# Round 5: no-op X launches left out -- GPU suite, C2/C3 bench lines with the skip on and off
# (same box), rocprof kernel trace of C2.
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/${TAG:-r05c}
mkdir -p $O
step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "== $name $(date +%T)" >&2
  timeout -k 10 "$t" "$@"
  local rc=$?
  echo "== $name rc=$rc" >&2
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >&2; exit $rc; fi
  return 0
}
PT="python -u -m pytest -x -v --timeout 280 --timeout-method thread -p no:cacheprovider"
if [ "${SKIP_TESTS:-0}" != "1" ]; then
step all_tests 900 $PT tests -m gpu > $O/gpu_tests.log 2>&1
tail -3 $O/gpu_tests.log >&2
fi
for w in ${WORKLOADS:-c2 c3}; do
  step bench_$w 600 python bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err
  FDBCS_SKIP_EDGES=0 step bench_${w}_noskip 600 python bench.py --workload $w > $O/bench_${w}_noskip.json 2> $O/bench_${w}_noskip.err
done
if [ "${PROFILE:-1}" = "1" ]; then
  WORKLOAD=c2 OUT=$O/prof_c2 step prof_c2 660 bash scripts/gpu_profile.sh
fi
echo done >&2
