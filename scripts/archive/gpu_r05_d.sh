#!/bin/bash
# Round 5: epilogue without the slot, bucket-sort prologue overlapped -- GPU suite, isolated sort
# sweep over the bucket size, a device trace of the sort sections, C2/C3 bench lines.
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/${TAG:-r05d}
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
WORKLOAD=c2 WHICH=1,2 step sweep 400 python3 scripts/kernel_sweep.py "FDBCS_SORT_BUCKET=32" "FDBCS_SORT_BUCKET=48" \
  "FDBCS_SORT_BUCKET=64" "FDBCS_SORT_BUCKET=96" > $O/sort_sweep.txt 2>&1
cat $O/sort_sweep.txt >&2
step trace 200 python3 scripts/trace_c2.py 8 5000 c2 > $O/trace_c2.txt 2>&1
for w in ${WORKLOADS:-c2 c3}; do
  step bench_$w 600 python bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err
done
echo done >&2
