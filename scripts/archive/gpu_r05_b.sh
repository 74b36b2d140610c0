#!/bin/bash
# Round 5: parallel addTransaction -- the new rejection test, the GPU suite, C2 and C4 bench lines
# (add time per batch in total_host_ms_per_batch).
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/${TAG:-r05b}
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
step new_tests 600 $PT tests/test_gpu_parity.py -k "inverted" > $O/new_tests.log 2>&1
tail -3 $O/new_tests.log >&2
step all_tests 900 $PT tests -m gpu > $O/gpu_tests.log 2>&1
tail -3 $O/gpu_tests.log >&2
step bench_c2 600 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err
step bench_c4 600 python bench.py --workload c4 > $O/bench_c4.json 2> $O/bench_c4.err
echo done >&2
