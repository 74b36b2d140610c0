#!/bin/bash
# Round 5, first GPU call: the new tests (RCCL leg at world 1, TooOld at full size, flag vs
# epilogue end, routed error paths), then the whole GPU suite, the smoke, and C2 bench lines
# (default, and with 2 % of snapshots at the window's edge).
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/r05a
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
step new_tests 900 $PT tests/test_gpu_multi.py::test_routed_batch_errors_leave_it_empty_and_reroutable \
  "tests/test_gpu_multi.py::test_rccl_leg_one_rank" tests/test_gpu_fullsize.py::test_full_c2_too_old_at_window_edge \
  tests/test_gpu_fullsize.py::test_flag_before_epilogue_end_without_submit_thread > $O/new_tests.log 2>&1
tail -3 $O/new_tests.log >&2
step all_tests 900 $PT tests -m gpu > $O/gpu_tests.log 2>&1
tail -3 $O/gpu_tests.log >&2
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
step bench_c2 600 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err
step bench_c2_tooold 600 python bench.py --too-old-frac 0.02 > $O/bench_c2_tooold.json 2> $O/bench_c2_tooold.err
echo done >&2
