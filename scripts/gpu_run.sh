#!/bin/bash
# One GPU session: parity tests, smoke, short bench.  Stops at the first step that faults,
# aborts, segfaults or times out (exit 124/134/137/139 or >128); a plain test failure (1)
# still lets the bench run so its numbers come back.
set -u
mkdir -p gpurun_out
step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "== $name" >&2
  timeout -k 10 "$t" "$@"
  local rc=$?
  echo "== $name rc=$rc" >&2
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)" >&2; exit $rc; fi
  return 0
}
step tests 900 python -m pytest tests -m gpu -q --timeout 600 -p no:cacheprovider ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
tail -30 gpurun_out/gpu_tests.log >&2
if [ "${REQUIRE_PASS:-1}" = "1" ] && ! grep -q " passed" gpurun_out/gpu_tests.log; then echo "no passing tests; stop" >&2; exit 1; fi
if [ "${REQUIRE_PASS:-1}" = "1" ] && grep -q " failed" gpurun_out/gpu_tests.log; then echo "tests failed; skipping bench" >&2; exit 1; fi
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
tail -5 gpurun_out/smoke.log >&2
step bench 600 python bench.py ${BENCH_ARGS:---steps 30 --warmup 3} > gpurun_out/bench.json 2> gpurun_out/bench.err
cat gpurun_out/bench.json >&2
tail -5 gpurun_out/bench.err >&2
if [ "${PROFILE:-0}" = "1" ]; then
  step profile 600 bash scripts/gpu_profile.sh
  cat gpurun_out/prof/summary.txt >&2 || true
fi
