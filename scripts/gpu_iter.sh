#!/bin/bash
# One build-measure iteration: GPU parity tests (optional), isolated kernel sweeps and a short C2
# bench.  TESTS=0 skips the tests; SWEEP="variant ..." (kernel_sweep.py specs); WORKLOADS for sweeps.
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/${TAG:-iter}
mkdir -p $O
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    -k "${TEST_K:-}" > $O/gpu_tests.log 2>&1
  rc=$?
  tail -3 $O/gpu_tests.log
  [ $rc -ne 0 ] && { grep -E "FAILED|Error|error" $O/gpu_tests.log | head -20; exit $rc; }
fi
for w in ${WORKLOADS:-c2}; do
  if [ -n "${SWEEP:-}" ]; then
    WORKLOAD=$w WHICH=${WHICH:-0} timeout -k 10 400 python scripts/kernel_sweep.py ${SWEEP} > $O/sweep_$w.txt 2>&1 || { cat $O/sweep_$w.txt; exit 1; }
    cat $O/sweep_$w.txt
  fi
done
for w in ${BENCH:-}; do
  timeout -k 10 400 python bench.py --workload $w ${BENCH_ARGS:---steps 40 --cpu-seconds 20} > $O/bench_$w.json 2> $O/bench_$w.err || { tail -20 $O/bench_$w.err; exit 1; }
  python scripts/bench_summary.py $O/bench_$w.json 2>/dev/null || head -c 600 $O/bench_$w.json
done
