#!/bin/bash
# GPU tests, then the bench under two settings of one env knob (A/B), e.g. AB_VAR=FDBCS_UPLOAD AB_A=kernel AB_B=dma.
set -u
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/ab
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 -p no:cacheprovider ${PYTEST_ARGS:-} > gpurun_out/ab/tests.log 2>&1
  rc=$?; tail -3 gpurun_out/ab/tests.log >&2; [ $rc -ne 0 ] && exit $rc
fi
for v in ${AB_A:-x} ${AB_B:-y}; do
  env ${AB_VAR:-FDBCS_NOOP}=$v timeout -k 10 300 python3 bench.py ${BENCH_ARGS:---steps 30 --warmup 3} > gpurun_out/ab/bench_$v.json 2> gpurun_out/ab/bench_$v.err || exit $?
  python3 -c "import json,sys;d=json.load(open('gpurun_out/ab/bench_$v.json'));print('$v', d['value'], d.get('device_resident_txns_per_s'), d.get('total_txns_per_s'), d.get('host_ms_per_batch'), d['parity']['mismatched_batches'] if d.get('parity') else None)" >&2
done
