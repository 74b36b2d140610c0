#!/bin/bash
# Upload A/B: the DMA engine's copy vs a copy kernel over PCIe, with and without the helper thread.
set -u
cd "$(dirname "$0")/.." || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "c2_reduced or kat or frozen" || exit $?
ROUNDS=2 BENCH_ARGS="--steps 400 --warmup 100 --no-cpu-baseline --breakdown-steps 64 --sync-steps 0 --resident-steps 100 --total-steps 0" \
  VARIANTS="base: upk:FDBCS_UPLOAD=kernel thr:FDBCS_SUBMIT_THREAD=1 thrupk:FDBCS_SUBMIT_THREAD=1,FDBCS_UPLOAD=kernel" \
  bash scripts/gpu_ab_env.sh 2>&1 | tee gpurun_out/ab_upload.txt || exit $?
for n in base upk; do python3 -c "
import json; d=json.loads(open('gpurun_out/ab/${n}_1.json').read().splitlines()[-1])
print('$n', 'resident', d['device_resident_txns_per_s'], 'upload_ms', d['phase_ms_per_batch']['ms_upload'])"; done
