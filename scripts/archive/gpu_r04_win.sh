#!/bin/bash
# In-flight window sweep of the C2 line (host-submitted pipeline vs the device-bound rate).
set -u
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/win
for w in 4 8 16 32; do
  for th in 0 1; do
    FDBCS_SUBMIT_THREAD=$th timeout -k 10 300 python bench.py --steps 400 --warmup 100 --no-cpu-baseline --breakdown-steps 0 \
      --sync-steps 0 --resident-steps 0 --total-steps 0 --window $w > gpurun_out/win/w${w}_t$th.json 2> gpurun_out/win/w${w}_t$th.err || exit 1
    python3 -c "
import json;d=json.loads(open('gpurun_out/win/w${w}_t$th.json').read().splitlines()[-1]);h=d['host_ms_per_batch']
print('window $w thread $th: %.2fM ms/step %.4f submit %.4f wait %.4f device_bound %.4f' % (d['value']/1e6, d['ms_per_step'], h['submit'], h['wait'], d['device_bound']['ms_per_batch']))"
  done
done
