#!/bin/bash
# The driver's command (C2, --steps 20 --warmup 5) REPS times on one box: value, H2D-inclusive,
# device-bound and the calling thread's submit time per batch, to see run-to-run spread.
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/${TAG:-r06rep}
mkdir -p $O
for r in $(seq 1 ${REPS:-5}); do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 ${BENCH_ARGS:-} > $O/c2_20_$r.json 2> $O/c2_20_$r.err || exit $?
  python3 -c "
import json; d=json.loads(open('$O/c2_20_$r.json').read().splitlines()[-1]); h=d['host_ms_per_batch']
print('rep $r', round(d['value']/1e6,2), 'h2d', round(d['h2d_inclusive_txns_per_s']/1e6,2), 'dev', round(d['device_bound']['txns_per_s']/1e6,2), 'submit_ms', round(h['submit'],4), 'engine_submit', round(h['engine_submit'],4), 'wait', round(h['wait'],4), 'parity', d['parity']['mismatched_batches'])" >&2
done
