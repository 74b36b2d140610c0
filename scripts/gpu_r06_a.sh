#!/bin/bash
# Round 6: the driver's command (--steps 20 --warmup 5) twice, then a 200-step window, at C2.
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/${TAG:-r06a}
mkdir -p $O
for n in 1 2; do
  timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/c2_20_$n.json 2> $O/c2_20_$n.err || exit $?
  python3 -c "import json,sys;d=json.load(open('$O/c2_20_$n.json'));print('20-step',d['value']/1e6,d['h2d_inclusive_txns_per_s']/1e6,d['device_bound']['txns_per_s']/1e6,d['parity']['mismatched_batches'])" >&2
done
timeout -k 10 300 python3 bench.py --gpus 1 --steps 200 --warmup 5 --cpu-seconds 20 > $O/c2_200.json 2> $O/c2_200.err || exit $?
python3 -c "import json,sys;d=json.load(open('$O/c2_200.json'));print('200-step',d['value']/1e6,d['h2d_inclusive_txns_per_s']/1e6,d['device_bound']['txns_per_s']/1e6,d['parity']['mismatched_batches'])" >&2
