#!/bin/bash
# Round 6: the GPU suite on the current build, then the driver's bench command.
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/${TAG:-r06c}
mkdir -p $O
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  > $O/gpu_tests.log 2>&1
rc=$?
tail -5 $O/gpu_tests.log >&2
grep -E 'PASSED|FAILED|ERROR' $O/gpu_tests.log | awk '{print $NF, $1}' | sort | uniq -c | sort -rn | head -3 >&2
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/c2_20.json 2> $O/c2_20.err || exit $?
python3 -c "import json;d=json.load(open('$O/c2_20.json'));print('c2 20-step',d['value']/1e6,d['h2d_inclusive_txns_per_s']/1e6,d['device_bound']['txns_per_s']/1e6,d['parity'],d['roofline']['kernel'],d['roofline']['frac'])" >&2
