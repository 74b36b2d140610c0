#!/bin/bash
# Round 6: the GPU suite on the three-tier build, then the driver's command at C2 and 20-step
# lines at C3 / C4, and a 200-step C2 window.
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/${TAG:-r06d}
mkdir -p $O
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  > $O/gpu_tests.log 2>&1
rc=$?
tail -4 $O/gpu_tests.log >&2
[ $rc -ne 0 ] && exit $rc
fi
summ() { python3 -c "import json,sys;d=json.load(open('$1'));k=d['kernels'];print('$2',round(d['value']/1e6,2),'h2d',round(d['h2d_inclusive_txns_per_s']/1e6,2),'dev',round((d['device_bound'] or {}).get('txns_per_s',0)/1e6,2),'par',d['parity']['mismatched_batches'],d['parity']['batches_checked'],'roof',d['roofline']['kernel'],round(d['roofline']['frac'],3),'cmp',d['compactions'],{n:round(x['avg_launch_ms']*1e3,1) for n,x in list(k.items())[:8]})" >&2; }
for w in c2 c3 c4; do
  timeout -k 10 400 python3 bench.py --workload $w --steps 20 --warmup 5 --cpu-seconds 15 > $O/${w}_20.json 2> $O/${w}_20.err || exit $?
  summ $O/${w}_20.json "$w-20"
done
timeout -k 10 400 python3 bench.py --steps 200 --warmup 5 --cpu-seconds 15 --breakdown-steps 128 > $O/c2_200.json 2> $O/c2_200.err || exit $?
summ $O/c2_200.json c2-200
