#!/bin/bash
# Round 6: the whole GPU suite on the working tree, then the same-box A/B of VARIANTS at WORKLOADS
# (20-step lines, REPS reps).
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/${TAG:-r06h}
mkdir -p $O
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  > $O/gpu_tests.log 2>&1
rc=$?
tail -3 $O/gpu_tests.log >&2
[ $rc -ne 0 ] && exit $rc
summ() { python3 -c "import json,sys;d=json.load(open('$1'));k=d['kernels'];print('$2',round(d['value']/1e6,2),'h2d',round(d['h2d_inclusive_txns_per_s']/1e6,2),'dev',round((d['device_bound'] or {}).get('txns_per_s',0)/1e6,2),'par',d['parity']['mismatched_batches'],{n:round(x['avg_launch_ms']*1e3,1) for n,x in list(k.items())[:7]})" >&2; }
for rep in $(seq 1 ${REPS:-2}); do
for w in ${WORKLOADS:-c2 c3 c4}; do
for v in ${VARIANTS:-two dir8h}; do
  FDBCS_LIB=foundationdb_amd/variants/libfdbcs_$v.so timeout -k 10 400 python3 bench.py --workload $w --steps 20 --warmup 5 --cpu-seconds 5 --total-steps 0 --breakdown-steps 0 --sync-steps 0 > $O/${w}_${v}_$rep.json 2> $O/${w}_${v}_$rep.err || exit $?
  summ $O/${w}_${v}_$rep.json "$w $v $rep"
done
done
done
