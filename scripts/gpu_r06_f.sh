#!/bin/bash
# Round 6: the GPU suite on the working tree (directory over group starts), then a same-box A/B
# against the previous build (variants/libfdbcs_two.so) at C2 / C3 / C4, 20-step lines, two reps,
# plus the isolated check kernels.
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/${TAG:-r06f}
mkdir -p $O
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  > $O/gpu_tests.log 2>&1
rc=$?
tail -3 $O/gpu_tests.log >&2
[ $rc -ne 0 ] && exit $rc
fi
for v in two dir8; do
  FDBCS_LIB=foundationdb_amd/variants/libfdbcs_$v.so WHICH=0,3,4 timeout -k 10 200 python3 scripts/kernel_sweep.py "V=$v" > $O/ks_$v.txt 2>&1 || exit $?
  cat $O/ks_$v.txt >&2
done
summ() { python3 -c "import json,sys;d=json.load(open('$1'));k=d['kernels'];print('$2',round(d['value']/1e6,2),'h2d',round(d['h2d_inclusive_txns_per_s']/1e6,2),'dev',round((d['device_bound'] or {}).get('txns_per_s',0)/1e6,2),'par',d['parity']['mismatched_batches'],{n:round(x['avg_launch_ms']*1e3,1) for n,x in list(k.items())[:6]})" >&2; }
for rep in 1 2; do
for w in ${WORKLOADS:-c2 c3 c4}; do
for v in two dir8; do
  FDBCS_LIB=foundationdb_amd/variants/libfdbcs_$v.so timeout -k 10 400 python3 bench.py --workload $w --steps 20 --warmup 5 --cpu-seconds 5 --total-steps 0 --breakdown-steps 0 --sync-steps 0 > $O/${w}_${v}_$rep.json 2> $O/${w}_${v}_$rep.err || exit $?
  summ $O/${w}_${v}_$rep.json "$w $v $rep"
done
done
done
