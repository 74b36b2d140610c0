#!/bin/bash
# Round 6: same-box A/B of the two-tier build (git f5196fd) against the three-tier build with the
# small-base check layout (base + delta in X, mid tier on the split stream): 20-step lines at C2,
# C3 and C4 (two reps, interleaved) and a 200-step C2 window each.
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/${TAG:-r06e}
mkdir -p $O
summ() { python3 -c "import json,sys;d=json.load(open('$1'));k=d['kernels'];print('$2',round(d['value']/1e6,2),'h2d',round(d['h2d_inclusive_txns_per_s']/1e6,2),'dev',round((d['device_bound'] or {}).get('txns_per_s',0)/1e6,2),'par',d['parity']['mismatched_batches'],'cmp',d['compactions'],{n:round(x['avg_launch_ms']*1e3,1) for n,x in list(k.items())[:6]})" >&2; }
for rep in 1 2; do
for w in c2 c3 c4; do
for v in two threeB; do
  FDBCS_LIB=foundationdb_amd/variants/libfdbcs_$v.so timeout -k 10 400 python3 bench.py --workload $w --steps 20 --warmup 5 --cpu-seconds 5 --total-steps 0 --breakdown-steps 0 --sync-steps 0 > $O/${w}_${v}_$rep.json 2> $O/${w}_${v}_$rep.err || exit $?
  summ $O/${w}_${v}_$rep.json "$w $v $rep"
done
done
done
for v in two threeB; do
  FDBCS_LIB=foundationdb_amd/variants/libfdbcs_$v.so timeout -k 10 400 python3 bench.py --steps 200 --warmup 5 --cpu-seconds 5 --total-steps 0 --breakdown-steps 0 --sync-steps 0 > $O/c2_200_$v.json 2> $O/c2_200_$v.err || exit $?
  summ $O/c2_200_$v.json "c2-200 $v"
done
