#!/bin/bash
# Round 6: D.Sort variants (bucket target, speculative slab slots): isolated kernel times and the
# driver's 20-step line, same box.
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/${TAG:-r06b}
mkdir -p $O
for v in ${VARIANTS:-base s80 t48 t48s64}; do
  FDBCS_LIB=foundationdb_amd/variants/libfdbcs_$v.so WHICH=1,2,0 timeout -k 10 200 python3 scripts/kernel_sweep.py "V=$v" > $O/ks_$v.txt 2>&1 || exit $?
  cat $O/ks_$v.txt >&2
done
for rep in 1 2; do
for v in ${VARIANTS:-base s80 t48 t48s64}; do
  FDBCS_LIB=foundationdb_amd/variants/libfdbcs_$v.so timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 --cpu-seconds 5 --total-steps 0 --breakdown-steps 0 > $O/b_${v}_$rep.json 2> $O/b_${v}_$rep.err || exit $?
  python3 -c "import json;d=json.load(open('$O/b_${v}_$rep.json'));k=d['kernels'];print('$v',round(d['value']/1e6,2),round(d['device_bound']['txns_per_s']/1e6,2),{n:round(x['avg_launch_ms']*1e3,1) for n,x in k.items() if 'sort' in n or 'check_lanes' in n},d['parity']['mismatched_batches'])" >&2
done
done
