#!/bin/bash
# Sort bucket target at C4 (FDBCS_SORT_BUCKET; default 64): same-box bench A/B, 200 timed batches.
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/${TAG:-r05sb4}
mkdir -p $O
for r in 1 2; do
  for t in ${TS:-64 32 48 96 128}; do
    FDBCS_SORT_BUCKET=$t timeout -k 10 300 python bench.py --workload ${W:-c4} --steps 200 --warmup 20 --no-cpu-baseline \
      --breakdown-steps 0 --sync-steps 0 --h2d-steps 0 --total-steps 0 > $O/b_${t}_$r.json 2> $O/b_${t}_$r.err || exit 1
    python3 -c "
import json;d=json.load(open('$O/b_${t}_$r.json'))
k=d['kernels']; sb=[v for n,v in k.items() if n.startswith('k_sort_bucket')]
print('${W:-c4} bucket $t r$r value %.2fM'%(d['value']/1e6), 'ms/step %.4f'%d['ms_per_step'], 'sort_bucket us %.1f'%(sb[0]['avg_launch_ms']*1e3 if sb else -1))"
  done
done
