#!/bin/bash
# Sort bucket target (FDBCS_SORT_BUCKET) same-box A/B at C2: line value and the sort kernels'
# per-launch times from the line's profile pass.
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/${TAG:-r05sb}
mkdir -p $O
for r in 1 2; do
  for t in 64 48 40; do
    FDBCS_SORT_BUCKET=$t timeout -k 10 300 python bench.py --workload c2 --steps 60 --no-cpu-baseline --breakdown-steps 0 \
      --sync-steps 0 --h2d-steps 0 --total-steps 0 > $O/b_${t}_${r}.json 2> $O/b_${t}_${r}.err || exit 1
    python3 -c "
import json;d=json.load(open('$O/b_${t}_${r}.json'));k=d['kernels']
f=lambda n:round(k[n]['avg_launch_ms']*1e3,1) if n in k else None
print('target $t r$r value %.2fM'%(d['value']/1e6), 'bucket', f('k_sort_bucket<false>'), 'partition', f('k_sort_partition'), 'edgescan', f('k_scan<3, fdbcs::EdgePairScan, 1>'))"
  done
done
