#!/bin/bash
# Delta bound at C4 (default N/16 = 3.1M at 50M): same-box A/B over 400 timed batches.
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/${TAG:-r05c4dl}
mkdir -p $O
for r in 1 2; do
  for dl in ${DLS:-0 6250000 12500000}; do
    timeout -k 10 300 python bench.py --workload c4 --steps 400 --warmup 20 --no-cpu-baseline --breakdown-steps 0 --sync-steps 0 \
      --h2d-steps 0 --total-steps 0 --delta-limit $dl > $O/b_${dl}_${r}.json 2> $O/b_${dl}_${r}.err || exit 1
    python3 -c "
import json;d=json.load(open('$O/b_${dl}_${r}.json'))
print('c4 delta-limit $dl r$r value %.2fM'%(d['value']/1e6), 'ms/step %.4f'%d['ms_per_step'], 'compactions', d.get('compactions'))"
  done
done
