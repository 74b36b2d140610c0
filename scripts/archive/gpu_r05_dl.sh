#!/bin/bash
# Delta bound at C2 (bench --delta-limit; default N/16 = 312500 at 5M): same-box A/B.
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/${TAG:-r05dl}
mkdir -p $O
for r in 1 2; do
  for dl in 0 625000 1250000; do  # 400 timed steps: several compaction cycles each
    timeout -k 10 300 python bench.py --workload c2 --steps 400 --warmup 20 --no-cpu-baseline --breakdown-steps 0 --sync-steps 0 \
      --h2d-steps 0 --total-steps 0 --delta-limit $dl > $O/b_${dl}_${r}.json 2> $O/b_${dl}_${r}.err || exit 1
    python3 -c "
import json;d=json.load(open('$O/b_${dl}_${r}.json'))
print('delta-limit $dl r$r value %.2fM'%(d['value']/1e6), 'ms/step %.4f'%d['ms_per_step'], 'compactions', d.get('compactions'))"
  done
done
