#!/bin/bash
# Same-box A/B of the previous engine build (worktree ab_old/) against the current one, C1 and C2.
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/${TAG:-r05abold}
mkdir -p $O
for r in 1 2; do
  for w in ${WLS:-c1 c2}; do
    for v in old new; do
      d=.; [ $v = old ] && d=ab_old
      (cd $d && timeout -k 10 300 python bench.py --workload $w --steps 200 --warmup 20 --no-cpu-baseline --breakdown-steps 0 \
        --sync-steps 0 --h2d-steps 0 --total-steps 0) > $O/b_${w}_${v}_$r.json 2> $O/b_${w}_${v}_$r.err || exit 1
      python3 -c "
import json;d=json.load(open('$O/b_${w}_${v}_$r.json'))
print('$w $v r$r value %.2fM'%(d['value']/1e6), 'ms/step %.4f'%d['ms_per_step'])"
    done
  done
done
