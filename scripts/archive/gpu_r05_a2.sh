#!/bin/bash
# Two stage-A streams (FDBCS_A2=1: every other batch's sort and edges on astream2, the next sort
# waiting only for the previous sort): parity suite under it, then same-box bench A/B.
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/${TAG:-r05a2}
mkdir -p $O
FDBCS_A2=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for w in ${WLS:-c2 c4 c3}; do
    for a in 0 1; do
      FDBCS_A2=$a timeout -k 10 300 python bench.py --workload $w --steps 200 --warmup 20 --no-cpu-baseline --breakdown-steps 0 \
        --sync-steps 0 --h2d-steps 0 --total-steps 0 > $O/b_${w}_${a}_$r.json 2> $O/b_${w}_${a}_$r.err || exit 1
      python3 -c "
import json;d=json.load(open('$O/b_${w}_${a}_$r.json'))
print('$w a2=$a r$r value %.2fM'%(d['value']/1e6), 'ms/step %.4f'%d['ms_per_step'], 'dev', d.get('device_bound',{}).get('ms_per_batch'))"
    done
  done
done
