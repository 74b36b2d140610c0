#!/bin/bash
# k_compact_search modes (FDBCS_COMPACT_LANES 0/1/2): parity, then same-box bench A/B at C4/C2/C3
# (200 timed batches: C4's 50M-base compactions inside the window).
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/${TAG:-r05cl}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -m gpu \
  -k "compaction_search_modes or delta_tier or long_shared or c4_tuple" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in ${REPS:-1}; do
  for w in c4 c2 c3; do
    for m in 0 1 2; do
      FDBCS_COMPACT_LANES=$m timeout -k 10 300 python bench.py --workload $w --steps 200 --warmup 20 --no-cpu-baseline \
        --breakdown-steps 0 --sync-steps 0 --h2d-steps 0 --total-steps 0 > $O/b_${w}_${m}_${r}.json 2> $O/b_${w}_${m}_${r}.err || exit 1
      python3 -c "
import json;d=json.load(open('$O/b_${w}_${m}_${r}.json'))
print('$w mode $m r$r value %.2fM'%(d['value']/1e6), 'ms/step %.4f'%d['ms_per_step'], 'compactions', d.get('compactions'))"
    done
  done
done
