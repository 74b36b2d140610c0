#!/bin/bash
# Non-temporal compaction copy at the 4096 tile (FDBCS_COPY_NT 0/1): parity, rocprof of C4 per
# setting, then same-box bench A/B.
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/${TAG:-r05nt}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -m gpu \
  -k "compaction_search_modes or long_shared or c4_tuple" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for c in 0 1; do
  FDBCS_COPY_NT=$c WORKLOAD=${W:-c4} OUT=$O/p_${W:-c4}_$c STEPS=200 timeout -k 10 400 bash scripts/gpu_profile.sh || exit 1
  echo "nt $c: $(grep -h 'CompactIns' $O/p_${W:-c4}_$c/summary.txt | sed 's/  */ /g' | cut -c1-90)"
done
for r in 1 2; do
  for c in 0 1; do
    FDBCS_COPY_NT=$c timeout -k 10 300 python bench.py --workload ${W:-c4} --steps 200 --warmup 20 --no-cpu-baseline \
      --breakdown-steps 0 --sync-steps 0 --h2d-steps 0 --total-steps 0 > $O/b_${c}_${r}.json 2> $O/b_${c}_$r.err || exit 1
    python3 -c "
import json;d=json.load(open('$O/b_${c}_${r}.json'))
print('${W:-c4} nt $c r$r value %.2fM'%(d['value']/1e6), 'ms/step %.4f'%d['ms_per_step'])"
  done
done
