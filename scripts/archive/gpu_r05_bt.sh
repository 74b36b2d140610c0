#!/bin/bash
# Compaction copy tile (FDBCS_BASE_TILE 1024/2048/4096): parity, then rocprof of C2 and C4 over 200
# timed batches per tile (k_merge_copy<CompactIns, tile> duration).
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/${TAG:-r05bt}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -m gpu \
  -k "compaction_search_modes or delta_tier or long_shared or c4_tuple" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for w in c2 c4; do
  for t in ${TILES:-1024 2048 4096}; do
    FDBCS_BASE_TILE=$t WORKLOAD=$w OUT=$O/p_${w}_$t STEPS=200 timeout -k 10 400 bash scripts/gpu_profile.sh || exit 1
    echo "$w tile $t: $(grep -h 'CompactIns\|compact_search\|CompactSum\|epilogue<true' $O/p_${w}_$t/summary.txt | sed 's/  */ /g' | cut -c1-90 | tr '\n' '|')"
    python3 -c "
import json;d=json.load(open('$O/p_${w}_$t/bench.json'))
print('   value %.2fM'%(d['value']/1e6), 'ms/step %.4f'%d['ms_per_step'])"
  done
done
