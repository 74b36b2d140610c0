#!/bin/bash
# C2 same-box A/B of the compaction knobs: defaults, FDBCS_BASE_TILE=4096, FDBCS_COMPACT_LANES=0, both.
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/${TAG:-r05c2k}
mkdir -p $O
for r in 1 2; do
  for v in def tile lanes both old; do
    case $v in def) E="" ;; tile) E="FDBCS_BASE_TILE=4096" ;; lanes) E="FDBCS_COMPACT_LANES=0" ;;
      both) E="FDBCS_BASE_TILE=4096 FDBCS_COMPACT_LANES=0" ;; old) E="" ;; esac
    d=.; [ $v = old ] && d=ab_old
    (cd $d && env $E timeout -k 10 300 python bench.py --workload c2 --steps 200 --warmup 20 --no-cpu-baseline --breakdown-steps 0 \
      --sync-steps 0 --h2d-steps 0 --total-steps 0) > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || exit 1
    python3 -c "
import json;d=json.load(open('$O/b_${v}_$r.json'))
print('c2 $v r$r value %.2fM'%(d['value']/1e6), 'ms/step %.4f'%d['ms_per_step'])"
  done
done
