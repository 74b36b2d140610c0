#!/bin/bash
# Delta bound 1.25M vs automatic (N/16) at C3 and at 32768-txn C2 batches, long windows.
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/${TAG:-r05dl3}
mkdir -p $O
for r in 1 2; do
  for a in "c3 400" "c2_32768 150"; do
    set -- $a
    w=${1%%_*}; st=$2; tx=""; [ "$1" = "c2_32768" ] && tx="--txns 32768"
    for dl in 0 1250000; do
      timeout -k 10 400 python bench.py --workload $w $tx --steps $st --warmup 20 --no-cpu-baseline --breakdown-steps 0 --sync-steps 0 \
        --h2d-steps 0 --total-steps 0 --delta-limit $dl > $O/b.json 2> $O/b.err || exit 1
      python3 -c "
import json;d=json.load(open('$O/b.json'))
print('$1 delta-limit $dl r$r value %.2fM'%(d['value']/1e6), 'ms/step %.4f'%d['ms_per_step'])"
    done
  done
done
