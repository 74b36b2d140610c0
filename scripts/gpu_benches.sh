#!/bin/bash
# The bench lines of every workload at the current build (after profiles/ holds its rocprof and
# PMC files): gpurun_out/$TAG/bench_<w>.json.
set -u
cd "$(dirname "$0")/.." || exit 1
TAG=${TAG:-r04e}
O=gpurun_out/$TAG
mkdir -p $O
for w in c2 c1 c3 c4; do
  timeout -k 10 600 python bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || { echo "bench $w failed"; tail -5 $O/bench_$w.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench_$w.json').read().splitlines()[-1]); r=d['roofline']
print('$w', round(d['value']/1e6,2), 'M; dominant', r['kernel'], 'frac', round(r['frac'],3), 'frac_rocprof', r.get('frac_rocprof'), 'traffic', r.get('traffic'), 'parity', d['parity']['mismatched_batches'], '/', d['parity']['batches_checked'])"
done
timeout -k 10 600 python bench.py --workload c2 --txns 32768 > $O/bench_c2_32768.json 2> $O/bench_c2_32768.err || exit 1
python3 -c "
import json; d=json.loads(open('$O/bench_c2_32768.json').read().splitlines()[-1]); print('c2 32768', round(d['value']/1e6,2))"
