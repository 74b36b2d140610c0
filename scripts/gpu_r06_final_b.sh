#!/bin/bash
# Round 6 evidence, part B (final build, profiles/ holding part A's rocprof rankings): PMC traffic
# passes of C2 and C4 (copied into profiles/ on the box so the bench lines carry `traffic`), then
# the driver's command (C2, 20 steps) twice and the builder's 200-step C2 line.
set -u
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06final}
mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  echo "== $name $(date +%T)" >&2
  timeout -k 10 "$t" "$@"
  local rc=$?
  echo "== $name rc=$rc" >&2
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >&2; exit $rc; fi
}
for w in c2 c4; do
  WORKLOAD=$w GIT_HEAD=${GIT_HEAD:-} step pmc_$w 600 bash scripts/gpu_pmc.sh
done
mkdir -p $O/pmc && cp gpurun_out/pmc/pmc_*.json $O/pmc/ && cp gpurun_out/pmc/pmc_*.json profiles/
line() {  # tag, args...
  local tag=$1; shift
  step bench_$tag 500 python3 bench.py "$@" > $O/bench_$tag.json 2> $O/bench_$tag.err
  python3 -c "
import json; d=json.loads(open('$O/bench_$tag.json').read().splitlines()[-1]); r=d['roofline']
print('$tag', round(d['value']/1e6,2), 'M; h2d', round((d['h2d_inclusive_txns_per_s'] or 0)/1e6,2), 'dev', round(((d['device_bound'] or {}).get('txns_per_s') or 0)/1e6,2), 'dominant', r['kernel'], 'frac', round(r['frac'],3), 'frac_rocprof', r.get('frac_rocprof'), 'traffic', r.get('traffic'), 'parity', d['parity']['mismatched_batches'], '/', d['parity']['batches_checked'])" >&2
}
line c2_20a --steps 20 --warmup 5
line c2_20b --steps 20 --warmup 5
line c2_200 --steps 200 --warmup 5
