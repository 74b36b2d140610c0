#!/bin/bash
# Round 6 evidence, part C (final build): the builder's 200-step lines of C1, C3, C4, C2 at
# 32768-txn batches and C2 with 5 % of the snapshots at the window's edge (TooOld), then the
# randomized parity stress for the time left.
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
line() {
  local tag=$1; shift
  step bench_$tag 500 python3 bench.py "$@" > $O/bench_$tag.json 2> $O/bench_$tag.err
  python3 -c "
import json; d=json.loads(open('$O/bench_$tag.json').read().splitlines()[-1]); r=d['roofline']
print('$tag', round(d['value']/1e6,2), 'M; h2d', round((d['h2d_inclusive_txns_per_s'] or 0)/1e6,2), 'dominant', r['kernel'], 'frac', round(r['frac'],3), 'parity', d['parity']['mismatched_batches'], '/', d['parity']['batches_checked'], 'mix_total', d.get('verdict_mix_total'))" >&2
}
for w in ${LINES:-c1 c3 c4}; do line ${w}_200 --workload $w --steps 200 --warmup 5; done
[ -n "${NO_32768:-}" ] || line c2_32768 --txns 32768 --steps 200 --warmup 5
[ -n "${NO_TOOOLD:-}" ] || line c2_tooold --steps 200 --warmup 5 --too-old-frac 0.05
[ "${STRESS_S:-0}" -gt 0 ] && step stress 900 python3 scripts/stress_parity.py ${STRESS_S} ${STRESS_SEED:-30001} > $O/stress.log 2>&1
tail -3 $O/stress.log >&2 2>/dev/null || true
