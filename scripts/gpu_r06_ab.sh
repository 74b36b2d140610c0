#!/bin/bash
# Round 6 same-box A/B of engine env knobs on the bench: VARIANTS="name:ENV=V,ENV=V ..." (an empty
# env list is the default build), WLS workloads, ROUNDS interleaved rounds.  Optional PARITY_ENV
# runs the GPU suite once under that env first.  Output gpurun_out/${TAG:-r06ab}/.
set -u
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06ab}
mkdir -p $O
if [ -n "${PARITY_ENV:-}" ]; then
  ( IFS=','; for e in $PARITY_ENV; do export "$e"; done; unset IFS
    timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 )
  rc=$?; tail -2 $O/gpu_tests.log >&2; [ $rc -ne 0 ] && exit $rc
fi
for w in ${WLS:-c2}; do
  for r in $(seq 1 ${ROUNDS:-2}); do
    for v in ${VARIANTS}; do
      name=${v%%:*}; envs=${v#*:}
      f=$O/${w}_${name}_$r
      (
        IFS=','; for e in $envs; do [ -n "$e" ] && export "$e"; done; unset IFS
        timeout -k 10 300 python3 bench.py --workload $w --steps ${STEPS:-60} --warmup 5 --no-cpu-baseline \
          --breakdown-steps 0 --sync-steps 0 --total-steps 0 --h2d-steps 0 ${BENCH_ARGS:-} > $f.json 2> $f.err
      ) || { echo "$w $name failed" >&2; tail -5 $f.err >&2; exit 1; }
      python3 -c "
import json;d=json.loads(open('$f.json').read().splitlines()[-1])
db=d.get('device_bound') or {}; k=d.get('kernels') or {}
top=sorted(k.items(), key=lambda x:-x[1]['avg_launch_ms'])[:8]
print('%s %-10s r$r %6.2fM dev %s | %s' % ('$w', '$name', d['value']/1e6, round((db.get('txns_per_s') or 0)/1e6,2), ' '.join('%s=%.1f' % (n.split('<')[0].replace('k_',''), v['avg_launch_ms']*1e3) for n,v in top)))" >&2
    done
  done
done
