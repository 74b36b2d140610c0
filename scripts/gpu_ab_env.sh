#!/bin/bash
# A/B of environment variants on the C2 bench (same box, interleaved): VARIANTS="name:ENV=V,ENV=V ..."
# ROUNDS times each.  Output gpurun_out/ab/<name>_<round>.json and a summary on stderr.
set -u
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/ab
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${VARIANTS}; do
    name=${v%%:*}; envs=${v#*:}
    (
      IFS=','; for e in $envs; do [ -n "$e" ] && export "$e"; done; unset IFS
      timeout -k 10 300 python bench.py ${BENCH_ARGS:---steps 60 --no-cpu-baseline --breakdown-steps 0 --sync-steps 0 --h2d-steps 0 --total-steps 0} \
        > gpurun_out/ab/${name}_$r.json 2> gpurun_out/ab/${name}_$r.err
    ) || { echo "$name failed"; tail -5 gpurun_out/ab/${name}_$r.err; exit 1; }
    python3 -c "
import json;d=json.loads(open('gpurun_out/ab/${name}_$r.json').read().splitlines()[-1])
h=d['host_ms_per_batch'];db=d.get('device_bound') or {}
print('%-14s r$r value %6.2fM  ms/step %.4f  submit %.4f  engine_submit %.4f  device_bound %s' % ('$name', d['value']/1e6, d['ms_per_step'], h['submit'], h['engine_submit'], db.get('ms_per_batch')))"
  done
done
