#!/bin/bash
# Cost of the timed loop's sampled kernel events: --timing 1 (1 batch in 4, FDBCS_TIMING_EVERY)
# against every 16th batch and --timing 0, C2, same box, interleaved.
set -u
cd "$(dirname "$0")/.." || exit 1
A="--workload c2 --steps 300 --warmup 60 --no-cpu-baseline --breakdown-steps 0 --sync-steps 0 --total-steps 0"
for r in 1 2; do
  for v in t1 t16 t0; do
    case $v in t1) E="FDBCS_TIMING_EVERY=4"; X="";; t16) E="FDBCS_TIMING_EVERY=16"; X="";; t0) E="FDBCS_TIMING_EVERY=4"; X="--timing 0";; esac
    env $E timeout -k 10 300 python bench.py $A $X > gpurun_out/tm_${v}_$r.json 2> gpurun_out/tm_${v}_$r.err || { tail -5 gpurun_out/tm_${v}_$r.err; exit 1; }
    python3 -c "
import json;d=json.loads(open('gpurun_out/tm_${v}_$r.json').read().splitlines()[-1]);h=d['host_ms_per_batch'];db=d.get('device_bound') or {}
print('$v r$r value %.2fM ms/step %.4f submit %.4f wait %.4f resident %.2fM device_bound %s' % (d['value']/1e6, d['ms_per_step'], h['submit'], h['wait'], (d.get('device_resident_txns_per_s') or 0)/1e6, db.get('ms_per_batch')))"
  done
done
