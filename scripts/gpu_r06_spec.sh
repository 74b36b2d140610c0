#!/bin/bash
# Round 6: the bucket sort's speculative slab loads (FDBCS_SPEC_SLOTS 0 / 40 / 80, variant builds):
# same-box rocprof A/B on C2 and C4, then PMC bytes of the sort kernels per variant on C2.
set -u
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/ablib
for w in c2 c4; do
  WORKLOAD=$w LIBS="s80:s80 s40:s40 s0:s0" ROUNDS=2 STEPS=40 timeout -k 10 900 bash scripts/gpu_ab_lib.sh > gpurun_out/ablib/spec_$w.txt 2>&1 || exit $?
  head -14 gpurun_out/ablib/spec_$w.txt >&2
done
for v in s80 s0; do
  FDBCS_LIB=$PWD/foundationdb_amd/variants/libfdbcs_$v.so WORKLOAD=c2 timeout -k 10 400 bash scripts/gpu_pmc.sh > /dev/null 2>&1 || exit $?
  mkdir -p gpurun_out/ablib/pmc_$v && cp gpurun_out/pmc/pmc_c2_5000_5000000.json gpurun_out/ablib/pmc_$v/
  python3 -c "
import json; d=json.load(open('gpurun_out/ablib/pmc_$v/pmc_c2_5000_5000000.json'))
print('$v', {k: (round(d['bytes_per_launch'][k]/1e6,2), round(d['model_bytes_per_launch'][k]/1e6,2)) for k in d['bytes_per_launch'] if 'sort' in k})" >&2
done
