#!/bin/bash
# Sample-sort tuning sweep: parity tests at the default and at a sparse sample, then C2 bench lines
# for (FDBCS_SORT_BUCKET, FDBCS_SORT_SAMPLES) pairs. Stops at the first non-zero exit.
set -u
mkdir -p gpurun_out/sweep
timeout -k 10 600 python -m pytest tests -m gpu -q --timeout 300 -p no:cacheprovider > gpurun_out/sweep/tests_default.log 2>&1 || { tail -20 gpurun_out/sweep/tests_default.log >&2; exit 1; }
tail -1 gpurun_out/sweep/tests_default.log >&2
FDBCS_SORT_SAMPLES=3 timeout -k 10 600 python -m pytest tests -m gpu -q --timeout 300 -p no:cacheprovider > gpurun_out/sweep/tests_s3.log 2>&1 || { tail -20 gpurun_out/sweep/tests_s3.log >&2; exit 1; }
tail -1 gpurun_out/sweep/tests_s3.log >&2
for rep in 1 2; do
  for cfg in "0 0" "0 6" "0 5" "0 4" "160 6" "192 8" "192 5" "96 8"; do
    set -- $cfg
    FDBCS_SORT_BUCKET=$1 FDBCS_SORT_SAMPLES=$2 timeout -k 10 300 python bench.py --steps 60 --warmup 3 --no-cpu-baseline \
      > gpurun_out/sweep/b_${1}_${2}_$rep.json 2> gpurun_out/sweep/b_${1}_${2}_$rep.err || exit $?
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);p=d['phase_ms_per_batch'];print(sys.argv[2],round(d['value']/1e6,2),'M', 'sort',round(p['ms_sort']*1e3,1),'us')" gpurun_out/sweep/b_${1}_${2}_$rep.json "B=$1 S=$2 rep=$rep" >&2
  done
done
