#!/bin/bash
# Second sample-sort sweep around (160, 6): C2 lines, then C3/C4 default vs (160, 6).
set -u
mkdir -p gpurun_out/sweep2
FDBCS_SORT_BUCKET=160 FDBCS_SORT_SAMPLES=6 timeout -k 10 600 python -m pytest tests -m gpu -q --timeout 300 -p no:cacheprovider > gpurun_out/sweep2/tests_160_6.log 2>&1 || { tail -20 gpurun_out/sweep2/tests_160_6.log >&2; exit 1; }
tail -1 gpurun_out/sweep2/tests_160_6.log >&2
run() {  # workload bucket samples rep
  FDBCS_SORT_BUCKET=$2 FDBCS_SORT_SAMPLES=$3 timeout -k 10 300 python bench.py --workload $1 --steps 60 --warmup 3 --no-cpu-baseline \
    > gpurun_out/sweep2/b_$1_$2_$3_$4.json 2> gpurun_out/sweep2/b_$1_$2_$3_$4.err || exit $?
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2],round(d['value']/1e6,2),'M')" gpurun_out/sweep2/b_$1_$2_$3_$4.json "$1 B=$2 S=$3 rep=$4" >&2
}
for rep in 1 2 3; do
  for cfg in "0 0" "160 6" "144 6" "176 6" "160 7" "160 5" "144 7"; do set -- $cfg; run c2 $1 $2 $rep; done
done
for rep in 1 2; do
  for cfg in "0 0" "160 6"; do set -- $cfg; run c3 $1 $2 $rep; run c4 $1 $2 $rep; done
done
