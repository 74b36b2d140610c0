#!/bin/bash
# Short A/B experiments on one box: C2 bench with the default engine and with each knob setting
# given as an argument ("FDBCS_X=1 FDBCS_Y=2"); one JSON line per run in gpurun_out/exp_<i>.json.
set -u
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
i=0
for knobs in "" "$@"; do
  env $knobs timeout -k 10 240 python bench.py --workload ${WL:-c2} --steps ${STEPS:-40} --warmup 3 \
    --total-steps 0 --breakdown-steps 0 --cpu-seconds 5 ${BENCH_ARGS:-} \
    > gpurun_out/exp_$i.json 2> gpurun_out/exp_$i.err || { tail -5 gpurun_out/exp_$i.err; exit 1; }
  echo "== [$knobs]" >> gpurun_out/exp_summary.txt
  python scripts/bench_summary.py gpurun_out/exp_$i.json | head -8 >> gpurun_out/exp_summary.txt
  i=$((i+1))
done
