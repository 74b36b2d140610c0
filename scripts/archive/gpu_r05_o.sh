#!/bin/bash
# addTransaction in the loop ("total"): add threads and their spin, same box.
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/r05o
mkdir -p $O
for cfg in "5 300" "0 0" "2 300" "8 300" "5 0" "8 0"; do
  set -- $cfg
  FDBCS_ADD_THREADS=$1 FDBCS_ADD_SPIN_US=$2 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 4 --warmup 5 \
    --profile-steps 0 --h2d-steps 0 --total-steps 60 --sync-steps 0 --hold-steps 0 --breakdown-steps 0 > $O/t_$1_$2.json 2> $O/t_$1_$2.err || exit 1
  echo "threads $1 spin $2: $(python3 -c "import json;d=json.load(open('$O/t_$1_$2.json'));print(round(d['total_txns_per_s']/1e6,2), {k: round(v,4) for k,v in d['total_host_ms_per_batch'].items()})")"
done
