#!/bin/bash
# C4: isolated base / delta check launches (directory code), and split check vs one check A/B.
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/${TAG:-r05x}
mkdir -p $O
WORKLOAD=c4 WHICH=0,3,4 timeout -k 10 400 python3 scripts/kernel_sweep.py "FDBCS_DIR_RANK=1" "FDBCS_DIR_RANK=0" > $O/sweep_c4.txt 2>&1 || { cat $O/sweep_c4.txt; exit 1; }
tail -2 $O/sweep_c4.txt
BENCH_ARGS="--workload c4 --steps 60 --no-cpu-baseline --breakdown-steps 0 --sync-steps 0 --h2d-steps 0 --total-steps 0" \
  VARIANTS="split2:FDBCS_SPLIT_CHECK=2 split0:FDBCS_SPLIT_CHECK=0" ROUNDS=2 timeout -k 10 900 bash scripts/gpu_ab_env.sh || exit 1
