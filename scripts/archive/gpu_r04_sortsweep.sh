#!/bin/bash
# C2 sort: device-trace sections of one batch at a time, and isolated partition / bucket times
# over the average bucket size (FDBCS_SORT_BUCKET).
set -u
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/ss
timeout -k 10 200 python3 scripts/trace_c2.py 10 5000 c2 > gpurun_out/ss/trace_c2.txt 2>&1 || { tail gpurun_out/ss/trace_c2.txt; exit 1; }
grep -E "sort|bucket|partition" gpurun_out/ss/trace_c2.txt | tail -8
WORKLOAD=c2 WHICH=1,2 timeout -k 10 400 python3 scripts/kernel_sweep.py "FDBCS_SORT_BUCKET=32" "FDBCS_SORT_BUCKET=48" \
  "FDBCS_SORT_BUCKET=64" "FDBCS_SORT_BUCKET=96" "FDBCS_SORT_BUCKET=128" || exit 1
