#!/bin/bash
# Directory slot budget A/B at C4 (default 2^19 vs 2^20 vs first two bytes) and C2 (default), then
# rocprof kernel tables of C2/C3/C4 at the current build.
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/${TAG:-r05u}
mkdir -p $O
WORKLOAD=c4 WHICH=0 timeout -k 10 400 python3 scripts/kernel_sweep.py "FDBCS_DIR_RANK=1" "FDBCS_DIR_BITS=20" "FDBCS_DIR_BITS=17" "FDBCS_DIR_RANK=0" > $O/sweep_c4.txt 2>&1 || { cat $O/sweep_c4.txt; exit 1; }
tail -4 $O/sweep_c4.txt
WORKLOAD=c2 WHICH=0 timeout -k 10 400 python3 scripts/kernel_sweep.py "FDBCS_DIR_RANK=1" "FDBCS_DIR_RANK=0" > $O/sweep_c2.txt 2>&1 || { cat $O/sweep_c2.txt; exit 1; }
tail -2 $O/sweep_c2.txt
for w in c2 c3 c4; do
  WORKLOAD=$w OUT=$O/prof_$w timeout -k 10 700 bash scripts/gpu_profile.sh || exit 1
  head -16 $O/prof_$w/summary.txt
done
