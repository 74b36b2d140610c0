#!/bin/bash
# C4 anatomy: device trace of the sort sections and isolated check / sort kernel times.
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/r05p
mkdir -p $O
timeout -k 10 400 python3 scripts/trace_c2.py 6 5000 c4 > $O/trace_c4.txt 2>&1 || { tail $O/trace_c4.txt; exit 1; }
grep -E "bucket|partition" $O/trace_c4.txt | tail -4
WORKLOAD=c4 WHICH=1,2,3,4 timeout -k 10 500 python3 scripts/kernel_sweep.py "FDBCS_SORT_EXP=0" "FDBCS_SORT_EXP=1" > $O/c4_sweep.txt 2>&1 || { cat $O/c4_sweep.txt; exit 1; }
cat $O/c4_sweep.txt
