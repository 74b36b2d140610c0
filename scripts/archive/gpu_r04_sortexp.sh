#!/bin/bash
# Isolated sort costs at C2/C3: partition (1) and bucket (2), with the tie ranking (exp 1) or the
# position writes (exp 2) skipped.
set -u
cd "$(dirname "$0")/.." || exit 1
for W in c2 c3; do
WORKLOAD=$W WHICH=0,1,2 timeout -k 10 300 python3 scripts/kernel_sweep.py "base" "FDBCS_SORT_EXP=1" "FDBCS_SORT_EXP=2" "FDBCS_SORT_EXP=3" || exit 1
done
