#!/bin/bash
# Isolated k_sort_bucket at C2 with parts switched off (FDBCS_SORT_EXP bits: 2 writes, 4 network, 8 prologue).
set -u
cd "$(dirname "$0")/.." || exit 1
WORKLOAD=c2 WHICH=2 timeout -k 10 400 python3 scripts/kernel_sweep.py "FDBCS_SORT_EXP=0" "FDBCS_SORT_EXP=2" "FDBCS_SORT_EXP=4" \
  "FDBCS_SORT_EXP=8" "FDBCS_SORT_EXP=6" "FDBCS_SORT_EXP=12" "FDBCS_SORT_EXP=14" || exit 1
