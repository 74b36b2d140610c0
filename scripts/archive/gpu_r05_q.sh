#!/bin/bash
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/r05q
mkdir -p $O
timeout -k 10 400 python3 scripts/trace_c2.py 4 5000 c4 > $O/trace_c4.txt 2>&1 || { tail $O/trace_c4.txt; exit 1; }
grep -E "bucket" $O/trace_c4.txt | tail -6
