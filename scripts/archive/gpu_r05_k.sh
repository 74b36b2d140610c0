#!/bin/bash
# Whole-base index rebuild with its level-2 / level-3 atomics removed (timing experiment only).
set -u
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05k
mkdir -p $O
for v in epi0 epi2 epi3; do
  FDBCS_LIB=$PWD/foundationdb_amd/variants/libfdbcs_$v.so HISTORY=5000000 timeout -k 10 300 rocprofv3 --kernel-trace --stats \
    --output-format csv -d $O/$v -o run -- python3 scripts/epi_bench.py > $O/$v.log 2>&1 || { tail $O/$v.log; exit 1; }
  S=$(find $O/$v -name "*kernel_stats.csv" | head -1)
  echo "$v: $(python3 scripts/prof_summary.py $S | grep epilogue)"
  find $O/$v -name "*kernel_trace.csv" -delete
done
