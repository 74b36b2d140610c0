#!/bin/bash
# Isolated whole-base index rebuild (k_epilogue<true>) on 5M and 50M-boundary C2 histories.
set -u
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05j
mkdir -p $O
for h in 5000000 20000000; do
  HISTORY=$h timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/epi_$h -o run -- python3 scripts/epi_bench.py > $O/epi_$h.log 2>&1 || { tail $O/epi_$h.log; exit 1; }
  S=$(find $O/epi_$h -name "*kernel_stats.csv" | head -1)
  python3 scripts/prof_summary.py $S | head -8 > $O/epi_$h.txt
  echo "history $h"; cat $O/epi_$h.txt
  find $O/epi_$h -name "*kernel_trace.csv" -delete
done
