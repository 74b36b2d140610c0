#!/bin/bash
# addTransaction cost sweep (threads), C2 and C4 batches, then a C2 bench line.
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/r05add2
mkdir -p $O
for wl in c2 c4; do
  for th in 0 2 5 8; do
    FDBCS_ADD_PROFILE=1 FDBCS_ADD_THREADS=$th timeout -k 5 120 python scripts/add_sweep.py $wl >> $O/sweep.txt 2>&1 || { echo "fail $wl $th" >> $O/sweep.txt; exit 1; }
  done
done
cat $O/sweep.txt
timeout -k 10 600 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err
