#!/bin/bash
# Speculative slab loads in the bucket sort: isolated A/B against the previous commit (variant
# "head"), then the GPU sort tests and C2 bench lines of both.
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/r05g
mkdir -p $O
for v in head default head default; do
  L=""; [ $v != default ] && L="FDBCS_LIB=$PWD/foundationdb_amd/variants/libfdbcs_$v.so"
  env $L WORKLOAD=c2 WHICH=2 timeout -k 10 200 python3 scripts/kernel_sweep.py "FDBCS_SORT_BUCKET=64" > $O/s_$v.txt 2>&1 || { cat $O/s_$v.txt; exit 1; }
  echo "$v: $(tail -1 $O/s_$v.txt)"
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 280 --timeout-method thread -p no:cacheprovider tests -m gpu -k "sort or c2 or c3 or c4 or kat or random" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in head default; do
  L=""; [ $v != default ] && L="FDBCS_LIB=$PWD/foundationdb_amd/variants/libfdbcs_$v.so"
  env $L timeout -k 10 600 python bench.py --no-cpu-baseline > $O/bench_$v.json 2> $O/bench_$v.err || exit 1
done
