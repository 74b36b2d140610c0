#!/bin/bash
# Sort counter layout A/B (isolated partition and bucket-sort times): one 128-byte line per bucket
# (stride 16, the default build) against dense counters (stride 2 / 4 variants).
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/r05f
mkdir -p $O
for v in default cnt2 cnt4; do
  L=""; [ $v != default ] && L="FDBCS_LIB=$PWD/foundationdb_amd/variants/libfdbcs_$v.so"
  for b in 64 32; do
    env $L WORKLOAD=c2 WHICH=1,2 timeout -k 10 200 python3 scripts/kernel_sweep.py "FDBCS_SORT_BUCKET=$b" > $O/s_${v}_$b.txt 2>&1 || { cat $O/s_${v}_$b.txt; exit 1; }
    echo "$v bucket $b: $(tail -1 $O/s_${v}_$b.txt)"
    env $L WORKLOAD=c3 WHICH=1,2 timeout -k 10 200 python3 scripts/kernel_sweep.py "FDBCS_SORT_BUCKET=$b" > $O/s3_${v}_$b.txt 2>&1 || { cat $O/s3_${v}_$b.txt; exit 1; }
    echo "  c3 $v bucket $b: $(tail -1 $O/s3_${v}_$b.txt)"
  done
done
