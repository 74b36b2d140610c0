#!/bin/bash
# Round 5: isolated bucket-sort cost breakdown (FDBCS_SORT_EXP bits) and a HIP API + kernel trace of
# the pipelined C2 loop (host issue -> device start of every kernel, chain hand-offs).
set -u
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05e}
mkdir -p $O
WORKLOAD=c2 WHICH=2 timeout -k 10 400 python3 scripts/kernel_sweep.py "FDBCS_SORT_EXP=0" "FDBCS_SORT_EXP=2" \
  "FDBCS_SORT_EXP=4" "FDBCS_SORT_EXP=8" "FDBCS_SORT_EXP=14" "FDBCS_SORT_EXP=6" "FDBCS_SORT_BUCKET=32 FDBCS_SORT_EXP=4" \
  "FDBCS_SORT_BUCKET=32 FDBCS_SORT_EXP=14" > $O/sort_exp.txt 2>&1 || { cat $O/sort_exp.txt; exit 1; }
cat $O/sort_exp.txt >&2
timeout -k 10 300 rocprofv3 --hip-runtime-trace --kernel-trace --output-format csv -d $O/api -o run -- \
  python3 bench.py --workload c2 --steps 200 --warmup 20 --no-cpu-baseline --breakdown-steps 0 --sync-steps 0 \
  --resident-steps 0 --total-steps 0 --profile-steps 0 --hold-steps 0 --timing 0 > $O/api_bench.json 2> $O/api_bench.err || exit 1
A=$(find $O/api -name "*hip_api_trace.csv" | head -1)
K=$(find $O/api -name "*kernel_trace.csv" | head -1)
python3 scripts/launch_gaps.py $A $K > $O/launch_gaps.txt 2>&1
python3 scripts/crit_path.py $K > $O/crit.txt 2>&1
cat $O/launch_gaps.txt >&2
gzip -f $A $K
