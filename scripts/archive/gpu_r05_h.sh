#!/bin/bash
# Host spans (FDBCS_HOST_TRACE) + rocprofv3 kernel trace of the pipelined C2 loop: when each chain
# head was issued against when it ran.  Also the plain bench line of this build.
set -u
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05h}
mkdir -p $O
rm -f $O/host.*.csv
FDBCS_HOST_TRACE=$PWD/$O/host timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- \
  python3 bench.py --workload ${W:-c2} --steps 300 --warmup 20 --no-cpu-baseline --breakdown-steps 0 --sync-steps 0 \
  --resident-steps 0 --total-steps 0 --profile-steps 0 --hold-steps 0 --timing 0 ${BENCH_ARGS:-} > $O/kt_bench.json 2> $O/kt_bench.err || exit 1
K=$(find $O/kt -name "*kernel_trace.csv" | head -1)
H=$(ls $O/host.*.csv | head -1)
python3 scripts/host_trace.py $H $K > $O/host_trace.txt 2>&1
cat $O/host_trace.txt >&2
gzip -f $K $H
timeout -k 10 600 python bench.py --workload ${W:-c2} > $O/bench.json 2> $O/bench.err || exit 1
