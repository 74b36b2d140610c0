#!/bin/bash
# Anatomy of the device-bound (hold) pass: kernel trace of a bench run whose hold pass queues 64
# batches; per-chain busy fractions.
set -u
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05n}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- \
  python3 bench.py --workload ${W:-c2} --steps 4 --warmup 20 --no-cpu-baseline --breakdown-steps 0 --sync-steps 0 \
  --h2d-steps 0 --total-steps 0 --profile-steps 0 --hold-steps ${HOLD:-64} --timing 0 > $O/bench.json 2> $O/bench.err || exit 1
K=$(find $O/kt -name "*kernel_trace.csv" | head -1)
python3 scripts/hold_trace.py $K > $O/hold.txt 2>&1; cat $O/hold.txt
gzip -f $K
