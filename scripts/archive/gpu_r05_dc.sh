#!/bin/bash
# C4: the delta-tier check after the base-tier check on cstream (FDBCS_DELTA_ON_C=1) against heading
# half X (default): parity-checked line, then same-box A/B.
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/${TAG:-r05dc}
mkdir -p $O
FDBCS_DELTA_ON_C=1 timeout -k 10 600 python bench.py --workload c4 --cpu-seconds 20 > $O/bench_c4.json 2> $O/bench_c4.err || exit 1
python3 -c "import json;d=json.load(open('$O/bench_c4.json'));print('c4 delta_on_c', d['value'], d['parity'])"
BENCH_ARGS="--workload c4 --steps 60 --no-cpu-baseline --breakdown-steps 0 --sync-steps 0 --h2d-steps 0 --total-steps 0" \
VARIANTS="x:FDBCS_DELTA_ON_C=0 c:FDBCS_DELTA_ON_C=1" ROUNDS=3 timeout -k 10 900 bash scripts/gpu_ab_env.sh || exit 1
