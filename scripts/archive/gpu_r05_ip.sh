#!/bin/bash
# Host cost per replayed record (FDBCS_ISSUE_PROFILE) in the C2 timed loop.
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/${TAG:-r05ip}
mkdir -p $O
FDBCS_ISSUE_PROFILE=1 timeout -k 10 300 python bench.py --workload c2 --steps 200 --warmup 10 --no-cpu-baseline --breakdown-steps 0 \
  --sync-steps 0 --h2d-steps 0 --total-steps 0 --profile-steps 0 --hold-steps 0 > $O/bench.json 2> $O/bench.err || exit 1
grep "issue profile" $O/bench.err
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], d['host_ms_per_batch'])"
