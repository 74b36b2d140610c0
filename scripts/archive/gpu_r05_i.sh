#!/bin/bash
# Wait-spin stream queries rate-limited: C2 bench A/B on one box (query every 4096 spins vs every
# 2 ms), each with the host spans (no profiler), then the host-span summary of each.
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/r05i
mkdir -p $O
rm -f $O/host_*.csv
for rep in 1 2; do
  for q in 0 2; do
    FDBCS_WAIT_QUERY_MS=$q FDBCS_HOST_TRACE=$PWD/$O/host_q${q}_$rep timeout -k 10 600 python bench.py --no-cpu-baseline \
      > $O/bench_q${q}_$rep.json 2> $O/bench_q${q}_$rep.err || exit 1
    echo "q=$q rep=$rep $(python3 -c "import json;d=json.load(open('$O/bench_q${q}_$rep.json'));print(round(d['value']/1e6,2), d['host_ms_per_batch'])")"
  done
done
