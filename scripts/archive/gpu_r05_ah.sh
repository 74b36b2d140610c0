#!/bin/bash
# Resolution rounds reset only the group starts' minima: GPU suite, rocprof C3, C3 trace, bench C3.
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/${TAG:-r05ah}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 280 --timeout-method thread -p no:cacheprovider tests -m gpu > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
WORKLOAD=c3 OUT=$O/prof_c3 timeout -k 10 600 bash scripts/gpu_profile.sh || exit 1
grep -E "edge_fill|resolve|combine" $O/prof_c3/summary.txt
timeout -k 10 400 python3 scripts/trace_c2.py 4 5000 c3 > $O/trace_c3.txt 2>&1 || { tail -5 $O/trace_c3.txt; exit 1; }
grep "resolve pre-pass" $O/trace_c3.txt
timeout -k 10 600 python bench.py --workload c3 --cpu-seconds 5 > $O/bench_c3.json 2> $O/bench_c3.err || exit 1
python3 -c "import json;d=json.load(open('$O/bench_c3.json'));print('c3',d['value'],d['h2d_inclusive_txns_per_s'],d['parity']['mismatched_batches'],d['parity']['batches_checked'])"
