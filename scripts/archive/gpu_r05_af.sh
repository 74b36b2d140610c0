#!/bin/bash
# Edge fill step table from EdgePairScan (plus the staged operands and range lists):
# cooperative layout back for small batches: GPU suite, rocprof C3 / C2, bench C3 / C2.
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/${TAG:-r05af}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 280 --timeout-method thread -p no:cacheprovider tests -m gpu > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for w in c3 c2; do
  WORKLOAD=$w OUT=$O/prof_$w timeout -k 10 600 bash scripts/gpu_profile.sh || exit 1
  grep -E "edge_fill|EdgePairScan|seg_prep|sort_bucket|resolve<" $O/prof_$w/summary.txt
done
for w in c3 c2; do
  timeout -k 10 600 python bench.py --workload $w --cpu-seconds 5 > $O/bench_$w.json 2> $O/bench_$w.err || exit 1
  python3 -c "import json;d=json.load(open('$O/bench_$w.json'));print('$w',d['value'],d['h2d_inclusive_txns_per_s'],d['device_bound']['ms_per_batch'],d['parity']['mismatched_batches'],d['parity']['batches_checked'])"
done
