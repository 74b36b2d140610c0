#!/bin/bash
# Edge fill with staged per-range data and run-aggregated slot atomics: edge-heavy parity tests,
# GPU suite, C3/C2 rocprof tables, C4 directory default check time.
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/${TAG:-r05v}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_fullsize.py tests/test_gpu_parity.py -m gpu -k "chain or c3 or random or group or scenario" > $O/edge_tests.log 2>&1 || { tail -30 $O/edge_tests.log; exit 1; }
tail -1 $O/edge_tests.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 280 --timeout-method thread -p no:cacheprovider tests -m gpu > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for w in c3 c2; do
  WORKLOAD=$w OUT=$O/prof_$w timeout -k 10 700 bash scripts/gpu_profile.sh || exit 1
  head -14 $O/prof_$w/summary.txt
  python3 -c "import json;d=json.load(open('$O/prof_$w/bench.json'));print('$w',d['value'],d['parity']['mismatched_batches'])"
done
WORKLOAD=c4 WHICH=0 timeout -k 10 400 python3 scripts/kernel_sweep.py "FDBCS_DIR_RANK=1" "FDBCS_DIR_BITS=16" > $O/sweep_c4.txt 2>&1 || { cat $O/sweep_c4.txt; exit 1; }
tail -2 $O/sweep_c4.txt
timeout -k 10 400 python3 scripts/trace_c2.py 4 5000 c3 > $O/trace_c3.txt 2>&1 || { tail -5 $O/trace_c3.txt; exit 1; }
tail -40 $O/trace_c3.txt
