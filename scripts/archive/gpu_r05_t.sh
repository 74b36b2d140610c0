#!/bin/bash
# Directory code by value ranges (ALU only): directory tests, GPU suite, isolated read-check A/B
# (code vs first two bytes; slot budgets) for C4/C2/C3, C4/C2 benches.
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/${TAG:-r05t}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py -m gpu -k "directory" > $O/dir_tests.log 2>&1 || { tail -30 $O/dir_tests.log; exit 1; }
tail -1 $O/dir_tests.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 280 --timeout-method thread -p no:cacheprovider tests -m gpu > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
WORKLOAD=c4 WHICH=0 timeout -k 10 400 python3 scripts/kernel_sweep.py "FDBCS_DIR_RANK=1" "FDBCS_DIR_RANK=0" "FDBCS_DIR_BITS=18" > $O/sweep_c4.txt 2>&1 || { cat $O/sweep_c4.txt; exit 1; }
tail -3 $O/sweep_c4.txt
for w in c2 c3; do
  WORKLOAD=$w WHICH=0 timeout -k 10 400 python3 scripts/kernel_sweep.py "FDBCS_DIR_RANK=1" "FDBCS_DIR_RANK=0" "FDBCS_DIR_BITS=16" > $O/sweep_$w.txt 2>&1 || { cat $O/sweep_$w.txt; exit 1; }
  tail -3 $O/sweep_$w.txt
done
for w in c4 c2; do
  timeout -k 10 600 python bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || exit 1
  python3 -c "import json;d=json.load(open('$O/bench_$w.json'));print('$w',d['value'],d.get('h2d_inclusive_txns_per_s'),d['parity'])"
done
