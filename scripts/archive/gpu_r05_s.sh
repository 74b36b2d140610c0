#!/bin/bash
# Rank-code radix directory: directory tests first, GPU suite, isolated read-check A/B (rank vs
# first two bytes) for C4/C2/C3, C4/C2 benches.
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/${TAG:-r05s}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py -m gpu -k "directory" > $O/dir_tests.log 2>&1 || { tail -30 $O/dir_tests.log; exit 1; }
tail -1 $O/dir_tests.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 280 --timeout-method thread -p no:cacheprovider tests -m gpu > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for w in c4 c2 c3; do
  WORKLOAD=$w WHICH=0 timeout -k 10 400 python3 scripts/kernel_sweep.py "FDBCS_DIR_RANK=1" "FDBCS_DIR_RANK=0" > $O/sweep_$w.txt 2>&1 || { cat $O/sweep_$w.txt; exit 1; }
  tail -2 $O/sweep_$w.txt
done
for w in c4 c2; do
  timeout -k 10 600 python bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || exit 1
  python3 -c "import json;d=json.load(open('$O/bench_$w.json'));print('$w',d['value'],d.get('h2d_inclusive_txns_per_s'),d['conflicts_match'] if 'conflicts_match' in d else '')"
done
