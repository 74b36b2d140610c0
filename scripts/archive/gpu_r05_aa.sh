#!/bin/bash
# Wide k_seg_prep tiles of 511 segments (1024 threads) at 32768-txn C2 batches: the 32768-txn
# tests, rocprof, bench line.
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/${TAG:-r05aa}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 280 --timeout-method thread -p no:cacheprovider tests/test_gpu_fullsize.py -m gpu -k "32768 or max" > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
WORKLOAD=c2 OUT=$O/prof_c2_32768 STEPS=24 BENCH_ARGS="--txns 32768" timeout -k 10 600 bash scripts/gpu_profile.sh || exit 1
grep seg_prep $O/prof_c2_32768/summary.txt
timeout -k 10 600 python bench.py --workload c2 --txns 32768 --cpu-seconds 5 > $O/bench.json 2> $O/bench.err || exit 1
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['h2d_inclusive_txns_per_s'],d['device_bound']['ms_per_batch'],d['parity']['mismatched_batches'],d['parity']['batches_checked'])"
