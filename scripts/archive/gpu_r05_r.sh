#!/bin/bash
# Batched serial tie ranking, fewer held prefix registers: GPU suite, isolated sort times, C2/C4 benches.
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/${TAG:-r05r}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 280 --timeout-method thread -p no:cacheprovider tests -m gpu > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for w in c2 c4; do
  WORKLOAD=$w WHICH=1,2 timeout -k 10 400 python3 scripts/kernel_sweep.py "FDBCS_SORT_EXP=0" > $O/sweep_$w.txt 2>&1 || { cat $O/sweep_$w.txt; exit 1; }
  tail -1 $O/sweep_$w.txt
done
timeout -k 10 400 python3 scripts/trace_c2.py 4 5000 c4 > $O/trace_c4.txt 2>&1 && grep -E "tie runs" $O/trace_c4.txt | tail -1
for w in c2 c4; do
  timeout -k 10 600 python bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || exit 1
done
