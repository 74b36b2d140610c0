#!/bin/bash
# Headline on HBM-resident batches: multi-rank tests, C2 bench line.
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/r05m
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 290 --timeout-method thread -p no:cacheprovider tests/test_gpu_multi.py > $O/multi.log 2>&1 || { tail -30 $O/multi.log; exit 1; }
tail -1 $O/multi.log
timeout -k 10 600 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err || exit 1
