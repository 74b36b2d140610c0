#!/bin/bash
# C4 over 200 timed batches under rocprofv3: what its compactions cost.
set -u
cd "$(dirname "$0")/.." || exit 1
WORKLOAD=c4 OUT=gpurun_out/r05c4c STEPS=200 timeout -k 10 700 bash scripts/gpu_profile.sh || exit 1
cat gpurun_out/r05c4c/summary.txt | cut -c1-110
