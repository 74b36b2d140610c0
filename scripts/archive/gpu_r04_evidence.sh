#!/bin/bash
# Round evidence in one call: gpu_final.sh (tests, smoke, rocprof C1-C4 and C2 at 32768, PMC C2/C4),
# its rocprof and PMC summaries put in profiles/ on the box (the bench lines read them there), then
# the bench lines (gpu_benches.sh).  Copy the same files into the repo's profiles/ afterwards.
set -u
cd "$(dirname "$0")/.." || exit 1
T=${TAG:-r04g}
TAG=$T bash scripts/gpu_final.sh || exit 1
for w in c1 c2 c3 c4 c2_32768; do cp gpurun_out/$T/prof_$w/rocprof_*.json profiles/; done && cp gpurun_out/pmc/pmc_*.json profiles/ || exit 1
TAG=$T timeout -k 10 1000 bash scripts/gpu_benches.sh || exit 1
