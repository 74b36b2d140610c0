#!/bin/bash
# Copy a round-evidence call's outputs (gpu_r04_evidence.sh, TAG) from gpurun_out/ into profiles/.
set -eu
cd "$(dirname "$0")/.."
T=${TAG:-r04g}
O=gpurun_out/$T
for w in c1 c2 c3 c4 c2_32768; do cp $O/prof_$w/rocprof_*.json profiles/; done
cp gpurun_out/pmc/pmc_*.json profiles/
for w in c1 c2 c3 c4 c2_32768; do
  cp $O/prof_$w/summary.txt profiles/${T}_kernel_stats_$w.txt
  [ -f $O/prof_$w/timeline.txt ] && cp $O/prof_$w/timeline.txt profiles/${T}_timeline_$w.txt
done
cp $O/gpu_tests.log profiles/${T}_gpu_tests.log
cp $O/smoke.log profiles/${T}_smoke.log
for f in $O/bench_*.json; do cp $f profiles/${T}_$(basename $f); done
ls profiles | grep $T
