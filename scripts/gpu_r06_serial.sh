#!/bin/bash
# Round 6: every pipeline kernel's device time without the other chains beside it (FDBCS_SERIAL=1:
# one stream, each kernel alone on the chip), rocprofv3 kernel-trace of C2, C3 and C4.
set -u
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06serial}
for w in ${WLS:-c2 c3 c4}; do
  FDBCS_SERIAL=1 WORKLOAD=$w OUT=$O/prof_$w STEPS=24 timeout -k 10 700 bash scripts/gpu_profile.sh || exit $?
  head -22 $O/prof_$w/summary.txt >&2
done
