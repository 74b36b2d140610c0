#!/bin/bash
# Randomized parity stress (scripts/stress_parity.py) on the final build.
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/${TAG:-r05stress}
mkdir -p $O
timeout -k 10 $(( ${SECS:-240} + 60 )) python3 -u scripts/stress_parity.py ${SECS:-240} ${SEED:-1} > $O/stress.log 2>&1
rc=$?
tail -3 $O/stress.log
exit $rc
