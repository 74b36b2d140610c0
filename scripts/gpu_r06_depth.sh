#!/bin/bash
# Round 6: the check reading two previous batches' union segments (FDBCS_PREV_DEPTH 2, the new
# default) against one (1, rounds 3-6): GPU suite, randomized stress, then same-box bench A/B.
set -u
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06depth}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log >&2; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 scripts/stress_parity.py ${STRESS_S:-90} 41001 > $O/stress.log 2>&1
rc=$?; tail -2 $O/stress.log >&2; [ $rc -ne 0 ] && exit $rc
TAG=${TAG:-r06depth}_ab VARIANTS="d1:FDBCS_PREV_DEPTH=1 d2:FDBCS_PREV_DEPTH=2" WLS="${WLS:-c2 c3 c4}" ROUNDS=${ROUNDS:-2} bash scripts/gpu_r06_ab.sh
