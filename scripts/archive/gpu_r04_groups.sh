#!/bin/bash
# Stage A's edge scan with and without write groups (FDBCS_WRITE_GROUPS=0) at C2 and C3: per-kernel times.
set -u
cd "$(dirname "$0")/.." || exit 1
for W in c2 c3; do
  WORKLOAD=$W ROUNDS=1 LIBS="grp:cur nogrp:cur:FDBCS_WRITE_GROUPS=0" timeout -k 10 900 bash scripts/gpu_ab_lib.sh 2>&1 | grep -E "value|EdgePair|edge_fill|resolve|combine|sort_bucket|check" || exit 1
done
