#!/bin/bash
# HBM traffic of the dominant kernel from PMC counters: FETCH_SIZE and WRITE_SIZE in separate passes
# (TCC slots: FETCH_SIZE costs 3, WRITE_SIZE 2; MI355X_MICROARCH.md rocprofv3 PMC slots).
set -u
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc/$c -o run -- \
    python3 bench.py --workload ${WORKLOAD:-c2} --steps ${STEPS:-40} --warmup 2 --no-cpu-baseline > gpurun_out/pmc/$c.json 2> gpurun_out/pmc/$c.err
  rc=$?
  echo "pmc $c rc=$rc" >&2
  [ $rc -ne 0 ] && exit $rc
done
python3 scripts/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc/pmc_traffic_${WORKLOAD:-c2}.json
cat gpurun_out/pmc/pmc_traffic_${WORKLOAD:-c2}.json >&2
