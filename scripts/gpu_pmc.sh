#!/bin/bash
# HBM traffic of every pipeline kernel from PMC counters: FETCH_SIZE and WRITE_SIZE in separate
# passes (TCC slots: FETCH_SIZE costs 3, WRITE_SIZE 2; MI355X_MICROARCH.md rocprofv3 PMC slots),
# on the bench's own configuration.  Output: gpurun_out/pmc/pmc_<workload>_<txns>_<history>.json
# (copy to profiles/, where bench.py reads the dominant kernel's `traffic`).
set -u
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
W=${WORKLOAD:-c2}
case $W in c1) TX=2500; HI=0 ;; c4) TX=5000; HI=50000000 ;; *) TX=5000; HI=5000000 ;; esac
mkdir -p gpurun_out/pmc
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc/$c -o run -- \
    python3 bench.py --workload $W --steps ${STEPS:-24} --warmup 2 --no-cpu-baseline --total-steps 0 \
    --breakdown-steps 0 --sync-steps 0 --hold-steps 0 > gpurun_out/pmc/$c.json 2> gpurun_out/pmc/$c.err
  rc=$?
  echo "pmc $c rc=$rc" >&2
  [ $rc -ne 0 ] && exit $rc
done
GIT_HEAD=${GIT_HEAD:-} python3 scripts/pmc_summary.py gpurun_out/pmc $W $TX $HI > gpurun_out/pmc/pmc_${W}_${TX}_${HI}.json
rm -rf gpurun_out/pmc/FETCH_SIZE gpurun_out/pmc/WRITE_SIZE
head -c 1500 gpurun_out/pmc/pmc_${W}_${TX}_${HI}.json >&2
