#!/bin/bash
# Per-dispatch SQ counters of every kernel in a short bench run (instruction mix, wave cycles).
set -u
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/pmck
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmck/counters.txt 2>&1 || true
timeout -s KILL 120 rocprofv3 --pmc ${COUNTERS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM SQ_BUSY_CYCLES} \
  --output-format csv -d gpurun_out/pmck/run -o run -- \
  python3 bench.py --steps 12 --warmup 2 --no-cpu-baseline --breakdown-steps 0 > gpurun_out/pmck/bench.json 2> gpurun_out/pmck/bench.err
echo "pmc rc=$?" >&2
