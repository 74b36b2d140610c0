#!/bin/bash
# Same-box A/B of engine builds: for each NAME in LIBS (foundationdb_amd/variants/libfdbcs_<NAME>.so,
# "cur" = the in-tree library), ROUNDS interleaved rocprofv3 kernel-trace runs of a short bench of
# WORKLOAD; per-kernel averages and the bench value side by side.  Output gpurun_out/ablib/.
set -u
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
W=${WORKLOAD:-c2}
O=gpurun_out/ablib
mkdir -p $O
for r in $(seq 1 ${ROUNDS:-2}); do
  for n in ${LIBS}; do
    lib=foundationdb_amd/variants/libfdbcs_$n.so
    [ "$n" = "cur" ] && lib=foundationdb_amd/libfdbcs.so
    d=$O/${n}_${W}_$r
    FDBCS_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- \
      python3 bench.py --workload $W --steps ${STEPS:-40} --warmup 3 --no-cpu-baseline --breakdown-steps 0 \
      --sync-steps 0 --total-steps 0 --resident-steps 0 ${BENCH_ARGS:-} > $d.json 2> $d.err || { echo "$n failed"; tail -5 $d.err; exit 1; }
    find $d -name "*kernel_trace.csv" -delete
  done
done
python3 scripts/ab_table.py $O $W "${LIBS}" ${ROUNDS:-2}
