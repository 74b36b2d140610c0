#!/bin/bash
# Same-box A/B of engine builds and knobs: each entry of LIBS is label:lib[:ENV=V,ENV=V] with lib a
# name under foundationdb_amd/variants/libfdbcs_<lib>.so or "cur" (the in-tree library).  ROUNDS
# interleaved rocprofv3 kernel-trace runs of a short bench of WORKLOAD per entry; per-kernel averages
# and the bench value side by side.  Output gpurun_out/ablib/.
set -u
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
W=${WORKLOAD:-c2}
O=gpurun_out/ablib
mkdir -p $O
labels=""
for r in $(seq 1 ${ROUNDS:-2}); do
  for e in ${LIBS}; do
    label=${e%%:*}; rest=${e#*:}; libn=${rest%%:*}; envs=""
    [ "$rest" != "$libn" ] && envs=${rest#*:}
    [ $r -eq 1 ] && labels="$labels $label"
    lib=foundationdb_amd/variants/libfdbcs_$libn.so
    [ "$libn" = "cur" ] && lib=foundationdb_amd/libfdbcs.so
    d=$O/${label}_${W}_$r
    (
      IFS=','; for x in $envs; do [ -n "$x" ] && export "$x"; done; unset IFS
      FDBCS_LIB=$PWD/$lib timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- \
        python3 bench.py --workload $W --steps ${STEPS:-40} --warmup 3 --no-cpu-baseline --breakdown-steps 0 \
        --sync-steps 0 --total-steps 0 --h2d-steps 0 ${BENCH_ARGS:-} > $d.json 2> $d.err
    ) || { echo "$label failed"; tail -5 $d.err; exit 1; }
    find $d -name "*kernel_trace.csv" -delete
  done
done
python3 scripts/ab_table.py $O $W "$labels" ${ROUNDS:-2}
