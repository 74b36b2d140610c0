#!/bin/bash
# A/B kernel timing: one rocprofv3 kernel-trace run of a short bench per variant.
# Usage: VARIANTS="base: alt:FDBCS_SORT_ALG=1" bash scripts/gpu_kprof.sh
# Each variant is name:ENV=V[,ENV=V...]; summaries land in gpurun_out/kprof/<name>/.
set -u
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
for v in ${VARIANTS:-base:}; do
  name=${v%%:*}
  envs=${v#*:}
  mkdir -p gpurun_out/kprof/$name
  (
    IFS=','; for e in $envs; do [ -n "$e" ] && export "$e"; done
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kprof/$name -o run -- \
      python3 bench.py --steps ${STEPS:-30} --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} \
      > gpurun_out/kprof/$name/bench.json 2> gpurun_out/kprof/$name/bench.err
  )
  rc=$?
  echo "== $name ($envs) rc=$rc" >&2
  [ $rc -ne 0 ] && exit $rc
  python3 -c "import json;d=json.load(open('gpurun_out/kprof/$name/bench.json'));print('value %.3fM txns/s ms/step %.4f'%(d['value']/1e6,d['ms_per_step']))" >&2
  python3 scripts/prof_summary.py gpurun_out/kprof/$name/run_kernel_stats.csv >&2
done
