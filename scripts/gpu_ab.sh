#!/bin/bash
# GPU tests (unless SKIP_TESTS=1), then the bench under several settings: each AB_i is
# "ENV=val ... -- bench args" (ENV part optional), e.g. AB_1="FDBCS_UPLOAD=dma --" AB_2="-- --timing 0".
set -u
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/ab
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 -p no:cacheprovider ${PYTEST_ARGS:-} > gpurun_out/ab/tests.log 2>&1
  rc=$?; tail -3 gpurun_out/ab/tests.log >&2; [ $rc -ne 0 ] && exit $rc
fi
for i in 1 2 3 4 5 6; do
  var="AB_$i"; spec="${!var:-}"; [ -z "$spec" ] && continue
  envs="${spec%%--*}"; args="${spec#*--}"
  env $envs timeout -k 10 300 python3 bench.py --steps 30 --warmup 3 $args > gpurun_out/ab/bench_$i.json 2> gpurun_out/ab/bench_$i.err || exit $?
  python3 - "$i" "$spec" <<'PY' >&2
import json, sys
d = json.load(open(f"gpurun_out/ab/bench_{sys.argv[1]}.json"))
k = d.get("kernels", {})
print(sys.argv[2], "| value %.2fM resident %s total %s" % (d["value"] / 1e6, d.get("device_resident_txns_per_s"), d.get("total_txns_per_s")),
      "| host", {a: round(b, 3) for a, b in (d.get("host_ms_per_batch") or {}).items()},
      "| check_us", round(k["check"]["avg_launch_ms"] * 1e3, 1) if "check" in k else None,
      "| sort_us", round(k["sort"]["avg_launch_ms"] * 1e3, 1) if "sort" in k else None,
      "| parity", (d.get("parity") or {}).get("mismatched_batches"))
PY
done
