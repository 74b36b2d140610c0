#!/bin/bash
# HIP runtime API trace + kernel trace of a short bench (host-side cost of each call in the loop).
set -u
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/api
timeout -k 10 300 rocprofv3 --hip-runtime-trace --kernel-trace --output-format csv -d gpurun_out/api -o run -- \
  python3 bench.py --steps 20 --warmup 3 --resident-steps 0 --total-steps 0 --breakdown-steps 0 --no-cpu-baseline ${BENCH_ARGS:-} \
  > gpurun_out/api/bench.json 2> gpurun_out/api/bench.err
rc=$?
f=$(find gpurun_out/api -name "*hip_api_trace.csv" | head -1)
[ -n "$f" ] && python3 - "$f" > gpurun_out/api/api_summary.txt <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: [0, 0.0])
for r in rows:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
    a = agg[r["Function"]]; a[0] += 1; a[1] += d
for k, (n, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:40]:
    print(f"{k:40s} calls={n:7d} total_ms={t/1000:9.3f} avg_us={t/n:8.2f}")
PY
cat gpurun_out/api/api_summary.txt >&2
exit $rc
