#!/bin/bash
# Round-5 evidence, part 2 (after the part-1 profiles are in profiles/): bench lines C1-C4, C2 at
# 32768-txn batches, C2 with 5% of snapshots past the window (TooOld at full size), each with the
# CPU baseline and the parity replay of every measured batch.
set -u
cd "$(dirname "$0")/.." || exit 1
TAG=${TAG:-r05f}
O=gpurun_out/$TAG
mkdir -p $O
step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "== $name $(date +%T)" >&2
  timeout -k 10 "$t" "$@"
  local rc=$?
  echo "== $name rc=$rc" >&2
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >&2; exit $rc; fi
}
summ() {
  python3 -c "import json;d=json.load(open('$1'));p=d['parity'];print('$1', round(d['value']/1e6,2), 'h2d', round(d['h2d_inclusive_txns_per_s']/1e6,2), 'total', round(d['total_txns_per_s']/1e6,2), 'dev', d['device_bound']['ms_per_batch'], 'parity', p['batches_checked'], p['mismatched_batches'], 'mix', d['verdict_mix'], 'roof', d['roofline']['kernel'], round(d['roofline']['frac'],3), d['roofline'].get('frac_rocprof'), d['roofline'].get('traffic'), 'cpu', d['cpu_baseline']['value'])" >&2
}
for w in c2 c1 c3 c4; do
  step bench_$w 500 python bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err
  summ $O/bench_$w.json
done
step bench_c2_32768 500 python bench.py --workload c2 --txns 32768 > $O/bench_c2_32768.json 2> $O/bench_c2_32768.err
summ $O/bench_c2_32768.json
step bench_c2_tooold 500 python bench.py --workload c2 --too-old-frac 0.05 > $O/bench_c2_tooold.json 2> $O/bench_c2_tooold.err
summ $O/bench_c2_tooold.json

step rccl_world1 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 1 --dist --backend nccl --workload c2 --steps 20 --warmup 3 \
  --too-old-frac 0.05 > $O/rccl_world1_c2.json 2> $O/rccl_world1_c2.err
echo rccl done >&2
