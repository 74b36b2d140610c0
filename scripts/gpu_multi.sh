#!/bin/bash
# Rehearse the sharded bench path on one GPU: 2 ranks (gloo: RCCL refuses two ranks on one card),
# the proxy's routing on the device inside the timed region.  WL / TXNS / HIST select the shape.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --workload ${WL:-c2} --txns ${TXNS:-5000} --steps ${STEPS:-30} --warmup 3 \
  --history ${HIST:-1000000} --backend ${BACKEND:-gloo} --cpu-seconds 30 ${BENCH_ARGS:-} \
  > gpurun_out/bench_multi.json 2> gpurun_out/bench_multi.err
rc=$?
echo "multi rc=$rc" >&2
cat gpurun_out/bench_multi.json >&2
tail -5 gpurun_out/bench_multi.err >&2
exit $rc
