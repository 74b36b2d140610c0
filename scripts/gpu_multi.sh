#!/bin/bash
# Rehearse the sharded bench path on one GPU: 2 ranks (gloo for the verdict all-reduce), short run.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 2 --history 1000000 --backend ${BACKEND:-gloo} \
  > gpurun_out/bench_multi.json 2> gpurun_out/bench_multi.err
rc=$?
echo "multi rc=$rc" >&2
cat gpurun_out/bench_multi.json >&2
tail -5 gpurun_out/bench_multi.err >&2
exit $rc
