#!/bin/bash
# The RCCL leg at world size 1 (one MI355X): bench.py --dist --backend nccl under torchrun; the
# line goes to gpurun_out/r05f/rccl_world1_c2.json.
set -u
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/${TAG:-r05f}
mkdir -p $O
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 1 --dist --backend nccl --workload c2 --steps 20 --warmup 3 \
  --too-old-frac 0.05 > $O/rccl_world1_c2.json 2> $O/rccl_world1_c2.err || { tail -20 $O/rccl_world1_c2.err; exit 1; }
python3 -c "
import json;d=json.loads([l for l in open('$O/rccl_world1_c2.json') if l.startswith('{')][-1])
print(d['value'], d['distributed'], d['combine_check'], d['parity']['batches_checked'], d['parity']['mismatched_batches'], d['verdict_mix'])"
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_multi.py -m gpu -k rccl > $O/rccl_test.log 2>&1 || { tail -20 $O/rccl_test.log; exit 1; }
tail -1 $O/rccl_test.log
