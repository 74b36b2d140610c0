"""Device routing alone (fdbcs_batch_add_routed) on one GPU: G proxy shares of a C2 (or C4) global
batch gathered in device memory, every resolver's split routed and timed with events (the engine's
ms_route_kernels), no collectives.  Prints one JSON line per G: routing kernels' device ms per
global batch per resolver, host ms of the call, and the routed sizes against the host routing.
Usage: python scripts/route_bench.py [c2|c4] [G ...]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

torch.cuda.is_available()
from foundationdb_amd import build, conflict_set as C, workloads as W  # noqa: E402
from foundationdb_amd.sharding import KeyRangeSharding  # noqa: E402

build.build()
wl = sys.argv[1] if len(sys.argv) > 1 else "c2"
Gs = [int(x) for x in sys.argv[2:]] or [2, 4, 8]
for G in Gs:
    rng = np.random.default_rng(G)
    if wl == "c4":
        p = W.C4Params(txns=5000 * G, history=0)
        sh = KeyRangeSharding([W.c4_user_split(p, g * p.users // G) for g in range(1, G)])
        pb = W.c4_batch(p, rng, 10_000_000)
    else:
        p = W.C2Params(txns=5000 * G, history=0)
        sh = KeyRangeSharding.uniform(G)
        pb = W.c2_batch(p, rng, 10_000_000)
    shares = [C.share_pack(pb.slice_txns(g * 5000, (g + 1) * 5000)) for g in range(G)]
    stride = (max(len(x) for x in shares) + 4095) // 4096 * 4096
    host = np.zeros(G * stride, np.uint8)
    for g, x in enumerate(shares):
        host[g * stride: g * stride + len(x)] = x
    dev = torch.from_numpy(host).cuda()
    out = torch.empty(pb.n_txn, dtype=torch.uint8, device="cuda")
    ready = torch.ones(1, dtype=torch.int32, device="cuda")  # set by torch's stream; polled by the engine
    tail = int(np.maximum(np.diff(pb.key_offsets) - 16, 0).sum())
    routes = sh.route(pb)
    res = []
    for r in range(G):
        cs = C.ConflictSet(0)
        lo = sh.splits[r - 1] if r > 0 else None
        hi = sh.splits[r] if r < G - 1 else None
        for rep in range(12):
            if rep == 2:
                cs.reset_stats()
            b = C.ConflictBatch(cs)
            b.add_routed(dev.data_ptr(), stride, G, 5000, lo, hi, (pb.n_txn, pb.n_reads, pb.n_writes, tail),
                         out.data_ptr(), pb.n_txn, ready.data_ptr(), 1)
            T, R, Wn, _, _ = b.routed_info()
            sub = routes[r].batch
            assert (T, R, Wn) == (sub.n_txn, sub.n_reads, sub.n_writes), (T, R, Wn, sub.n_txn)
            b.detect_async(10_000_000 + rep, 5_000_000)
            b.wait()
            b.close()
        st = cs.stats()
        res.append((st["ms_route_kernels"] / st["routed_batches"], st["host_ms_route"] / st["routed_batches"]))
        cs.close()
    print(json.dumps({"workload": wl, "resolvers": G, "global_txns": pb.n_txn, "share_stride": stride,
                      "route_kernels_ms_per_batch": max(x[0] for x in res),
                      "route_kernels_ms_mean": sum(x[0] for x in res) / G,
                      "route_host_ms_per_batch": max(x[1] for x in res), "sizes_match_host_routing": True}),
          flush=True)
