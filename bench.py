#!/usr/bin/env python3
"""Benchmark: resolved transactions/s of the MI355X conflict-resolution engine.

Workload (BASELINE.json configs[1], "C2"): a single-MI355X resolver with 5000-transaction commit
batches, 5 read + 2 write conflict ranges per transaction, 16-byte uniform keys, over a
5M-boundary MVCC history prefilled across a 5e6-version window.  `--workload c1|c3|c4` selects the
other BASELINE configurations (skipListTest, Zipf hot keys, tuple keys over a 50M-boundary window).

A step is one ConflictBatch::detectConflicts (SkipList.cpp:844-890) over one batch.  The timed
region of `value` holds, per batch, every kernel and the verdict bytes back in host memory, with
the packed batch already resident in HBM when the region starts (the task's measurement contract:
inputs resident, the PCIe-inclusive rate reported beside it as `h2d_inclusive_txns_per_s`, where
each batch's H2D copy runs inside the loop as SURVEY §8(d) first planned); addTransaction (the
host-side normalization into pinned staging) happens before it, as the reference's "Detect only"
figure excludes addTransaction (SkipList.cpp:1069-1078, 1087-1090).  `total_txns_per_s` is the
reference's "total" figure: addTransaction (and the H2D) inside the timed loop as well.

Passes, in order, each on its own batches: warmup; a per-kernel profile (events around every
kernel, timing level 3) that names the dominant kernel (largest device time); the timed region
(events around that kernel only, on 1 batch in 4: `roofline`); PCIe-inclusive, add+detect
("total"), synchronous (one batch at a time through detect_conflicts, as Resolver.actor.cpp:179-194
calls it: `sync_*` and per-batch latency), device-bound (batches queued behind a hold kernel, then
released: the device's own rate) and per-phase breakdown passes.

After timing, the whole batch sequence is replayed on the CPU restatement of the reference
algorithm (oracle/skiplist_baseline.cpp, with the reference's bounded removeBefore,
SkipList.cpp:880-889) and every GPU verdict is compared: `parity` in the JSON line.  That replay's
time over the timed batches is `cpu_baseline`: one thread pinned to one core like skipListTest's
setAffinity(0) (SkipList.cpp:1015), per phase as the reference's PerfDoubleCounters
(SkipList.cpp:49-51, 1082-1102); at N > 1 every rank replays its own routed sub-batches on its own
pinned core at the same time (G resolvers on G cores), over the max of their times.

N > 1 (torchrun, one rank per GPU): the key space is range-sharded across ranks like FDB's
multi-resolver split (CommitProxyServer.actor.cpp:147-174).  Every rank builds the same global batch
of N x 5000 transactions, keeps its routed sub-batch, resolves it on its GPU, and the verdicts are
combined by an RCCL all-reduce MAX of conflict bytes (= proxy min over resolvers,
CommitProxyServer.actor.cpp:772-777).  Weak scaling: per-GPU work is fixed.  Parity at N > 1:
every rank replays its own routed sub-batches on its own CPU restatement (G reference conflict
sets fed the same routing).

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import roofline  # noqa: E402

WINDOW = 8  # batches in flight (submitted, not yet waited) in the timed loops


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--window", type=int, default=8, help="batches in flight in the timed loops")
    ap.add_argument("--steps", type=int, default=20,
                    help="timed batches (the driver's count); --steps 200 spans several delta compactions")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--txns", type=int, default=0, help="transactions per batch per GPU; 0 = the workload's")
    ap.add_argument("--history", type=int, default=0,
                    help="history boundaries per GPU; 0 = the workload's (5M for c2/c3, 50M for c4, empty for c1)")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--gc-interval", type=int, default=0,
                    help="force a compaction (+GC) at least every N batches; 0 = when the delta tier is full")
    ap.add_argument("--delta-limit", type=int, default=0, help="delta-tier bound; 0 = automatic (~base/16)")
    ap.add_argument("--roof-steps", type=int, default=32,
                    help="batches of the roofline pass (events around the dominant kernel, 1 batch in 4), run "
                    "after the timed region so that no event record sits inside it; 0 = no roofline")
    ap.add_argument("--total-steps", type=int, default=-1,
                    help="batches of the add+detect ('total') pass; -1 = --steps, 0 = skip")
    ap.add_argument("--h2d-steps", type=int, default=20,
                    help="batches of the PCIe-inclusive pass (each batch's H2D inside the loop; reported beside "
                    "`value`, which is measured on batches already resident in HBM)")
    ap.add_argument("--breakdown-steps", type=int, default=128,
                    help="extra batches after the timed region with every phase timed: the per-phase split and the "
                    "compaction + GC cost amortized per batch (>= 128 batches hold several compactions and GC runs)")
    ap.add_argument("--profile-steps", type=int, default=16,
                    help="batches with events around every kernel (per-kernel table, dominant kernel)")
    ap.add_argument("--sync-steps", type=int, default=20,
                    help="batches resolved one at a time (window 1: the Resolver's synchronous call)")
    ap.add_argument("--hold-steps", type=int, default=16,
                    help="batches queued behind a hold kernel, then released (device-bound rate)")
    ap.add_argument("--cpu-seconds", type=float, default=60.0,
                    help="bound on the CPU replay (parity + cpu_baseline); batches past it are not checked")
    ap.add_argument("--no-cpu-baseline", action="store_true", help="skip the CPU replay (no parity, no baseline)")
    ap.add_argument("--workload", default="c2", choices=["c1", "c2", "c3", "c4"])
    ap.add_argument("--reshard", action="store_true",
                    help="N>1: dynamic resharding (resolver iops samples + resolutionBalancing + keyResolvers "
                    "history, foundationdb_amd/balancing.py) instead of the static split")
    ap.add_argument("--reshard-preroll", type=int, default=200,
                    help="global batches routed (not resolved) to train the balancer before the run")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="collective backend for the verdict all-reduce (nccl = RCCL over xGMI)")
    ap.add_argument("--dist", action="store_true",
                    help="run the multi-resolver path (process group, device routing of gathered shares, "
                    "conflict-byte MAX all-reduce) even at world size 1: the RCCL leg on one GPU")
    ap.add_argument("--too-old-frac", type=float, default=0.0,
                    help="share of transactions whose snapshot sits at the MVCC window's edge (about half of "
                    "them TooOld, SkipList.cpp:770)")
    return ap.parse_args()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def workload_params(args):
    from foundationdb_amd import workloads as W

    if args.workload == "c4":
        return W.C4Params(txns=args.txns or 5000, history=args.history or 50_000_000, too_old_frac=args.too_old_frac)
    if args.workload == "c1":
        return W.C2Params(txns=args.txns or 2500, reads=1, writes=1, history=args.history or 0)
    return W.C2Params(txns=args.txns or 5000, history=args.history or 5_000_000, too_old_frac=args.too_old_frac)


def sharding_for(args, p, world):
    from foundationdb_amd import workloads as W
    from foundationdb_amd.sharding import KeyRangeSharding

    if world == 1:  # one resolver (the --dist rehearsal of the multi-resolver path: it owns every key)
        return KeyRangeSharding([]) if args.dist else None
    if args.workload == "c4":  # every key shares the subspace: split by user
        return KeyRangeSharding([W.c4_user_split(p, g * p.users // world) for g in range(1, world)])
    if args.workload == "c1":  # setK keys share 12 bytes of '.': split on the integer
        return KeyRangeSharding([W.setk([g * 20_000_000 // world])[0].tobytes() for g in range(1, world)])
    if args.workload == "c3":  # Mako keys share 'mako': split on the item index (Zipf: rank 0 is hot)
        return KeyRangeSharding([W.mako_keys(np.array([g * 1_000_000 // world]))[0].tobytes() for g in range(1, world)])
    return KeyRangeSharding.uniform(world)


def route_all(args, p, world, gbatches):
    """Per global batch, the ShardBatches of every rank (identical on all ranks: the routing and the
    balancer are deterministic functions of the global batches)."""
    from foundationdb_amd import balancing as B
    from foundationdb_amd.sharding import KeyResolvers

    sh = sharding_for(args, p, world)
    if sh is None:
        return None, None
    if not args.reshard:
        return [sh.route(pb) for pb, _, _ in gbatches], None
    # compressed time: balance every 20 batches (MIN_BALANCE_TIME is 0.2 s = 200 batches at 1e6
    # versions/s); the reference's simulation knobs for the sample and the threshold
    br = B.BalancedRouting(world, KeyResolvers.from_sharding(sh), seed=args.seed, min_balance_difference=10_000,
                           balance_time=20 * p.version_step / B.VERSIONS_PER_SECOND, key_bytes_per_sample=1_000)
    first = gbatches[0][1] - p.version_step * (args.reshard_preroll + 1)
    pre = make_batches(args, p, args.reshard_preroll, world, first, seed_offset=7919)
    for pb, now, _ in pre:
        br.route(pb, now)
    routed = [br.route(pb, now) for pb, now, _ in gbatches]
    return routed, {"moves": br.balancer.moves_made, "map": [(b.hex(), o) for b, o in br.kr.current_map()]}


def shard_history(args, p, seed, rank, world, start_version):
    """Prefill: p.history boundaries inside this rank's key range."""
    from foundationdb_amd.workloads import c2_history, c4_history

    if args.workload == "c1" or p.history == 0:
        return np.zeros(0, np.uint8), np.zeros(1, np.int64), np.zeros(0, np.int64)
    if args.workload == "c4":
        users = (rank * p.users // world, (rank + 1) * p.users // world)
        return c4_history(p, seed=seed * 1000 + rank, start_version=start_version, users=users)
    kb, ko, vers = c2_history(p, seed=seed * 1000 + rank, start_version=start_version)
    if world > 1:
        keys = kb.reshape(-1, 16).copy()
        lo = (rank * 256) // world
        hi = ((rank + 1) * 256) // world
        keys[:, 0] = lo + (keys[:, 0].astype(np.int64) * (hi - lo) // 256).astype(np.uint8)
        hi64 = keys[:, :8].copy().view(">u8").reshape(-1)
        lo64 = keys[:, 8:].copy().view(">u8").reshape(-1)
        order = np.lexsort((lo64, hi64))
        keys = keys[order]
        keep = np.ones(len(keys), bool)
        keep[1:] = (keys[1:] != keys[:-1]).any(axis=1)
        keys = keys[keep]
        vers = vers[: len(keys)]
        kb = keys.reshape(-1)
        ko = np.arange(len(keys) + 1, dtype=np.int64) * 16
    return kb, ko, vers


def make_batches(args, p, n_batches, world, start_version, seed_offset=0):
    """Global batches (identical on every rank) with their (now, newOldest)."""
    from foundationdb_amd import workloads as W

    import dataclasses

    if args.workload == "c1":  # skipListTest: snapshot v, now v + 50, newOldest v (SkipList.cpp:1063-1077)
        return list(W.c1_batches(n_batches, seed=args.seed + seed_offset, data_per_batch=2 * p.txns * world))
    rng = np.random.default_rng(args.seed + seed_offset)
    zipf = W.ZipfGenerator(1_000_000, 0.99) if args.workload == "c3" else None
    gp = dataclasses.replace(p, txns=p.txns * world)
    out = []
    now = start_version
    for _ in range(n_batches):
        now += p.version_step
        if args.workload == "c4":
            pb = W.c4_batch(gp, rng, now)
        else:
            pb = W.c3_batch(gp, rng, now, zipf) if zipf else W.c2_batch(gp, rng, now)
        out.append((pb, now, now - p.window))
    return out


def directory_share(kb, ko, batches):
    """Share of the read lookups whose first two key bytes fall in a sparse slot (<= 16 level-0
    samples) of the base tier's radix directory, estimated on the prefilled history: those start
    at level 0 (roofline.lookup_bytes)."""
    n = len(ko) - 1
    if n < 64:
        return 0.0

    def slot(bytes_, offs, idx):
        a = offs[idx]
        ln = offs[idx + 1] - a
        b0 = np.where(ln > 0, bytes_[np.minimum(a, len(bytes_) - 1)], 0).astype(np.int64)
        b1 = np.where(ln > 1, bytes_[np.minimum(a + 1, len(bytes_) - 1)], 0).astype(np.int64)
        return b0 * 256 + b1

    counts = np.bincount(slot(kb, ko, np.arange(0, n, 64)), minlength=65536)
    hits = tot = 0
    for b in batches[:4]:
        nk = 2 * b.n_reads
        if nk == 0:
            continue
        sl = slot(b.key_bytes, b.key_offsets, np.arange(nk))
        hits += int((counts[sl] <= 16).sum())
        tot += nk
    return hits / tot if tot else 0.0


def cpu_model():
    cpu = platform.processor() or platform.machine()
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return cpu


def cpu_replay(args, kb, ko, vers, mine, gbatches, gpu_verdicts, timed, rank, n_batches=None, add_oldest=None,
               sample_from=None):
    """Replay every batch in order on the CPU restatement (oracle/skiplist_baseline.cpp): compare
    each GPU verdict vector and time the batches in `timed` (single thread, pinned to one core),
    and with sample_from every batch the GPU resolved from that index on (the same workload, a
    sample of ~10 s of CPU work at C2 instead of the timed region's ~0.7 s).
    add_oldest[i]: the oldest version the engine's addTransaction saw for batch i (its TooOld test,
    SkipList.cpp:770): a batch packed ahead of its predecessor's detect is replayed as added then."""
    from oracle import oracle

    oracle.build()
    try:  # skipListTest pins itself to one core (setAffinity(0), SkipList.cpp:1015)
        cores = sorted(os.sched_getaffinity(0))
        os.sched_setaffinity(0, {cores[(len(cores) // 2 + 2 * rank) % len(cores)]})  # away from core 0's IRQs
    except (AttributeError, OSError):
        cores = []
    sl = oracle.SkipListBaseline()
    t0 = time.time()
    sl.load_history(kb, ko, vers)
    load_s = time.time() - t0
    checked = mismatches = txn_mismatch = 0
    spent = 0.0
    done_txn = done_batches = 0
    done_global = 0
    phases = {k: 0.0 for k in oracle.SkipListBaseline.PHASES}
    first_bad = None
    t_begin = time.time()
    n_batches = len(gbatches) if n_batches is None else n_batches
    for i in range(n_batches):
        if gpu_verdicts[i] is None and i not in timed:
            # a batch the GPU never resolved (the hold pass is skipped on the multi-resolver path):
            # the device history never held it, so neither may the restatement's
            continue
        b = mine(i)  # this resolver's sub-batch (host routing, CommitProxyServer.actor.cpp:118-187)
        _, now, no = gbatches[i]
        t = time.perf_counter()
        # the reference's removeBefore: bounded to 3|combined|+10 nodes, resumed at removalKey
        # (SkipList.cpp:880-889); verdict-neutral, so parity holds against the GPU's full GC
        v, _ = sl.detect(b, now, no, gc="bounded", add_oldest=(add_oldest or {}).get(i))
        dt = time.perf_counter() - t
        if i in timed or (sample_from is not None and i >= sample_from and gpu_verdicts[i] is not None):
            spent += dt
            done_txn += b.n_txn
            done_global += gbatches[i][0].n_txn
            done_batches += 1
            for k, x in sl.last_times().items():
                phases[k] += x
        g = gpu_verdicts[i]
        if g is not None:
            checked += 1
            # a device-routed batch must hold exactly the host routing's sub-transactions
            bad = int((g != v).sum()) if len(g) == len(v) else max(len(g), len(v))
            if bad:
                mismatches += 1
                txn_mismatch += bad
                if first_bad is None:
                    first_bad = i
        if time.time() - t_begin > args.cpu_seconds:
            break
    if cores:
        os.sched_setaffinity(0, set(cores))
    parity = {
        "reference": "oracle/skiplist_baseline.cpp (reference algorithm, restated; cross-checked vs "
        "oracle/semantic_oracle.cpp in tests/test_oracle.py)",
        "batches_checked": checked,
        "batches_total": n_batches,
        "mismatched_batches": mismatches,
        "mismatched_txns": txn_mismatch,
        "first_mismatch": first_bad,
    }
    names = {"add": "Add", "sort": "D.Sort", "check_read": "D.CheckRead", "intra": "D.CheckIntraBatch",
             "combine": "D.Combine", "merge": "D.MergeWrite", "remove_before": "D.RemoveBefore", "total": "Detect"}
    base = {
        "value": done_txn / spent if spent > 0 else None,
        "unit": "txns/s",
        "cores": 1,
        "kind": "port",
        "label": "reference algorithm, restated (oracle/skiplist_baseline.cpp)",
        "gc": "bounded removeBefore (3*|combined|+10 nodes from removalKey, SkipList.cpp:880-889)",
        "phase_ms_per_batch": {names[k]: 1e3 * x / max(1, done_batches) for k, x in phases.items()},
        "sample": f"{done_batches} {args.workload.upper()} batches from the timed region on (after replaying the "
        f"warmup batches) on a "
        f"{len(vers)}-boundary history ({spent:.1f}s CPU, history load {load_s:.1f}s), bounded removeBefore, "
        f"1 thread pinned to one core of {cpu_model()} (nproc {os.cpu_count()})",
        "_spent": spent,
        "_global_txns": done_global,
        "_batches": done_batches,
    }
    return parity, base


def main():
    args = parse()
    global WINDOW
    WINDOW = max(1, args.window)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch

    dist = None
    ndev = max(1, torch.cuda.device_count())
    device = local % ndev  # one rank per GPU; more ranks than GPUs only for rehearsals (gloo)
    if world > 1 or args.dist:
        import torch.distributed as dist

        torch.cuda.set_device(device)
        dist.init_process_group(args.backend)
    # collectives run on device tensors whenever there is a GPU: RCCL ("nccl"), or gloo's CUDA
    # all-reduce in one-GPU rehearsals (several ranks on one card, where RCCL refuses)
    cdev = "cuda" if torch.cuda.is_available() else "cpu"
    from foundationdb_amd import build as fbuild

    fbuild.build()
    from foundationdb_amd import conflict_set as C
    from foundationdb_amd.sharding import KeyRangeSharding

    p = workload_params(args)
    start_version = 10_000_000
    t0 = time.time()
    kb, ko, vers = shard_history(args, p, args.seed, rank, world, start_version)
    n_total = args.steps if args.total_steps < 0 else args.total_steps
    # batch index ranges of the passes, in order
    spans = {}
    at = 0
    for name, n in (("warmup", args.warmup), ("timed", args.steps), ("profile", args.profile_steps),
                    ("roof", args.roof_steps), ("h2d", args.h2d_steps), ("total", n_total), ("sync", args.sync_steps),
                    ("hold", args.hold_steps), ("breakdown", args.breakdown_steps)):
        spans[name] = (at, at + n)
        at += n
    n_all = at
    timed_lo, timed_hi = spans["timed"]
    gbatches = make_batches(args, p, n_all, world, start_version)
    # N > 1: the proxy's routing (CommitProxyServer.actor.cpp:118-187) runs on the GPUs inside the
    # timed region: every rank is the proxy of one share (p.txns transactions) of each global batch,
    # the shares are all-gathered over xGMI, and every resolver keeps its key range's part on the
    # device (fdbcs_batch_add_routed).  --reshard keeps the host routing of balancing.py (its
    # ownership history is not on the device): that path is a feature check, routed before timing.
    multi = world > 1 or args.dist  # the multi-resolver path (one resolver of G, G >= 1)
    droute = multi and not args.reshard and cdev != "cpu"
    sh = sharding_for(args, p, world)
    all_routed, reshard = route_all(args, p, world, gbatches) if (multi and not droute) else (None, None)
    route_cache = {}

    def routed_at(i):
        """This rank's ShardBatch of global batch i by the host routing (parity replay, checks)."""
        if all_routed is not None:
            return all_routed[i][rank]
        if i not in route_cache:
            route_cache[i] = sh.route(gbatches[i][0])[rank]
        return route_cache[i]

    def mine_at(i):
        return routed_at(i).batch if multi else gbatches[i][0]

    log(f"[rank {rank}] generated history {len(vers)} + {n_all} batches in {time.time() - t0:.1f}s")

    cs = C.ConflictSet(device)
    cs.set_gc_interval(args.gc_interval)
    cs.set_delta_limit(args.delta_limit)
    if len(vers):
        cs.load_history(kb, ko, vers, 0)

    def tail_bytes(ko):  # history tail bytes, each tail padded to 8 (engine.cpp padded_tail)
        t = np.diff(ko) - 16
        return int(((t[t > 0] + 7) // 8 * 8).sum())

    # capacity: a resolver's batch is at most the global batch (device routing) or its host-routed part
    sized = [pb for pb, _, _ in gbatches] if (not multi or droute) else [mine_at(i) for i in range(n_all)]
    maxT = max(b.n_txn for b in sized)
    maxR = max(b.n_reads for b in sized)
    maxW = max(b.n_writes for b in sized)
    maxTail = max(int(np.maximum(np.diff(b.key_offsets) - 16, 0).sum()) for b in sized)
    tail_total = tail_bytes(ko) + sum(tail_bytes(b.key_offsets) for b in sized) // (world if droute else 1) + (1 << 20)
    cs.reserve(len(vers) + 2 * sum(b.n_writes for b in sized) + 1024, tail_total, maxT, maxR, maxW)
    del sized
    verdicts = [None] * n_all

    # Multi-GPU combine (CommitProxyServer.actor.cpp:764-780): each batch's stage B also writes its
    # conflict bytes 2 - verdict at the routed transactions' global indices (0 elsewhere) into a
    # T-byte device buffer, complete when the batch is; one MAX all-reduce over the ranks (RCCL;
    # gloo's CUDA all-reduce in one-GPU rehearsals) combines them.
    on_device = dist is not None and cdev != "cpu"
    outbuf = {}
    if on_device:
        for i in range(n_all):
            outbuf[i] = torch.empty(gbatches[i][0].n_txn, dtype=torch.uint8, device=cdev)
    combined = {}

    # device routing: this rank's share of every batch in the wire layout (pinned host memory,
    # packed per pass like addTransaction), a ring of device share / all-gather buffers
    RING = WINDOW + 3
    stride = 0
    if droute:
        lo_key = sh.splits[rank - 1] if rank > 0 else None
        hi_key = sh.splits[rank] if rank < world - 1 else None
        share_bytes = max(len(C.share_pack(gbatches[i][0].slice_txns(rank * p.txns, (rank + 1) * p.txns)))
                          for i in range(0, n_all, max(1, n_all // 16)))
        tb = torch.tensor([share_bytes], dtype=torch.int64, device=cdev)
        dist.all_reduce(tb, op=dist.ReduceOp.MAX)
        stride = (int(tb.item()) * 5 // 4 + 4095) // 4096 * 4096  # headroom over the sampled batches
        share_dev = [torch.empty(stride, dtype=torch.uint8, device=cdev) for _ in range(RING)]
        gathered = [torch.empty(world * stride, dtype=torch.uint8, device=cdev) for _ in range(RING)]
        # torch's collectives run in their own HIP runtime: the engine cannot wait on their streams,
        # so the current stream sets ready[k] = i + 1 once batch i's shares are gathered and the
        # engine's first routing kernel polls it
        ready = torch.zeros(RING, dtype=torch.int32, device=cdev)
        caps = (maxT, maxR, maxW, maxTail)

        def pack_share(i):
            pin = torch.empty(stride, dtype=torch.uint8, pin_memory=True)
            C.share_pack(gbatches[i][0].slice_txns(rank * p.txns, (rank + 1) * p.txns), pin.numpy())
            return pin

        def route_batch(i, pin):
            """H2D of this rank's share (unless `pin` is the share already in HBM), the all-gather, and
            the device split into a new batch."""
            k = i % RING
            src = pin
            if not pin.is_cuda:
                share_dev[k].copy_(pin, non_blocking=True)
                src = share_dev[k]
            if args.backend == "nccl":
                dist.all_gather_into_tensor(gathered[k], src)
            else:  # gloo (one-GPU rehearsals): list form
                dist.all_gather(list(gathered[k].view(world, stride).unbind(0)), src)
            ready[k].fill_(i + 1)
            o = C.ConflictBatch(cs)
            o.add_routed(gathered[k].data_ptr(), stride, world, p.txns, lo_key, hi_key, caps, outbuf[i].data_ptr(),
                         gbatches[i][0].n_txn, ready[k:k + 1].data_ptr(), i + 1)
            return o

    def attach(i, o):
        if on_device:
            r = routed_at(i)
            o.set_conflict_output(r.txn_ids, gbatches[i][0].n_txn, outbuf[i].data_ptr())

    def combine(i, v):
        if on_device:
            c = outbuf[i]
        else:
            c = torch.from_numpy(KeyRangeSharding.conflict_bytes(gbatches[i][0].n_txn, routed_at(i), v)).to(cdev)
        dist.all_reduce(c, op=dist.ReduceOp.MAX)
        combined[i] = c

    host = {"add": 0.0, "submit": 0.0, "wait": 0.0}
    # the oldest version the engine held when each batch was added (its TooOld test is made then,
    # SkipList.cpp:770): batches packed ahead of their predecessors' detects are replayed that way
    add_oldest = {}

    def add_batch(i):
        o = C.ConflictBatch(cs)
        add_oldest[i] = cs.oldest_version
        o.add_packed(mine_at(i))
        attach(i, o)
        return o

    def run(lo, hi, objs, window=WINDOW, lat=None):
        """Submit batches lo..hi-1 (objs: packed ConflictBatch objects — or, with device routing,
        packed shares — or None: pack inside the loop), keeping at most `window` in flight;
        upload (H2D), routing, kernels and verdicts each time.  lat: per-batch submit-to-verdicts
        seconds are appended (window 1: the synchronous call)."""
        inflight = []
        pc = time.perf_counter

        def retire(j, oj, t_sub):
            t = pc()
            verdicts[j] = oj.wait()
            host["wait"] += pc() - t
            if lat is not None:
                lat.append(pc() - t_sub)
            if dist is not None:
                combine(j, verdicts[j])
            oj.close()

        pending = None  # device routing: a batch routed, its detect issued after the next one's routing

        def detect(j, oj, t_sub):
            _, now_j, no_j = gbatches[j]
            t1 = pc()
            oj.detect_async(now_j, no_j)
            host["submit"] += pc() - t1
            inflight.append((j, oj, t_sub))
            while len(inflight) >= window:
                retire(*inflight.pop(0))

        for i in range(lo, hi):
            _, now, no = gbatches[i]
            t = pc()
            if droute:
                pin = objs[i] if objs is not None else pack_share(i)
                t1 = pc()
                o = route_batch(i, pin)
                host["add"] += t1 - t
                host["submit"] += pc() - t1
                if pending is not None:
                    detect(*pending)
                pending = (i, o, t1)
                if window == 1:  # the synchronous call: this batch's detect and wait now
                    detect(*pending)
                    pending = None
                continue
            if objs is None:  # the Resolver's order: added after the previous batch's detect
                o = add_batch(i)
            else:
                o = objs[i]
            t1 = pc()
            o.detect_async(now, no)
            host["add"] += t1 - t
            host["submit"] += pc() - t1
            inflight.append((i, o, t1))
            if len(inflight) >= window:
                retire(*inflight.pop(0))
        if pending is not None:
            detect(*pending)
        for j, oj, ts in inflight:
            retire(j, oj, ts)
        inflight.clear()

    def packed(lo, hi):
        objs = {}
        for i in range(lo, hi):
            if droute:  # the proxy's addTransaction: its share in the wire layout
                objs[i] = pack_share(i)
                continue
            objs[i] = add_batch(i)  # addTransaction: normalized into pinned staging, not uploaded
        return objs

    def barrier():
        # the engine's streams live in its own HIP runtime: torch.cuda.synchronize()
        # does not wait for them, so every upload and stage already issued is drained here
        cs.sync()
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    def max_over_ranks(x):
        if dist is None:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def pass_txns(name):
        lo, hi = spans[name]
        return sum(gbatches[i][0].n_txn for i in range(lo, hi))

    run(*spans["warmup"], packed(*spans["warmup"]))

    def resident(lo, hi):
        """Batches lo..hi-1 packed and their H2D issued (a rank's proxy share likewise); the caller's
        barrier() then waits for the copies on the engine's upload stream."""
        objs = packed(lo, hi)
        for i, o in objs.items():
            if droute:
                objs[i] = o.to(cdev)
            else:
                o.upload()
        return objs

    # `value`: the batches' inputs resident in HBM when the timed region starts (each batch's packed
    # H2D issued and drained by barrier() before it; a rank's proxy share likewise) -- the
    # PCIe-inclusive rate is the h2d pass below.  No event is recorded inside the region.
    objs = resident(timed_lo, timed_hi)
    cs.reset_stats()
    barrier()
    for k in host:
        host[k] = 0.0
    t_start = time.perf_counter()
    run(timed_lo, timed_hi, objs)
    barrier()
    elapsed = max_over_ranks(time.perf_counter() - t_start)
    st = cs.stats()
    host_timed = {k: v / args.steps * 1e3 for k, v in host.items()}
    for k in ("host_ms_prepare", "host_ms_record", "host_ms_submit"):  # inside detect_async (engine's clock)
        host_timed["engine_" + k[8:]] = st[k] / max(1, st["batches"])

    # per-kernel profile, after the timed region so that it sees the history the roofline pass runs
    # on (the kernels can change with it: a base tier past kSplitCheckMinBase splits the read check):
    # events around every kernel of every batch (timing level 3), pipelined as in the timed region;
    # the dominant kernel (largest device time) is then timed by the roofline pass (level 1, 1 batch
    # in 4, on the stream it runs on)
    kprof = {}
    dominant = None
    if args.profile_steps > 0:
        cs.reset_stats()
        cs.set_timing(3)
        run(*spans["profile"], packed(*spans["profile"]))
        kprof = cs.kernel_profile()
        st_prof = cs.stats()
        dominant = max(kprof, key=lambda k: kprof[k]["ms"]) if kprof else None
    # The dominant kernel by rocprofv3 kernel-trace time (dispatch to completion) when a summary of
    # this configuration and build is committed: the profile pass's events also count the time a
    # kernel waits for its stream's turn behind the other streams' kernels.
    build = roofline.build_id(ROOT)
    rp_kernels, rp_note = roofline.rocprof_kernels(ROOT, args.workload, p.txns, p.history, build)
    dominant_source = "profile pass (events around every kernel)"
    if rp_kernels:
        ranked = [k for k in rp_kernels if k in kprof]  # (kernels this history state launches)
        if ranked:
            dominant = ranked[0]
            dominant_source = "rocprofv3 kernel trace: " + rp_note
    cs.set_timing(0)
    # resolved now, while the profile pass's kernel list still names it; recorded only at timing 1
    cs.set_timed_kernel(dominant)

    # roofline pass: the same pipeline on its own resident batches, with events around the dominant
    # kernel on 1 batch in 4 (on the stream it runs on)
    kprof_timed = {}
    st_roof = st
    roof_elapsed = None
    if dominant and args.roof_steps > 0:
        objs = resident(*spans["roof"])
        cs.set_timing(1)
        cs.reset_stats()
        barrier()
        t_start = time.perf_counter()
        run(*spans["roof"], objs)
        barrier()
        roof_elapsed = max_over_ranks(time.perf_counter() - t_start)
        kprof_timed = cs.kernel_profile()
        st_roof = cs.stats()
        cs.set_timed_kernel(None)
        cs.set_timing(0)

    h2d_elapsed = None
    if args.h2d_steps > 0:  # PCIe-inclusive: each batch's H2D (the proxy share's, with routing) inside the loop
        objs = packed(*spans["h2d"])
        barrier()
        t_start = time.perf_counter()
        run(*spans["h2d"], objs)
        barrier()
        h2d_elapsed = max_over_ranks(time.perf_counter() - t_start)

    total_elapsed = None
    total_host = None
    if n_total > 0:  # the reference's "total": addTransaction inside the loop as well
        for k in host:
            host[k] = 0.0
        cs.reset_stats()
        barrier()
        t_start = time.perf_counter()
        run(*spans["total"], None)
        barrier()
        total_elapsed = max_over_ranks(time.perf_counter() - t_start)
        stt = cs.stats()
        # where a batch's host time goes when addTransaction is in the loop (the calling thread):
        # add = ConflictBatch + addTransaction of the packed batch (engine_add: inside
        # fdbcs_batch_add_packed alone), submit = detect_async, wait = waiting for verdicts
        total_host = {k: v / n_total * 1e3 for k, v in host.items()}
        total_host["engine_add"] = stt["host_ms_add"] / max(1, stt["added_txns"]) * p.txns
        total_host["elapsed"] = total_elapsed / n_total * 1e3

    sync = None
    if args.sync_steps > 0:
        # one batch at a time, as the Resolver calls detectConflicts (Resolver.actor.cpp:179-194): the
        # batch is added beforehand, then detect (H2D, kernels, verdicts back) and wait back to back
        lat = []
        objs = packed(*spans["sync"])
        barrier()
        t_start = time.perf_counter()
        run(*spans["sync"], objs, window=1, lat=lat)
        barrier()
        sync_elapsed = max_over_ranks(time.perf_counter() - t_start)
        lat_ms = np.array(lat) * 1e3
        sync = {"txns_per_s": pass_txns("sync") / sync_elapsed,
                "latency_ms_p50": float(np.percentile(lat_ms, 50)),
                "latency_ms_p99": float(np.percentile(lat_ms, 99)),
                "latency_ms_mean": float(lat_ms.mean()), "batches": len(lat)}

    device_bound = None
    if args.hold_steps > 0 and dist is None:
        # every stream held, the batches submitted behind the hold, then released: the device runs
        # them back to back at its own rate, whatever the submitting thread's cost
        objs = packed(*spans["hold"])
        for o in objs.values():
            o.upload()
        torch.cuda.synchronize()
        cs.debug_hold(True)
        lo, hi = spans["hold"]
        for i in range(lo, hi):
            _, now, no = gbatches[i]
            objs[i].detect_async(now, no)
        t_start = time.perf_counter()
        cs.debug_hold(False)
        for i in range(lo, hi):
            verdicts[i] = objs[i].wait()
            objs[i].close()
        dev_elapsed = time.perf_counter() - t_start
        device_bound = {"txns_per_s": pass_txns("hold") / dev_elapsed, "ms_per_batch": dev_elapsed / (hi - lo) * 1e3,
                        "batches": hi - lo}

    # diagnostic phase split: extra batches with every phase timed (each event costs queue time,
    # so these are outside the timed region)
    phase = None
    amortized = None
    if args.breakdown_steps > 0:
        cs.set_timing(2)
        cs.reset_stats()
        run(*spans["breakdown"], packed(*spans["breakdown"]))
        torch.cuda.synchronize()
        sb = cs.stats()
        phase = {
            k: sb[k] / max(1, sb["batches"])
            for k in ("ms_upload", "ms_check_read", "ms_sort", "ms_intra", "ms_combine", "ms_merge", "ms_compact",
                      "ms_gc", "ms_epilogue", "ms_total")
        }
        phase["batches"] = sb["batches"]
        phase["compactions"] = sb["compactions"]
        phase["intra_edges"] = sb["intra_edges"] / max(1, sb["batches"] - sb["intra_fallbacks"])
        phase["intra_rounds"] = sb["intra_rounds"] / max(1, sb["batches"] - sb["intra_fallbacks"])
        phase["intra_fallbacks"] = sb["intra_fallbacks"]
        phase["gc_runs"] = sb["gc_runs"]
        # what the headline's short window may not hold: compaction (delta folded into the base) and
        # removeBefore, amortized over the breakdown pass (the reference pays a bounded removeBefore
        # every batch, SkipList.cpp:880-889)
        amortized = {"compaction_ms_per_batch": phase["ms_compact"], "gc_ms_per_batch": phase["ms_gc"],
                     "merge_ms_per_batch": phase["ms_merge"], "batches": sb["batches"],
                     "compactions": sb["compactions"], "gc_runs": sb["gc_runs"],
                     "timed_region_compactions": st["compactions"], "timed_region_gc_runs": st["gc_runs"]}
    # The Resolver's verdict counters over the timed batches (Resolver.actor.cpp:206-208:
    # TransactionsAccepted / TooOld / Conflicted), combined over resolvers at N > 1
    def verdict_mix(lo, hi):
        mix = {"committed": 0, "conflict": 0, "too_old": 0}
        for i in range(lo, hi):
            v = combined[i].cpu().numpy() if (dist is not None and i in combined) else verdicts[i]
            if v is None:
                continue
            v = np.asarray(v)
            if dist is not None and i in combined:  # conflict bytes: 2 - min verdict, 0 = not routed anywhere
                v = np.where(v == 0, 2, 2 - v.astype(np.int64))
            mix["committed"] += int((v == 2).sum())
            mix["conflict"] += int((v == 0).sum())
            mix["too_old"] += int((v == 1).sum())
        return mix

    mix = verdict_mix(timed_lo, timed_hi)
    # the "total" pass adds every batch after the previous batch's detect was issued: the Resolver's
    # order (Resolver.actor.cpp:179-194), so its TooOld tests (SkipList.cpp:770) see the oldest
    # version the previous detect left; the timed pass packs its batches ahead of the region, so
    # its TooOld tests use the oldest version at pack time
    mix_total = verdict_mix(*spans["total"]) if n_total > 0 else None
    gtxn = pass_txns("timed")
    granges = sum(gbatches[i][0].n_reads + gbatches[i][0].n_writes for i in range(timed_lo, timed_hi))
    ttxn = pass_txns("total")
    hist_end = cs.history_size()
    cs.close()

    # Roofline.  The per-kernel table comes from the profile pass (events around every kernel);
    # the dominant kernel's line from the timed region's own events (fdbcs_set_timed_kernel).
    # Algorithmic bytes per launch: roofline.py (SURVEY §8(d) model per kernel, batch shapes of
    # this run).
    sample = [mine_at(i) for i in range(timed_lo, min(timed_hi, timed_lo + 8))]
    shape = roofline.shape_of(sample, st_prof if args.profile_steps > 0 else st, len(vers),
                              dir_share=directory_share(kb, ko, sample))
    table = roofline.kernel_table(kprof, shape, st_prof if args.profile_steps > 0 else None)
    roof = None
    if dominant and args.roof_steps > 0 and dominant not in kprof_timed:
        print(f"[rank {rank}] roofline pass timed no launch of {dominant!r} (timed: {sorted(kprof_timed)}, "
              f"batches {st_roof.get('batches')})", file=sys.stderr)
    if dominant and dominant in kprof_timed:
        k = kprof_timed[dominant]
        ent = roofline.entry(dominant, k["ms"], k["launches"], shape, st_roof)
        traffic, traffic_note = roofline.pmc_traffic(ROOT, args.workload, dominant, p.txns, p.history, build)
        rp = (rp_kernels or {}).get(dominant)
        rp_frac = None
        if rp and ent["algorithmic_bytes_per_launch"]:
            rp_frac = ent["algorithmic_bytes_per_launch"] / (rp["avg_us"] * 1e-6) / 1e9 / roofline.HBM_PEAK_GBS
        roof = {
            "kernel": dominant,
            "bound": "hbm",
            "achieved": ent["achieved_GBps"],
            "peak": roofline.HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": ent["frac"],
            "traffic": traffic,
            "traffic_source": traffic_note,
            "dominant_source": dominant_source,
            "build_id": build,
            "avg_launch_ms": ent["avg_launch_ms"],
            # the same kernel's rocprofv3 average (committed summary of this build and configuration)
            "rocprof_avg_launch_ms": rp["avg_us"] / 1e3 if rp else None,
            "frac_rocprof": rp_frac,
            "rocprof_source": rp_note,
            "launches_timed": k["launches"],
            "algorithmic_bytes_per_launch": ent["algorithmic_bytes_per_launch"],
            "model": ent["model"],
            "profile_avg_launch_ms": table.get(dominant, {}).get("avg_launch_ms"),
        }

    combine_check = None
    if dist is not None:
        # the device-side combine against host-built conflict bytes of the same verdicts
        bad = 0
        # (the same batches on every rank: the first 24 of the timed region and after)
        for i in sorted(k for k in combined if k >= timed_lo)[:24]:
            h = torch.from_numpy(KeyRangeSharding.conflict_bytes(gbatches[i][0].n_txn, routed_at(i), verdicts[i])).to(cdev)
            dist.all_reduce(h, op=dist.ReduceOp.MAX)
            bad += int(not torch.equal(h, combined[i]))
        combine_check = {"batches": len(sorted(k for k in combined if k >= timed_lo)[:24]), "mismatched": bad,
                         "path": (f"device conflict bytes + {'RCCL' if args.backend == 'nccl' else 'gloo'} MAX all-reduce"
                                  if on_device else "host bytes + all-reduce")}
    parity = cpu_base = None
    if not args.no_cpu_baseline:
        timed = set(range(timed_lo, timed_hi))
        parity, cpu_base = cpu_replay(args, kb, ko, vers, mine_at, gbatches, verdicts, timed, rank,
                                      add_oldest=add_oldest, sample_from=timed_lo)
        if dist is not None:
            t = torch.tensor([parity["batches_checked"], parity["mismatched_batches"], parity["mismatched_txns"]],
                             dtype=torch.int64, device=cdev)
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
            parity["batches_checked"], parity["mismatched_batches"], parity["mismatched_txns"] = (
                int(x) for x in t.tolist())
            parity["scope"] = f"{world} ranks, each against its own restatement fed the same routing"
            # G resolvers on G cores: every rank replayed its routed sub-batches on its own pinned
            # core at the same time; the global batches' transactions over the slowest rank's time
            spent = max_over_ranks(cpu_base["_spent"])
            cpu_base["value"] = cpu_base["_global_txns"] / spent if spent > 0 else None
            cpu_base["cores"] = world
            cpu_base["sample"] = (f"{cpu_base['_batches']} global batches from the timed region on, each rank replaying its routed "
                                  f"sub-batches on its own pinned core ({world} cores at once), slowest rank "
                                  f"{spent:.1f}s; " + cpu_base["sample"].split(", ", 1)[1])
        for k in ("_spent", "_global_txns", "_batches"):
            cpu_base.pop(k, None)

    cfg_desc = {
        "c1": "skipListTest (SkipList.cpp:1023-1077): 1R+1W per txn, setK 16-byte keys over [0, 2e7), empty initial "
        "history, now = v+50, newOldest = v",
        "c2": "5R+2W ranges/txn, 16-byte uniform keys",
        "c3": "5R+2W ranges/txn, YCSB Zipf(0.99) hot keys over 1M Mako-style 16-byte keys",
        "c4": "1 wide Tuple.range() read + 4 point reads + 2 point writes per txn, tuple keys (subspace, user string, "
        "int) up to 100 B",
    }[args.workload]
    dist_info = None
    if dist is not None:
        rccl = None
        try:
            rccl = ".".join(str(x) for x in torch.cuda.nccl.version())
        except Exception:
            pass
        dist_info = {"world_size": world, "backend": args.backend, "rccl_version": rccl,
                     "routing": ("device: each rank packs its share of the global batch (proxy), H2D, all-gather of "
                                 "the shares, fdbcs_batch_add_routed (k_route_wait, k_route_mark, k_scan<RouteScan>, k_route_write) per resolver, "
                                 "inside the timed region" if droute else
                                 "host (balancing.BalancedRouting) before the timed region: a feature check, not a "
                                 "throughput figure"),
                     "share_stride_bytes": stride or None,
                     # the routing kernels' device time and the host time of fdbcs_batch_add_routed per
                     # batch, over the timed region (the all-gather is not included: RCCL's own kernels)
                     "route_kernels_ms_per_batch": st["ms_route_kernels"] / max(1, st["routed_batches"]) if droute else None,
                     "route_host_ms_per_batch": st["host_ms_route"] / max(1, st["routed_batches"]) if droute else None}
    out = {
        "metric": "resolved txns/sec (conflict ranges checked/sec) per batch; HBM GB/s vs peak",
        "value": gtxn / elapsed,
        "unit": "txns/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8/int64 (byte keys, int64 versions)",
        "data": "synthetic",
        "config": {
            "workload": f"{args.workload.upper()}: {p.txns}-txn batches per GPU, {cfg_desc}, "
            + (f"{p.history}-boundary MVCC history per GPU (5e6-version window)" if p.history else "no prefill"),
            "global_batch_txns": p.txns * world,
            "parallelism": f"key-range shards x{world}" if world > 1 else "single resolver",
            "timed_region": "per batch: all kernels and the verdict bytes in host memory, the packed batch resident "
            f"in HBM when the region starts ({WINDOW} batches in flight); addTransaction packing and the H2D copy "
            "outside (reference 'Detect only'); h2d_inclusive_txns_per_s: the H2D inside the loop",
            "gc_interval": args.gc_interval,
            "delta_limit": args.delta_limit or "auto",
        },
        "conflict_ranges_per_s": granges / elapsed,
        "total_txns_per_s": ttxn / total_elapsed if total_elapsed else None,
        "total_host_ms_per_batch": total_host,
        "h2d_inclusive_txns_per_s": pass_txns("h2d") / h2d_elapsed if h2d_elapsed else None,
        "sync": sync,
        "sync_txns_per_s": sync["txns_per_s"] if sync else None,
        "device_bound": device_bound,
        "host_ms_per_batch": host_timed,
        "total_note": "reference 'total' (SkipList.cpp:1082-1085): addTransaction + detect, per batch in the loop",
        "parity": parity,
        "combine_check": combine_check,
        "distributed": dist_info,
        "reshard": reshard,
        "history_boundaries_end": hist_end,
        "phase_ms_per_batch": phase,
        "amortized_ms_per_batch": amortized,
        "verdict_mix": mix,
        "verdict_mix_total": mix_total,
        "verdict_mix_note": "verdict_mix: timed batches, packed (addTransaction, TooOld test) before the region; "
        "verdict_mix_total: the total pass, each batch added after the previous detect (the Resolver's order)",
        "roofline_pass_txns_per_s": pass_txns("roof") / roof_elapsed if roof_elapsed else None,
        "compactions": st["compactions"],
        # batch-order launches (k_resolve, k_combine, k_intra_report) left out of the timed batches'
        # X halves: the host had seen their stage A find no candidate edge
        "x_launches_skipped": st["x_launches_skipped"],
        "kernels": table,
        "sort_phase": roofline.sort_phase(table),
        "roofline": roof,
    }
    if rank == 0:
        out["cpu_baseline"] = cpu_base
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
