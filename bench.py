#!/usr/bin/env python3
"""Benchmark: resolved transactions/s of the MI355X conflict-resolution engine.

Workload (BASELINE.json configs[1], "C2"): a single-MI355X resolver with 5000-transaction commit
batches, 5 read + 2 write conflict ranges per transaction, 16-byte uniform keys, over a
5M-boundary MVCC history prefilled across a 5e6-version window.  A step is one
ConflictBatch::detectConflicts pass (SkipList.cpp:844-890) over one batch, inputs already resident
in HBM (uploaded before the timed region).

N > 1 (torchrun, one rank per GPU): the key space is range-sharded across ranks like FDB's
multi-resolver split (CommitProxyServer.actor.cpp:147-174).  Every rank builds the same global batch
of N x 5000 transactions, keeps its routed sub-batch, resolves it on its GPU, and the verdicts are
combined by an RCCL all-reduce MAX of conflict bytes (= proxy min over resolvers,
CommitProxyServer.actor.cpp:772-777).  Weak scaling: per-GPU work is fixed.

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

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--txns", type=int, default=5000)
    ap.add_argument("--history", type=int, default=0,
                    help="history boundaries per GPU; 0 = the workload's (5M for c2/c3, 50M for c4)")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--gc-interval", type=int, default=0,
                    help="force a compaction (+GC) at least every N batches; 0 = when the delta tier is full")
    ap.add_argument("--delta-limit", type=int, default=0, help="delta-tier bound; 0 = automatic (~base/16)")
    ap.add_argument("--timing", type=int, default=1, choices=[0, 1],
                    help="events in the timed region: 0 none, 1 around the copy kernels (roofline)")
    ap.add_argument("--breakdown-steps", type=int, default=16,
                    help="extra batches after the timed region with every phase timed (diagnostic)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="bounded CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--workload", default="c2", choices=["c2", "c3", "c4"])
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="collective backend for the verdict all-reduce (nccl = RCCL over xGMI)")
    return ap.parse_args()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def workload_params(args):
    from foundationdb_amd import workloads as W

    if args.workload == "c4":
        return W.C4Params(txns=args.txns, history=args.history or 50_000_000)
    return W.C2Params(txns=args.txns, history=args.history or 5_000_000)


def sharding_for(args, p, world):
    from foundationdb_amd import workloads as W
    from foundationdb_amd.sharding import KeyRangeSharding

    if world == 1:
        return None
    if args.workload == "c4":  # every key shares the subspace: split by user
        return KeyRangeSharding([W.c4_user_split(p, g * p.users // world) for g in range(1, world)])
    return KeyRangeSharding.uniform(world)


def shard_history(args, p, seed, rank, world, start_version):
    """Prefill: p.history boundaries inside this rank's key range."""
    from foundationdb_amd.workloads import c2_history, c4_history

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


def make_batches(args, p, n_batches, world, start_version):
    """Global batches (identical on every rank) with their (now, newOldest)."""
    from foundationdb_amd import workloads as W

    import dataclasses

    rng = np.random.default_rng(args.seed)
    zipf = W.ZipfGenerator(1_000_000, 0.99) if args.workload == "c3" else None
    gp = dataclasses.replace(p, txns=args.txns * world)
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


def cpu_baseline(args, p, kb, ko, vers, batches):
    """Skip-list restatement of the reference (oracle/skiplist_baseline.cpp), single thread,
    over a bounded sample of the same workload."""
    from oracle import oracle

    oracle.build()
    sl = oracle.SkipListBaseline()
    t0 = time.time()
    sl.load_history(kb, ko, vers)
    load_s = time.time() - t0
    done_txn = 0
    done_batches = 0
    spent = 0.0
    for pb, now, no in batches:
        t = time.perf_counter()
        sl.detect(pb, now, no)
        spent += time.perf_counter() - t
        done_txn += pb.n_txn
        done_batches += 1
        if spent >= args.cpu_seconds:
            break
    cpu = platform.processor() or platform.machine()
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {
        "value": done_txn / spent if spent > 0 else None,
        "unit": "txns/s",
        "cores": 1,
        "kind": "port",
        "sample": f"{done_batches} {args.workload.upper()} batches x {args.txns} txns on a {len(vers)}-boundary history "
        f"({spent:.1f}s CPU, load {load_s:.1f}s), skip-list restatement oracle/skiplist_baseline.cpp, "
        f"1 thread on {cpu}",
    }


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch

    dist = None
    ndev = max(1, torch.cuda.device_count())
    device = local % ndev  # one rank per GPU; more ranks than GPUs only for rehearsals (gloo)
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(device)
        dist.init_process_group(args.backend)
    cdev = "cuda" if args.backend == "nccl" else "cpu"
    from foundationdb_amd import build as fbuild

    fbuild.build()
    from foundationdb_amd import conflict_set as C
    from foundationdb_amd import workloads as W
    from foundationdb_amd.sharding import KeyRangeSharding

    p = workload_params(args)
    start_version = 10_000_000
    t0 = time.time()
    kb, ko, vers = shard_history(args, p, args.seed, rank, world, start_version)
    total = args.warmup + args.steps
    n_all = total + args.breakdown_steps
    gbatches = make_batches(args, p, n_all, world, start_version)
    sharding = sharding_for(args, p, world)
    routed = [sharding.route(pb)[rank] for pb, _, _ in gbatches] if sharding else None
    log(f"[rank {rank}] generated history {len(vers)} + {n_all} batches in {time.time() - t0:.1f}s")

    cs = C.ConflictSet(device)
    cs.set_gc_interval(args.gc_interval)
    cs.set_delta_limit(args.delta_limit)
    cs.set_timing(args.timing)
    cs.load_history(kb, ko, vers, 0)
    mine = [r.batch for r in routed] if routed else [pb for pb, _, _ in gbatches]
    maxT = max(b.n_txn for b in mine)
    maxR = max(b.n_reads for b in mine)
    maxW = max(b.n_writes for b in mine)
    def tail_bytes(ko):
        return int(np.maximum(np.diff(ko) - 16, 0).sum())

    tail_total = tail_bytes(ko) + sum(tail_bytes(b.key_offsets) for b in mine) + (1 << 20)
    cs.reserve(len(vers) + 2 * sum(b.n_writes for b in mine) + 1024, tail_total, maxT, maxR, maxW)
    objs = []
    for b in mine:
        o = C.ConflictBatch(cs)
        o.add_packed(b)
        o.upload()
        objs.append(o)
    torch.cuda.synchronize()

    def run(lo, hi, combine):
        for i in range(lo, hi):
            _, now, no = gbatches[i]
            objs[i].detect_async(now, no)
        for i in range(lo, hi):
            v = objs[i].wait()
            if combine:
                T = gbatches[i][0].n_txn
                c = torch.from_numpy(KeyRangeSharding.conflict_bytes(T, routed[i], v)).to(cdev)
                dist.all_reduce(c, op=dist.ReduceOp.MAX)

    run(0, args.warmup, dist is not None)
    torch.cuda.synchronize()
    cs.reset_stats()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    run(args.warmup, total, dist is not None)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    st = cs.stats()
    # diagnostic phase split: extra batches with every phase timed (each event costs queue time,
    # so these are outside the timed region)
    phase = None
    if args.breakdown_steps > 0:
        cs.set_timing(2)
        cs.reset_stats()
        run(total, n_all, dist is not None)
        torch.cuda.synchronize()
        sb = cs.stats()
        phase = {
            k: sb[k] / max(1, sb["batches"])
            for k in ("ms_check_read", "ms_sort", "ms_intra", "ms_combine", "ms_merge", "ms_compact", "ms_gc",
                      "ms_epilogue", "ms_total")
        }
        phase["batches"] = sb["batches"]
        phase["compactions"] = sb["compactions"]
        phase["intra_edges"] = sb["intra_edges"] / max(1, sb["batches"] - sb["intra_fallbacks"])
        phase["intra_rounds"] = sb["intra_rounds"] / max(1, sb["batches"] - sb["intra_fallbacks"])
        phase["intra_fallbacks"] = sb["intra_fallbacks"]
    gtxn = sum(gbatches[i][0].n_txn for i in range(args.warmup, total))
    granges = sum(gbatches[i][0].n_reads + gbatches[i][0].n_writes for i in range(args.warmup, total))
    hist_end = cs.history_size()

    # Dominant kernel: of the two copy kernels (delta merge every batch, compaction of the base every
    # ~16 batches) the one with the larger total device time; both are HBM-bound rewrites of a
    # sorted boundary array reading 32 B per old boundary and writing 32 B per kept one.
    kernels = {
        "merge": ("k_merge_copy<BatchIns> (delta-tier merge)", st["ms_merge_kernel"], st["merge_launches"],
                  st["merge_bytes"]),
        "compact": ("k_merge_copy<CompactIns> (base-tier compaction)", st["ms_compact_kernel"], st["compactions"],
                    st["compact_bytes"]),
    }
    dom = max(kernels, key=lambda k: kernels[k][1])
    kname, kms, klaunch, kbytes = kernels[dom]
    launches = max(1, klaunch)
    avg_ms = kms / launches
    bytes_per_launch = kbytes / launches
    achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    traffic = None
    # PMC HBM bytes per launch (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE, separate rocprofv3
    # passes: scripts/gpu_pmc.sh) of this workload's copy kernels, measured on the same command
    pmc = os.path.join(ROOT, "profiles", f"pmc_traffic_{args.workload}.json")
    if os.path.exists(pmc):
        try:
            with open(pmc) as f:
                traffic = json.load(f).get(f"{dom}_bytes_per_launch")
        except Exception:
            traffic = None
    other = kernels["compact" if dom == "merge" else "merge"]

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
            "workload": f"{args.workload.upper()}: {args.txns}-txn batches per GPU, 5R+2W ranges/txn, "
            + {"c2": "16-byte uniform keys", "c3": "YCSB Zipf(0.99) hot keys over 1M Mako-style 16-byte keys",
               "c4": "tuple keys (subspace, user string, int) up to 100 B, 1 wide Tuple.range() read per txn"}[
                args.workload]
            + f", {p.history}-boundary MVCC history per GPU (5e6-version window)",
            "global_batch_txns": args.txns * world,
            "parallelism": f"key-range shards x{world}" if world > 1 else "single resolver",
            "gc_interval": args.gc_interval,
            "delta_limit": args.delta_limit or "auto",
        },
        "conflict_ranges_per_s": granges / elapsed,
        "history_boundaries_end": hist_end,
        "phase_ms_per_batch": phase,
        "compactions": st["compactions"],
        "other_copy_kernel": {
            "kernel": other[0],
            "launches": other[2],
            "avg_launch_ms": other[1] / max(1, other[2]),
            "achieved_GBps": (other[3] / max(1, other[2])) / (other[1] / max(1, other[2]) * 1e-3) / 1e9
            if other[1] > 0 else None,
        },
        "roofline": {
            "kernel": kname,
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            "avg_launch_ms": avg_ms,
            "algorithmic_bytes_per_launch": bytes_per_launch,
        },
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args, p, kb, ko, vers, gbatches[args.warmup :])
    elif rank == 0:
        out["cpu_baseline"] = None
    for o in objs:
        o.close()
    cs.close()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
