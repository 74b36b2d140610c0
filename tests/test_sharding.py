"""Multi-resolver (key-range sharded) path on CPU: routing restates CommitProxyServer.actor.cpp:118-187,
the combine restates determineCommittedTransactions (:764-780), and a world_size-2 gloo run with one
resolver per rank reproduces G sequential resolvers fed by the same routing."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from foundationdb_amd import workloads as W
from foundationdb_amd.packing import CommitTransaction, KeyRange, PackedBatch
from foundationdb_amd.sharding import KeyRangeSharding


def _batches(seed, n=6, txns=80):
    rng = np.random.default_rng(seed)
    out = []
    now = 10
    for _ in range(n):
        pb = W.random_small_batch(rng, txns, alphabet=256, max_len=2, now=now, staleness=10, report_frac=0.0)
        out.append((pb, now, now - 5))
        now += 3
    return out


def test_routing_matches_intersecting_ranges():
    sh = KeyRangeSharding.uniform(4)
    slow = KeyRangeSharding([bytes([64]), bytes([128]), bytes([192])])
    slow._byte_splits = None  # force the generic bisect path
    for pb, _, _ in _batches(1, n=3):
        fast_parts, slow_parts = sh.route(pb), slow.route(pb)
        for a, b in zip(fast_parts, slow_parts):
            assert (a.txn_ids == b.txn_ids).all()
            assert (a.batch.key_bytes == b.batch.key_bytes).all()
        # every range lands on exactly the shards it intersects (unclipped)
        for r in range(pb.n_reads):
            rr = pb.read_range(r)
            for g in range(4):
                lo, hi = sh.shard_bounds(g)
                inter = (hi is None or rr.begin < hi) and (rr.end > lo or (rr.empty() and rr.begin >= lo))
                t = int(np.searchsorted(pb.read_offsets, r, side="right") - 1)
                got = t in set(fast_parts[g].txn_ids.tolist())
                if inter:
                    assert got


def test_single_shard_is_identity():
    sh = KeyRangeSharding.uniform(1)
    for pb, _, _ in _batches(2, n=2):
        part = sh.route(pb)[0]
        has_range = (np.diff(pb.read_offsets) + np.diff(pb.write_offsets)) > 0
        assert (part.txn_ids == np.nonzero(has_range)[0]).all()


def test_combine_is_min_over_resolvers():
    T = 5
    from foundationdb_amd.sharding import ShardBatch

    a = ShardBatch(None, np.array([0, 1, 2]), None)
    b = ShardBatch(None, np.array([1, 2, 3]), None)
    v = KeyRangeSharding.combine(T, [a, b], [np.array([2, 1, 2]), np.array([0, 2, 1])])
    # txn0: only a -> 2; txn1: min(1,0)=0; txn2: min(2,2)=2; txn3: only b -> 1; txn4: routed nowhere -> 2
    assert v.tolist() == [2, 0, 2, 1, 2]


def _sequential_reference(batches, G, oracle):
    sh = KeyRangeSharding.uniform(G)
    sets = [oracle.OracleConflictSet() for _ in range(G)]
    out = []
    for pb, now, no in batches:
        parts = sh.route(pb)
        vs = [sets[g].detect(parts[g].batch, now, no)[0] for g in range(G)]
        out.append(KeyRangeSharding.combine(pb.n_txn, parts, vs))
    return out


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, seed, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle

    sh = KeyRangeSharding.uniform(world)
    cs = oracle.OracleConflictSet()
    res = []
    for pb, now, no in _batches(seed):
        part = sh.route(pb)[rank]
        v, _ = cs.detect(part.batch, now, no)
        c = torch.from_numpy(KeyRangeSharding.conflict_bytes(pb.n_txn, part, v).astype(np.int32))
        dist.all_reduce(c, op=dist.ReduceOp.MAX)
        res.append((2 - c.numpy()).astype(np.uint8))
    if rank == 0:
        q.put([r.tolist() for r in res])
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_matches_sequential_resolvers(oracle_built):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, 5, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = _sequential_reference(_batches(5), 2, oracle_built)
    assert got == [w.tolist() for w in want]


def test_sharded_verdicts_are_conservative(oracle_built):
    """Routing may only add conflicts relative to one resolver (architecture.rst:247-258): a
    transaction committed by the sharded resolvers is committed by a single resolver too when
    every transaction's ranges live in one shard."""
    rng = np.random.default_rng(3)
    sh = KeyRangeSharding.uniform(2)
    single = oracle_built.OracleConflictSet()
    sets = [oracle_built.OracleConflictSet() for _ in range(2)]
    now = 10
    for _ in range(6):
        txns = []
        for _ in range(60):
            half = int(rng.integers(0, 2)) * 128

            def key():
                return bytes([half + int(rng.integers(0, 4))]) + bytes(rng.integers(0, 3, size=int(rng.integers(0, 2))).astype(np.uint8))

            def rr():
                a, b = key(), key()
                return KeyRange(min(a, b), max(a, b))

            txns.append(CommitTransaction([rr() for _ in range(2)], [rr()], now - int(rng.integers(0, 6))))
        pb = PackedBatch.from_transactions(txns)
        parts = sh.route(pb)
        vs = [sets[g].detect(parts[g].batch, now, now - 4)[0] for g in range(2)]
        comb = KeyRangeSharding.combine(pb.n_txn, parts, vs)
        v1, _ = single.detect(pb, now, now - 4)
        assert (comb == v1).all()  # disjoint shards: identical to one resolver
        now += 2
