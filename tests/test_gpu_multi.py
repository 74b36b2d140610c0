"""The multi-GPU bench path, rehearsed on one GPU: two ranks (gloo, since RCCL refuses two ranks
on one card) each resolve their key-range shard with the HIP engine, scatter conflict bytes on
the device and all-reduce them; every rank's verdicts must equal its own CPU restatement fed the
same routing, and the device-side combine must equal the host-built one."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,workload,extra", [(2, "c2", []), (2, "c3", []),
                                                  (2, "c3", ["--reshard", "--reshard-preroll", "60"]),
                                                  (8, "c2", [])])
def test_multi_rank_bench_parity(engine, world, workload, extra):
    """bench.py's N-rank path rehearsed on one GPU over gloo (RCCL refuses several ranks on one
    card): 2 ranks, and the 8-way split of C5 with 500-transaction shares."""
    txns, history = ("1000", "200000") if world == 2 else ("500", "50000")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", str(world), "--workload", workload, "--steps", "8", "--warmup", "2", "--txns", txns,
           "--history", history, "--h2d-steps", "0", "--total-steps", "0", "--breakdown-steps", "0",
           "--profile-steps", "4", "--sync-steps", "4", "--roof-steps", "0", "--backend", "gloo",
           "--cpu-seconds", "20"] + extra
    env = dict(os.environ, OMP_NUM_THREADS="1" if world > 2 else "2")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=280 if world > 2 else 110)
    assert r.returncode == 0, "\n".join([l for l in r.stderr.splitlines() if "[rank1]" in l][-30:]) + r.stderr[-1500:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    out = json.loads(line)
    assert out["n_gpus"] == world and out["value"] > 0
    # warmup 2 + timed 8 + profile 4 + sync 4 batches, every one combined and replayed on each rank
    assert out["parity"]["batches_checked"] >= world * 18 and out["parity"]["mismatched_batches"] == 0
    # the combine check covers the timed and later batches (timed 8 + profile 4 + sync 4)
    assert out["combine_check"]["mismatched"] == 0 and out["combine_check"]["batches"] == 16
    # G resolvers on G cores: every rank's restatement timed at once, over the slowest one
    assert out["cpu_baseline"]["cores"] == world and out["cpu_baseline"]["value"] > 0
    assert out["distributed"]["world_size"] == world and out["distributed"]["backend"] == "gloo"
    assert out["combine_check"]["path"].startswith("device conflict bytes")
    if extra:
        assert out["reshard"]["moves"] > 0  # the hot rank gave key ranges away
    else:  # the proxy's split ran on the GPUs inside the timed region
        assert out["distributed"]["routing"].startswith("device")


@pytest.mark.parametrize("G,alphabet,max_len,long_split", [(2, 6, 3, False), (3, 200, 3, False), (4, 5, 24, True),
                                                           (1, 6, 3, False)])
def test_device_routing_matches_host_routing(engine, G, alphabet, max_len, long_split):
    """fdbcs_batch_add_routed against the host routing (sharding.KeyRangeSharding.route,
    CommitProxyServer.actor.cpp:118-187): G resolvers on one GPU, each routing the same gathered
    shares; sizes, verdicts (vs a restatement per resolver fed the host routing) and the device
    conflict bytes (vs host-built ones) must be equal, over batches with empty and touching ranges,
    empty keys, keys equal to split keys, long keys and TooOld transactions."""
    import numpy as np
    import torch

    from foundationdb_amd import workloads as W
    from foundationdb_amd.sharding import KeyRangeSharding
    from oracle import oracle as O

    O.build()
    rng = np.random.default_rng(100 + G + alphabet)
    Tshare = 120
    # split keys: short ones at alphabet letters (keys equal to them occur), one long one
    letters = sorted(set(int(x) for x in rng.integers(1, alphabet, size=3 * G)))[: G - 1]
    while len(letters) < G - 1:
        letters.append(letters[-1] + 1 if letters else 1)
    splits = [bytes([x]) for x in sorted(set(letters))][: G - 1]
    if long_split and G > 2:
        splits[1] = bytes([splits[1][0]] * 20)  # > 16 bytes: tail comparisons against the bound
        splits = sorted(set(splits))
    sh = KeyRangeSharding(splits)  # G = 1: one resolver still gets only transactions with ranges (:107-116)
    sets = [engine.ConflictSet(0) for _ in range(G)]
    oras = [O.OracleConflictSet() for _ in range(G)]
    now = 10
    for step in range(10):
        pb = W.random_small_batch(rng, G * Tshare, alphabet=alphabet, max_len=max_len, now=now, staleness=12)
        shares = [engine.share_pack(pb.slice_txns(g * Tshare, (g + 1) * Tshare)) for g in range(G)]
        stride = (max(len(x) for x in shares) + 255) // 256 * 256
        host = np.zeros(G * stride, np.uint8)
        for g, x in enumerate(shares):
            host[g * stride: g * stride + len(x)] = x
        dev = torch.from_numpy(host).cuda()
        # the gathered shares' ready flag, set on torch's stream (another HIP runtime) after the
        # copy; odd steps pass none, the shares being complete once torch has synchronised
        ready = torch.zeros(1, dtype=torch.int32, device="cuda")
        ready.fill_(step + 1)
        if step % 2:
            torch.cuda.synchronize()
        flag = (ready.data_ptr(), step + 1) if step % 2 == 0 else (0, 0)
        routes = sh.route(pb)
        tail = int(np.maximum(np.diff(pb.key_offsets) - 16, 0).sum())
        out = [torch.full((pb.n_txn,), 7, dtype=torch.uint8, device="cuda") for _ in range(G)]
        for g in range(G):
            lo = splits[g - 1] if g > 0 else None
            hi = splits[g] if g < G - 1 else None
            b = engine.ConflictBatch(sets[g])
            b.add_routed(dev.data_ptr(), stride, G, Tshare, lo, hi, (pb.n_txn, pb.n_reads, pb.n_writes, tail),
                         out[g].data_ptr(), pb.n_txn, *flag)
            sub = routes[g].batch
            T, R, Wn, _, _ = b.routed_info()
            # every kept range is placed, TooOld sub-transactions' included (their TooOld test,
            # SkipList.cpp:770, is made at detect time)
            nr, nw = np.diff(sub.read_offsets), np.diff(sub.write_offsets)
            assert (T, R, Wn) == (sub.n_txn, int(nr.sum()), int(nw.sum()))
            b.detect_async(now, now - 9)
            got = b.wait()
            b.close()
            want, _ = oras[g].detect(sub, now, now - 9)
            np.testing.assert_array_equal(got, want)
            ids = routes[g].txn_ids
            ref = np.zeros(pb.n_txn, np.uint8)
            ref[ids] = 2 - want.astype(np.uint8)
            np.testing.assert_array_equal(out[g].cpu().numpy(), ref)
        now += 4
    for cs in sets:
        cs.close()


def _route_and_gather(engine, torch, np, pb, G, Tshare):
    shares = [engine.share_pack(pb.slice_txns(g * Tshare, (g + 1) * Tshare)) for g in range(G)]
    stride = (max(len(x) for x in shares) + 255) // 256 * 256
    host = np.zeros(G * stride, np.uint8)
    for g, x in enumerate(shares):
        host[g * stride: g * stride + len(x)] = x
    return torch.from_numpy(host).cuda(), stride


@pytest.mark.parametrize("G,workload", [(8, "c2"), (8, "c3"), (4, "c2")])
def test_pipelined_device_routing_eight_resolvers(engine, G, workload):
    """The 8-way key-range split on one card (C5 shape, CommitProxyServer.actor.cpp:107-187,
    764-780): G resolvers route C2/C3-shaped global batches on the device in bench.py's order (batch
    i+1 routed before batch i's detect), with snapshots straddling the oldest version as it moves.
    Each resolver's verdicts equal its own restatement fed the host routing in the Resolver's
    order (add after the previous detect: TooOld against the oldest that detect left,
    SkipList.cpp:770, 880-882), and the device conflict bytes max-combined over the resolvers equal
    the host combine (the proxy's min over verdicts)."""
    import numpy as np
    import torch

    from foundationdb_amd import workloads as W
    from foundationdb_amd.sharding import KeyRangeSharding
    from oracle import oracle as O

    O.build()
    rng = np.random.default_rng(800 + G)
    Tshare = 250
    p = W.C2Params(txns=G * Tshare, staleness=60)
    sh = KeyRangeSharding.uniform(G) if workload == "c2" else KeyRangeSharding(
        [W.mako_keys(np.array([g * 1_000_000 // G]))[0].tobytes() for g in range(1, G)])
    z = W.ZipfGenerator(1_000_000, 0.99) if workload == "c3" else None
    sets = [engine.ConflictSet(0) for _ in range(G)]
    oras = [O.OracleConflictSet() for _ in range(G)]
    now = 1000
    pending = None
    saw_too_old = 0
    too_old_window = 0

    def finish(pend):
        pb_, now_, no_, objs, outs = pend
        routes = sh.route(pb_)
        comb = np.zeros(pb_.n_txn, np.uint8)
        want_comb = np.zeros(pb_.n_txn, np.uint8)
        nonlocal saw_too_old, too_old_window
        for g in range(G):
            objs[g].detect_async(now_, no_)
        for g in range(G):
            got = objs[g].wait()
            objs[g].close()
            sub = routes[g].batch
            old_before = oras[g].oldest_version
            want, _ = oras[g].detect(sub, now_, no_)
            np.testing.assert_array_equal(got, want, err_msg=f"resolver {g}")
            saw_too_old += int((want == 1).sum())
            # TooOld only because the previous detect raised the oldest version
            too_old_window += int(((want == 1) & (sub.read_snapshot >= old_before - 4)).sum())
            comb = np.maximum(comb, outs[g].cpu().numpy())
            want_comb = np.maximum(want_comb, KeyRangeSharding.conflict_bytes(pb_.n_txn, routes[g], want))
        np.testing.assert_array_equal(comb, want_comb)

    for step in range(8):
        now += 4
        pb = W.c3_batch(p, rng, now, z) if z else W.c2_batch(p, rng, now)
        dev, stride = _route_and_gather(engine, torch, np, pb, G, Tshare)
        tail = int(np.maximum(np.diff(pb.key_offsets) - 16, 0).sum())
        objs, outs = [], []
        for g in range(G):
            lo = sh.splits[g - 1] if g > 0 else None
            hi = sh.splits[g] if g < G - 1 else None
            out = torch.full((pb.n_txn,), 7, dtype=torch.uint8, device="cuda")
            b = engine.ConflictBatch(sets[g])
            b.add_routed(dev.data_ptr(), stride, G, Tshare, lo, hi, (pb.n_txn, pb.n_reads, pb.n_writes, tail),
                         out.data_ptr(), pb.n_txn)
            objs.append(b)
            outs.append(out)
        if pending is not None:  # the previous batch's detect after this batch's routing
            finish(pending)
        pending = (pb, now, now - 30, objs, outs)
    finish(pending)
    assert saw_too_old > 0 and too_old_window > 0
    for cs in sets:
        cs.close()


def test_routed_batch_errors_leave_it_empty_and_reroutable(engine, monkeypatch):
    """fdbcs_batch_add_routed's error paths: a ready flag that is never set times out
    (FDBCS_E_TIMEOUT after FDBCS_ROUTE_TIMEOUT_MS), and n_global differing from the shares'
    transaction count fails (FDBCS_E_INVALID); either way the batch is empty again, and routing it
    anew with correct arguments detects exactly like the host routing's restatement."""
    import numpy as np
    import torch

    from foundationdb_amd import workloads as W
    from foundationdb_amd.sharding import KeyRangeSharding
    from oracle import oracle as O

    O.build()
    monkeypatch.setenv("FDBCS_ROUTE_TIMEOUT_MS", "50")
    cs = engine.ConflictSet(0)
    ora = O.OracleConflictSet()
    rng = np.random.default_rng(77)
    Tshare = 100
    pb = W.random_small_batch(rng, Tshare, alphabet=6, max_len=3, now=10, staleness=12)
    dev, stride = _route_and_gather(engine, torch, np, pb, 1, Tshare)
    tail = int(np.maximum(np.diff(pb.key_offsets) - 16, 0).sum())
    caps = (pb.n_txn, pb.n_reads, pb.n_writes, tail)
    out = torch.zeros(pb.n_txn, dtype=torch.uint8, device="cuda")
    never = torch.zeros(1, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    b = engine.ConflictBatch(cs)
    # 1. the shares' ready flag is never set: bounded wait, then FDBCS_E_TIMEOUT
    b.add_routed(dev.data_ptr(), stride, 1, Tshare, None, None, caps, out.data_ptr(), pb.n_txn, never.data_ptr(), 5)
    with pytest.raises(engine.FdbcsError) as e:
        b.routed_info()
    assert e.value.status == engine.FDBCS_E_TIMEOUT
    # 2. n_global differs from the shares' transaction count: FDBCS_E_INVALID, batch empty again
    # (more than the shares can hold is refused on the host at once; fewer is found on the device)
    with pytest.raises(engine.InvertedRange):
        b.add_routed(dev.data_ptr(), stride, 1, Tshare, None, None, caps, out.data_ptr(), pb.n_txn + 3)
    b.add_routed(dev.data_ptr(), stride, 1, Tshare, None, None, caps, out.data_ptr(), pb.n_txn - 3)
    with pytest.raises(engine.FdbcsError) as e:
        b.routed_info()
    assert e.value.status == engine.FDBCS_E_INVALID
    # 3. routed anew, correctly: the same verdicts as the restatement
    b.add_routed(dev.data_ptr(), stride, 1, Tshare, None, None, caps, out.data_ptr(), pb.n_txn)
    b.detect_async(10, 1)
    got = b.wait()
    b.close()
    route = KeyRangeSharding([]).route(pb)[0]  # one resolver: transactions with at least one range
    want, _ = ora.detect(route.batch, 10, 1)
    np.testing.assert_array_equal(got, want)
    ref = np.zeros(pb.n_txn, np.uint8)
    ref[route.txn_ids] = 2 - want.astype(np.uint8)
    np.testing.assert_array_equal(out.cpu().numpy(), ref)
    cs.close()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("workload", ["c2", "c3"])
def test_rccl_leg_one_rank(engine, workload):
    """C5's RCCL leg executed on one MI355X: torchrun with one rank and the
    nccl backend (RCCL), --dist forcing the multi-resolver path at world size 1 -- the proxy's
    share packed, H2D, all_gather_into_tensor over RCCL, the ready-flag hand-off from torch's HIP
    runtime to the engine's, fdbcs_batch_add_routed on the device, the device conflict bytes and
    their uint8 all_reduce(MAX) over RCCL (CommitProxyServer.actor.cpp:764-780).  Parity against
    the restatement fed the same routing, the device combine against host-built bytes."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "1", "--dist", "--backend", "nccl", "--workload", workload, "--steps", "12", "--warmup", "2",
           "--txns", "2000", "--history", "300000", "--h2d-steps", "0", "--total-steps", "4",
           "--breakdown-steps", "2", "--profile-steps", "4", "--sync-steps", "4", "--hold-steps", "2",
           "--roof-steps", "8", "--too-old-frac", "0.05", "--cpu-seconds", "30"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    d = out["distributed"]
    assert d["world_size"] == 1 and d["backend"] == "nccl" and d["rccl_version"]
    assert d["routing"].startswith("device")
    assert "RCCL" in out["combine_check"]["path"] and out["combine_check"]["mismatched"] == 0
    assert out["combine_check"]["batches"] >= 12
    # warmup 2 + profile 4 + timed 12 + total 4 + sync 4 + breakdown 2, every batch routed on the
    # device; the 2 hold-pass batches are never resolved on this path (no hold pass under a process
    # group), so the replay must leave them out of its history too
    assert out["parity"]["batches_checked"] >= 28 and out["parity"]["mismatched_batches"] == 0
    assert out["verdict_mix"]["too_old"] > 0
