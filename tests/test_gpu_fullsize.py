"""GPU parity at the BASELINE configurations' full sizes, on the measured path.

Every test drives the engine the way bench.py does (detect_async with several batches in flight,
three rotating workspaces, stage A running ahead, size-triggered compaction and GC) and compares
every verdict with the CPU restatement of the reference (oracle/skiplist_baseline.cpp, itself
cross-checked against the semantic oracle in test_oracle.py).  A second, independent model, a
key-space brute force over committed write ranges, pins verdicts and conflicting-key reports
(ConflictRange / ReportConflictingKeys workload properties, fdbserver/workloads/
ConflictRange.actor.cpp:226-316, ReportConflictingKeys.actor.cpp:201-278).
"""
import time

import numpy as np
import pytest

from foundationdb_amd import workloads as W
from foundationdb_amd.packing import CommitTransaction, KeyRange, PackedBatch

pytestmark = pytest.mark.gpu

WINDOW = 8


@pytest.fixture(scope="module")
def oracle_mod():
    from oracle import oracle

    oracle.build()
    return oracle


def pipeline(engine, cs, seq, on_done, window=WINDOW):
    """Submit (pb, now, newOldest) batches with `window` in flight; on_done(i, verdicts) in order."""
    inflight = []
    for i, (pb, now, no) in enumerate(seq):
        b = engine.ConflictBatch(cs)
        b.add_packed(pb)
        b.detect_async(now, no)
        inflight.append((i, b))
        if len(inflight) > window:
            j, bj = inflight.pop(0)
            on_done(j, bj.wait())
            bj.close()
    for j, bj in inflight:
        on_done(j, bj.wait())
        bj.close()


def check_against_restatement(oracle_mod, kb, ko, vers, seq, got, gc="bounded"):
    sl = oracle_mod.SkipListBaseline()
    if len(vers):
        sl.load_history(kb, ko, vers)
    for i, (pb, now, no) in enumerate(seq):
        v, _ = sl.detect(pb, now, no, gc=gc)
        bad = np.nonzero(got[i] != v)[0]
        assert len(bad) == 0, (i, bad[:10], got[i][bad[:10]], v[bad[:10]])
    return sl


@pytest.mark.parametrize("submit_thread", ["0", "1"])
def test_async_pipeline_full_c2(engine, oracle_mod, monkeypatch, submit_thread):
    """C2 at full size (5M-boundary history, 5000 txns x 5R+2W) through the async pipeline for 72
    batches: crosses several size-triggered compactions and a removeBefore pass; with one and with
    two submitting threads (FDBCS_SUBMIT_THREAD)."""
    monkeypatch.setenv("FDBCS_SUBMIT_THREAD", submit_thread)
    p = W.C2Params()
    start = 10_000_000
    kb, ko, vers = W.c2_history(p, seed=1, start_version=start)
    rng = np.random.default_rng(101)
    seq, now = [], start
    for _ in range(72):
        now += p.version_step
        seq.append((W.c2_batch(p, rng, now), now, now - p.window))
    cs = engine.ConflictSet(0)
    cs.load_history(kb, ko, vers, 0)
    cs.set_delta_limit(len(vers) // 16)  # the N/16 bound: a compaction every ~16 batches
    got = {}
    pipeline(engine, cs, seq, lambda i, v: got.__setitem__(i, v))
    st = cs.stats()
    assert st["compactions"] >= 3, st["compactions"]
    assert st["gc_runs"] >= 1, st["gc_runs"]
    check_against_restatement(oracle_mod, kb, ko, vers, seq, got)
    cs.close()


@pytest.mark.parametrize("order", ["resolver", "ahead"])
def test_full_c2_too_old_at_window_edge(engine, oracle_mod, order):
    """TooOld at full size: C2 over the 5M-boundary history with 2 % of the
    snapshots at the MVCC window's edge (now - 5e6 +- 2 batches), the oldest version following
    now - 5e6 every batch (Resolver.actor.cpp:194).  resolver: each batch added after the previous
    batch's detect_async returned (Resolver.actor.cpp:179-194), so its TooOld test sees the oldest
    that detect left (SkipList.cpp:770, 880-882); ahead: all batches added before the first detect
    (bench.py's timed pass), replayed with the oldest each add saw.  Exact either way, with many
    TooOld verdicts; the TooOld transactions' writes never reach the history (:779-790)."""
    p = W.C2Params(too_old_frac=0.02)
    start = 10_000_000
    kb, ko, vers = W.c2_history(p, seed=3, start_version=start)
    rng = np.random.default_rng(103)
    seq, now = [], start
    for _ in range(24):
        now += p.version_step
        seq.append((W.c2_batch(p, rng, now), now, now - p.window))
    cs = engine.ConflictSet(0)
    cs.load_history(kb, ko, vers, 0)
    got, add_oldest = {}, {}
    if order == "resolver":
        pipeline(engine, cs, seq, lambda i, v: got.__setitem__(i, v))
    else:  # bench.py's passes: each group of 8 batches added before the group's first detect
        for g0 in range(0, len(seq), 8):
            objs = []
            for i in range(g0, min(g0 + 8, len(seq))):
                b = engine.ConflictBatch(cs)
                add_oldest[i] = cs.oldest_version
                b.add_packed(seq[i][0])
                objs.append((i, b))
            for i, b in objs:
                b.detect_async(seq[i][1], seq[i][2])
            for i, b in objs:
                got[i] = b.wait()
                b.close()
    sl = oracle_mod.SkipListBaseline()
    sl.load_history(kb, ko, vers)
    too_old = 0
    for i, (pb, now_, no_) in enumerate(seq):
        v, _ = sl.detect(pb, now_, no_, gc="bounded", add_oldest=add_oldest.get(i))
        bad = np.nonzero(got[i] != v)[0]
        assert len(bad) == 0, (i, bad[:10], got[i][bad[:10]], v[bad[:10]])
        too_old += int((v == 1).sum())
    # ~2 % of 120k transactions sit at the edge, about half of them below it
    assert too_old > (300 if order == "resolver" else 25), too_old
    cs.close()


def test_flag_before_epilogue_end_without_submit_thread(engine, oracle_mod, monkeypatch):
    """the completion flag is published by the epilogue's first workgroup while
    the others may still build levels and zero workspace scratch.  Without the helper thread the
    host's dependency checks may skip an event wait once the flag is seen; they must also find the
    epilogue's event complete.  Window 3 with three workspaces: each wait is followed at once by the
    detect that reuses the waited batch's workspace, and every second batch compacts and runs
    removeBefore over a 2M-boundary base (a whole-base epilogue of thousands of workgroups)."""
    monkeypatch.setenv("FDBCS_SUBMIT_THREAD", "0")
    p = W.C2Params(history=2_000_000, txns=2000, too_old_frac=0.01)
    start = 10_000_000
    kb, ko, vers = W.c2_history(p, seed=4, start_version=start)
    rng = np.random.default_rng(104)
    seq, now = [], start
    for _ in range(30):
        now += p.version_step
        seq.append((W.c2_batch(p, rng, now), now, now - p.window))
    cs = engine.ConflictSet(0)
    cs.load_history(kb, ko, vers, 0)
    cs.set_gc_interval(2)
    got = {}
    pipeline(engine, cs, seq, lambda i, v: got.__setitem__(i, v), window=2)
    assert cs.stats()["compactions"] >= 10
    check_against_restatement(oracle_mod, kb, ko, vers, seq, got)
    cs.close()


@pytest.mark.parametrize("mode", ["default", "split"])
def test_async_pipeline_full_c3(engine, oracle_mod, monkeypatch, mode):
    """C3 at full size: Zipf(0.99) hot keys, 5000 txns per batch over the 5M-boundary history,
    heavy intra-batch conflicts resolved in batch order on the device.  split: the base-tier check
    on its own stream (FDBCS_SPLIT_CHECK=1) and compactions every few batches, so a base-tier check
    is issued before the previous batch's compaction (and must wait for it)."""
    if mode == "split":
        monkeypatch.setenv("FDBCS_SPLIT_CHECK", "1")
    p = W.C2Params()
    start = 10_000_000
    kb, ko, vers = W.c2_history(p, seed=2, start_version=start)
    z = W.ZipfGenerator(1_000_000, 0.99)
    rng = np.random.default_rng(102)
    seq, now = [], start
    for _ in range(24):
        now += p.version_step
        seq.append((W.c3_batch(p, rng, now, z), now, now - p.window))
    cs = engine.ConflictSet(0)
    cs.load_history(kb, ko, vers, 0)
    if mode == "split":
        cs.set_delta_limit(60_000)  # a compaction every few batches
    got = {}
    pipeline(engine, cs, seq, lambda i, v: got.__setitem__(i, v))
    st = cs.stats()
    assert st["intra_edges"] > 0
    if mode == "split":
        assert st["compactions"] >= 3, st["compactions"]
    check_against_restatement(oracle_mod, kb, ko, vers, seq, got)
    assert any((got[i] == 0).sum() > 500 for i in got)  # heavy contention really happened
    cs.close()


@pytest.fixture(scope="module")
def c4_history():
    """The 50M-boundary C4 window (tuple keys), generated once for the module's C4 tests."""
    p = W.C4Params()
    start = 10_000_000
    kb, ko, vers = W.c4_history(p, seed=1000, start_version=start)
    return p, start, kb, ko, vers


def test_async_pipeline_full_c4(engine, oracle_mod, c4_history):
    """C4 in production mode: 50M boundaries of tuple keys, 8 batches in
    flight, the default stream layout (the base-tier check on its own stream above 16M
    boundaries, the submit thread's defaults), size-triggered compactions of the 50M base (the
    long-key lane search, the non-temporal copy) with removeBefore on every fourth, the window
    sliding every batch (SkipList.cpp:844-890).  A small delta bound makes the compactions come
    every few batches.  Every verdict matches the restatement with the reference's bounded
    removeBefore (verdict-neutral against the device's full GC)."""
    p, start, kb, ko, vers = c4_history
    rng = np.random.default_rng(104)
    seq, now = [], start
    for _ in range(20):
        now += p.version_step
        seq.append((W.c4_batch(p, rng, now), now, now - p.window))
    cs = engine.ConflictSet(0)
    cs.load_history(kb, ko, vers, 0)
    cs.set_delta_limit(60_000)  # ~20k boundaries per batch: a compaction every three batches
    got = {}
    pipeline(engine, cs, seq, lambda i, v: got.__setitem__(i, v))
    st = cs.stats()
    assert st["compactions"] >= 4, st["compactions"]
    assert st["gc_runs"] >= 1, st["gc_runs"]
    check_against_restatement(oracle_mod, kb, ko, vers, seq, got)
    cs.close()


def test_full_c4_window_gc_and_tail_reclaim(engine, oracle_mod, monkeypatch, c4_history):
    """C4 at full size: 50M boundaries of tuple keys (~1.9 GB of tail bytes), the window sliding
    every batch.  The tail-reclaim threshold is lowered to just above the loaded arena so the
    size-triggered path compacts, runs removeBefore and repacks the tails within a few batches.
    Every verdict matches the restatement, and after each device removeBefore the boundary count
    equals the restatement's after a full removeBefore on the same batch."""
    t0 = time.time()
    p, start, kb, ko, vers = c4_history
    tl = np.diff(ko) - 16
    tail0 = int(((tl[tl > 0] + 7) // 8 * 8).sum())  # the loaded arena: tails padded to 8 bytes
    monkeypatch.setenv("FDBCS_TAIL_RECLAIM", str(tail0 + 3_000_000))
    rng = np.random.default_rng(103)
    seq, now = [], start
    for _ in range(8):
        now += p.version_step
        seq.append((W.c4_batch(p, rng, now), now, now - p.window))
    cs = engine.ConflictSet(0)
    cs.load_history(kb, ko, vers, 0)
    n0 = cs.history_size()
    assert n0 == len(vers)
    sl = oracle_mod.SkipListBaseline()
    sl.load_history(kb, ko, vers)
    gcs = 0
    for i, (pb, now_i, no) in enumerate(seq):  # one batch at a time: the GC schedule is observed
        b = engine.ConflictBatch(cs)
        b.add_packed(pb)
        v = b.detect_conflicts(now_i, no)
        b.close()
        ran = cs.stats()["gc_runs"] > gcs
        gcs = cs.stats()["gc_runs"]
        vo, _ = sl.detect(pb, now_i, no, gc=ran)  # full removeBefore exactly where the device ran one
        bad = np.nonzero(v != vo)[0]
        assert len(bad) == 0, (i, bad[:10])
        if ran:
            assert cs.history_size() == sl.history_size(), (i, cs.history_size(), sl.history_size())
    assert gcs >= 1, "tail reclaim never forced a removeBefore"
    assert time.time() - t0 < 600


def brute_force(seq, history=(), oldest0=0):
    """Key-space model over committed write ranges (versions only grow, so the history's max over a
    read range exceeds the snapshot iff some committed write intersecting it is newer).  Returns per
    batch (verdicts, reports): reports hold every history-conflicting read, or the first read that
    meets an earlier committed write of the same batch (SkipList.cpp:641-645, 821-828)."""
    written = list(history)  # (begin, end, version)
    oldest = oldest0
    out = []
    for pb, now, no in seq:
        txns = pb.to_transactions()
        verdict, conf, batch_w = [], {}, []
        for t, tr in enumerate(txns):
            if tr.read_snapshot < oldest and tr.read_conflict_ranges:
                verdict.append(1)
                continue
            hist = [i for i, r in enumerate(tr.read_conflict_ranges)
                    if any(b < r.end and r.begin < e and v > tr.read_snapshot for b, e, v in written)]
            if hist:
                verdict.append(0)
                if tr.report_conflicting_keys:
                    conf[t] = hist
                continue
            intra = [i for i, r in enumerate(tr.read_conflict_ranges)
                     if any(w.begin < r.end and r.begin < w.end for w in batch_w)]
            if intra:
                verdict.append(0)
                if tr.report_conflicting_keys:
                    conf[t] = intra[:1]
            else:
                verdict.append(2)
                batch_w.extend(w for w in tr.write_conflict_ranges if w.begin < w.end)
        written.extend((w.begin, w.end, now) for w in batch_w)
        oldest = max(oldest, no)
        out.append((np.array(verdict, np.uint8), conf))
    return out


def nonempty_batch(rng, n, now, alphabet=3, max_len=3):
    def key():
        return bytes(int(x) for x in rng.integers(0, alphabet, size=int(rng.integers(0, max_len + 1))))

    def rr():
        while True:
            a, b = key(), key()
            if a != b:
                return KeyRange(min(a, b), max(a, b))

    txns = [CommitTransaction([rr() for _ in range(int(rng.integers(0, 4)))],
                              [rr() for _ in range(int(rng.integers(0, 3)))],
                              int(now - rng.integers(0, 12)), bool(rng.random() < 0.6)) for _ in range(n)]
    return PackedBatch.from_transactions(txns)


@pytest.mark.parametrize("gc_interval,delta_limit", [(1, 0), (0, 12)])
def test_engine_matches_keyspace_bruteforce(engine, gc_interval, delta_limit):
    """An independent model (no skip list, no step function: committed write ranges with versions)
    pins the engine's verdicts and conflicting-key reports.  Non-empty ranges only (NativeAPI never
    sends empty ones, NativeAPI.actor.cpp:3192-3194); touching, nesting and shared prefixes abound."""
    rng = np.random.default_rng(404 + gc_interval)
    for trial in range(6):
        seq, now = [], 20
        for _ in range(10):
            seq.append((nonempty_batch(rng, int(rng.integers(5, 80)), now), now, now - int(rng.integers(3, 9))))
            now += int(rng.integers(1, 4))
        want = brute_force(seq)
        cs = engine.ConflictSet(0)
        cs.set_gc_interval(gc_interval)
        cs.set_delta_limit(delta_limit)
        for i, (pb, now_i, no) in enumerate(seq):
            m = {}
            b = engine.ConflictBatch(cs, m)
            b.add_packed(pb)
            v = b.detect_conflicts(now_i, no)
            b.close()
            wv, wc = want[i]
            assert (v == wv).all(), (trial, i, np.nonzero(v != wv)[0][:8])
            got = {t: sorted(x) for t, x in m.items() if x}
            assert got == wc, (trial, i)
            # entries exist exactly for reporting, admitted transactions with reads (SkipList.cpp:777-784)
            roff = pb.read_offsets
            assert set(m) == {t for t in range(pb.n_txn) if pb.report[t] and roff[t + 1] > roff[t] and v[t] != 1}
            # ConflictRange soundness / precision (ConflictRange.actor.cpp:226-316): a committed txn
            # read nothing newer than its snapshot; every aborted non-TooOld txn has a reason
            for t, tr in enumerate(pb.to_transactions()):
                if v[t] == 0 and tr.report_conflicting_keys:
                    assert got.get(t), (trial, i, t)
        cs.close()


def test_worst_case_dependency_chain(engine, oracle_mod):
    """Batch-order resolution's adversarial case: transaction t reads the key transaction t-1
    writes, 5000 deep, so each verdict depends on the previous one (commit, abort, commit, ...)."""
    T = 5000
    keys = [b"chain%06d" % i for i in range(T + 1)]
    txns = [CommitTransaction([KeyRange(keys[t], keys[t] + b"\x00")], [KeyRange(keys[t + 1], keys[t + 1] + b"\x00")],
                              100, False) for t in range(T)]
    pb = PackedBatch.from_transactions(txns)
    cs = engine.ConflictSet(0)
    cs.set_timing(2)
    b = engine.ConflictBatch(cs)
    b.add_packed(pb)
    v = b.detect_conflicts(100, 0)
    b.close()
    expect = np.array([2 if t % 2 == 0 else 0 for t in range(T)], np.uint8)
    assert (v == expect).all()
    vo, _ = oracle_mod.OracleConflictSet().detect(pb, 100, 0)
    assert (vo == v).all()
    st = cs.stats()
    print(f"chain of {T}: {st['intra_rounds']} resolution rounds, intra phase {st['ms_intra']:.3f} ms")
    cs.close()


def test_reference_max_batch_32768(engine, oracle_mod):
    """The reference's largest commit batch (COMMIT_TRANSACTION_BATCH_COUNT_MAX = 32768,
    fdbserver/Knobs.cpp:370) at the C2 shape over the 5M-boundary history: T > 8192 takes the
    resolution rounds' global-memory path and W = 65536 > kMaxGroupWrites turns write groups off.
    Three batches, pipelined, against the restatement."""
    p = W.C2Params(txns=32768)
    kb, ko, vers = W.c2_history(p, seed=9, start_version=10_000_000)
    rng = np.random.default_rng(32768)
    seq, now = [], 10_000_000
    for _ in range(3):
        now += p.version_step
        seq.append((W.c2_batch(p, rng, now), now, now - p.window))
    cs = engine.ConflictSet(0)
    cs.load_history(kb, ko, vers, 0)
    got = {}
    pipeline(engine, cs, seq, lambda i, v: got.__setitem__(i, v), window=3)
    assert seq[0][0].n_txn == 32768 and seq[0][0].n_writes == 65536
    check_against_restatement(oracle_mod, kb, ko, vers, seq, got)
    committed = sum(int((got[i] == 2).sum()) for i in got)
    assert 0 < committed < 3 * 32768
    cs.close()


def rck_key(n, node_count=10000, client=0, prefix=b"RCK", key_bytes=64):
    """keyForIndex of the ReportConflictingKeys workload (ReportConflictingKeys.actor.cpp:87-95):
    prefix + "Cid_%04d" + the bits of the double n / nodeCount as zero-padded hex."""
    import struct

    bits = struct.unpack("<Q", struct.pack("<d", n / node_count))[0]
    pad = key_bytes - 8 - len(prefix)
    return prefix + b"Cid_%04d" % client + b"%0*x" % (pad, bits)


def rck_batch(rng, n_txn, now, node_count=10000, mean_ranges=10):
    """A batch of the workload's transactions (tests/fast/ReportConflictingKeys.toml: keyPrefix RCK,
    keyBytes 64, nodeCount 10000, 10 read and 10 write ranges per transaction on average; each range
    [keyForIndex(s), keyForIndex(e)) with s uniform in [0, nodeCount), e in (s, nodeCount], the
    count geometric with at least one, ReportConflictingKeys.actor.cpp:98-125)."""
    keys = {}

    def key(i):
        if i not in keys:
            keys[i] = rck_key(i, node_count)
        return keys[i]

    def ranges():
        out = []
        while True:
            s = int(rng.integers(0, node_count))
            e = int(rng.integers(s + 1, node_count + 1))
            out.append(KeyRange(key(s), key(e)))
            if rng.random() >= (mean_ranges - 1.0) / mean_ranges:
                return out

    txns = [CommitTransaction(ranges(), ranges(), int(now - rng.integers(0, 6)), True) for _ in range(n_txn)]
    return PackedBatch.from_transactions(txns)


def test_report_conflicting_keys_workload_shape(engine):
    """The reference's own ReportConflictingKeys spec shape (64-byte keys sharing their first ~47
    bytes, wide ranges, ~10 reads and ~10 writes per transaction) against the key-space model: the
    verdicts, and the reported conflicting reads exactly (ReportConflictingKeys.actor.cpp:201-278:
    every reported range is one of the transaction's reads and meets a write it conflicts with; a
    transaction with no conflict has no such intersection)."""
    rng = np.random.default_rng(201)
    seq, now = [], 50
    for _ in range(6):
        seq.append((rck_batch(rng, int(rng.integers(60, 160)), now), now, now - 8))
        now += 3
    want = brute_force(seq)
    cs = engine.ConflictSet(0)
    cs.set_gc_interval(2)
    for i, (pb, now_i, no) in enumerate(seq):
        m = {}
        b = engine.ConflictBatch(cs, m)
        b.add_packed(pb)
        v = b.detect_conflicts(now_i, no)
        b.close()
        wv, wc = want[i]
        assert (v == wv).all(), (i, np.nonzero(v != wv)[0][:8])
        got = {t: sorted(x) for t, x in m.items() if x}
        assert got == wc, i
        for t in range(pb.n_txn):  # a conflict always carries a report (the workload's check)
            if v[t] == 0:
                assert got.get(t), (i, t)
    cs.close()
