"""GPU parity: the HIP engine (through the C-ABI) against the CPU oracle, bit-exact verdicts and
conflicting-key reports, on the reference's known answers, frozen fixtures, live random batches,
the BASELINE configurations (reduced where the oracle must keep up) and size-independent
properties at full size."""
import os

import numpy as np
import pytest

from foundationdb_amd import workloads as W
from foundationdb_amd.packing import CommitTransaction, KeyRange, PackedBatch
from tests.helpers import EngineDriver, load_json, nonempty, random_fixture_sequences, scenario_batches

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def oracle_mod():
    from oracle import oracle

    oracle.build()
    return oracle


def run_pair(engine, oracle_mod, seq, gc_interval=1, clear=None, check_conf=True, ref="oracle", delta_limit=0):
    e = EngineDriver(engine, gc_interval=gc_interval, delta_limit=delta_limit)
    o = oracle_mod.OracleConflictSet() if ref == "oracle" else oracle_mod.SkipListBaseline()
    if clear is not None:
        e.clear(clear)
        o.clear(clear)
    for i, (pb, now, no) in enumerate(seq):
        ve, ce = e.detect(pb, now, no)
        vo, co = o.detect(pb, now, no)
        assert (ve == vo).all(), (i, np.nonzero(ve != vo)[0][:10], ve[ve != vo][:10], vo[ve != vo][:10])
        if check_conf:  # the whole conflictingKeyRangeMap: entries (even empty ones) and contents
            assert ce == co, i
    return e, o


def test_kat_scenarios(engine):
    for scn in load_json("kat_scenarios.json"):
        e = EngineDriver(engine)
        for i, (pb, now, no, expect, conf) in enumerate(scenario_batches(scn)):
            if scn.get("clear_before") == i:
                e.clear(scn["clear_version"])
            v, c = e.detect(pb, now, no)
            assert v.tolist() == expect, (scn["name"], i, v.tolist(), expect)
            if conf:
                assert nonempty(c) == conf, (scn["name"], c, conf)


def test_frozen_random_fixtures(engine):
    for s, seq in random_fixture_sequences():
        e = EngineDriver(engine)
        for pb, now, no, verdict, conf in seq:
            v, c = e.detect(pb, now, no)
            assert (v == verdict).all(), s
            assert nonempty(c) == conf, s


@pytest.mark.parametrize("alphabet,max_len", [(2, 2), (3, 3), (4, 5), (256, 2), (3, 24), (2, 40)])
def test_random_vs_oracle(engine, oracle_mod, alphabet, max_len):
    rng = np.random.default_rng(alphabet * 100 + max_len)
    for trial in range(12):
        seq = []
        now = 10
        for _ in range(6):
            pb = W.random_small_batch(rng, int(rng.integers(1, 120)), alphabet=alphabet, max_len=max_len, now=now,
                                      staleness=15, max_reads=4, max_writes=3)
            seq.append((pb, now, now - int(rng.integers(0, 12))))
            now += int(rng.integers(1, 6))
        # trials alternate: compaction every 1-3 batches, size-triggered compaction with a tiny delta
        # bound, and a delta tier that is never compacted
        gc, dl = [(1, 0), (2, 0), (3, 0), (0, 7), (0, 40), (0, 0)][trial % 6]
        run_pair(engine, oracle_mod, seq, gc_interval=gc, delta_limit=dl, clear=(5 if trial % 5 == 0 else None))


def _prefixed(pb, prefix: bytes):
    """The batch with `prefix` before every key: the same verdicts, every comparison in the tails."""
    n = len(pb.key_offsets) - 1
    lens = np.diff(pb.key_offsets)
    parts = []
    for k in range(n):
        parts.append(prefix)
        parts.append(pb.key_bytes[pb.key_offsets[k]:pb.key_offsets[k + 1]].tobytes())
    offs = np.concatenate([[0], np.cumsum(lens + len(prefix))]).astype(np.int64)
    return PackedBatch(pb.read_snapshot, pb.report, pb.read_offsets, pb.write_offsets,
                         np.frombuffer(b"".join(parts), np.uint8).copy(), offs)


@pytest.mark.parametrize("gc_interval,delta_limit", [(0, 0), (0, 40), (3, 0)])
def test_long_shared_prefix_tails(engine, oracle_mod, gc_interval, delta_limit):
    """Keys behind a 60-byte shared prefix: every order decision is made in the tails, and a batch's
    tail region holds several words per endpoint.  The next batch's check reads the previous
    batch's union segments with their tails from the workspace copy (PrevSegs), so a short copy
    shows up as wrong verdicts."""
    rng = np.random.default_rng(77 + gc_interval + delta_limit)
    prefix = bytes(rng.integers(0, 256, 60, dtype=np.uint8))
    seq = []
    now = 10
    for _ in range(24):
        pb = W.random_small_batch(rng, int(rng.integers(20, 200)), alphabet=3, max_len=5, now=now, staleness=12,
                                  max_reads=4, max_writes=3)
        seq.append((_prefixed(pb, prefix), now, now - int(rng.integers(0, 10))))
        now += int(rng.integers(1, 4))
    run_pair(engine, oracle_mod, seq, gc_interval=gc_interval, delta_limit=delta_limit)


@pytest.mark.parametrize("gc_interval,delta_limit", [(1, 0), (0, 0), (0, 25), (4, 0)])
def test_delta_tier_configurations(engine, oracle_mod, gc_interval, delta_limit):
    """The two-tier history (delta merges, compaction, GC at compaction) is verdict- and
    report-exact whatever the compaction cadence: long sequences over tiny alphabets make
    delta boundaries overwrite, nest in and touch base boundaries."""
    rng = np.random.default_rng(1000 + 10 * gc_interval + delta_limit)
    seq = []
    now = 10
    for _ in range(30):
        pb = W.random_small_batch(rng, int(rng.integers(1, 60)), alphabet=3, max_len=3, now=now, staleness=12,
                                  max_reads=3, max_writes=3, report_frac=0.5)
        seq.append((pb, now, now - int(rng.integers(0, 10))))
        now += int(rng.integers(1, 4))
    run_pair(engine, oracle_mod, seq, gc_interval=gc_interval, delta_limit=delta_limit)


def test_delta_tier_history_size_after_compaction(engine, oracle_mod):
    """After a compaction with GC the device holds exactly the reference's boundary count (skip-list
    restatement running removeBefore on the same batches), although the batches in between lived
    in the delta tier."""
    seq = list(W.c1_batches(12, seed=11))
    e = EngineDriver(engine, gc_interval=4)
    o = oracle_mod.SkipListBaseline()
    for i, (pb, now, no) in enumerate(seq):
        ve, _ = e.detect(pb, now, no)
        vo, _ = o.detect(pb, now, no, gc=(i + 1) % 4 == 0)
        assert (ve == vo).all(), i
        if (i + 1) % 4 == 0:
            assert e.cs.history_size() == o.history_size(), i


def test_shared_long_prefixes(engine, oracle_mod):
    """Tuple-like keys sharing > 16-byte prefixes exercise the tail comparison everywhere."""
    rng = np.random.default_rng(99)
    prefix = b"\x01subspace\x00\x02users\x00"
    seq = []
    now = 10
    for _ in range(8):
        txns = []
        for _ in range(80):
            def key():
                return prefix + bytes(rng.integers(0, 3, size=int(rng.integers(0, 4))).astype(np.uint8))

            def rr():
                a, b = key(), key()
                return KeyRange(min(a, b), max(a, b))

            txns.append(CommitTransaction([rr() for _ in range(int(rng.integers(0, 3)))],
                                          [rr() for _ in range(int(rng.integers(0, 3)))],
                                          now - int(rng.integers(0, 10)), bool(rng.random() < 0.5)))
        seq.append((PackedBatch.from_transactions(txns), now, now - 8))
        now += 3
    run_pair(engine, oracle_mod, seq)
    run_pair(engine, oracle_mod, seq, gc_interval=0, delta_limit=30)


@pytest.mark.parametrize("split", ["1", "2"])
@pytest.mark.parametrize("tail_max", [40, 8])
def test_long_shared_prefix_runs(engine, oracle_mod, monkeypatch, split, tail_max):
    """Thousands of history boundaries behind one 16-byte prefix (a few huge tuple subspaces): the
    search must order them by their tail bytes over a run far longer than one 64-boundary block
    (the cooperative probe rounds start at a stride of 512 or more; with keys of at most 24 bytes
    the per-lane lookups' binary search over the run)."""
    monkeypatch.setenv("FDBCS_SPLIT_CHECK", split)
    rng = np.random.default_rng(123 + tail_max)
    prefixes = [b"\x15\x2a\x02huge-subspa%d\x00" % i for i in range(3)]
    assert all(len(x) == 16 for x in prefixes)

    def key():
        pre = prefixes[int(rng.integers(0, len(prefixes)))]
        return pre + bytes(rng.integers(0, 256, size=int(rng.integers(0, tail_max + 1))).astype(np.uint8))

    hist = sorted({key() for _ in range(20000)})
    kb = np.frombuffer(b"".join(hist), np.uint8)
    ko = np.zeros(len(hist) + 1, np.int64)
    np.cumsum([len(k) for k in hist], out=ko[1:])
    vers = rng.integers(0, 1000, size=len(hist)).astype(np.int64)
    e = EngineDriver(engine, gc_interval=0, delta_limit=4000)
    o = oracle_mod.SkipListBaseline()
    e.load_history(kb, ko, vers)
    o.load_history(kb, ko, vers)
    now = 1000
    for i in range(6):
        now += 10
        txns = []
        for _ in range(400):
            def rr():
                a, b = key(), key()
                return KeyRange(min(a, b), max(a, b))

            txns.append(CommitTransaction([rr() for _ in range(int(rng.integers(1, 4)))],
                                          [rr() for _ in range(int(rng.integers(0, 3)))],
                                          now - int(rng.integers(0, 600)), False))
        pb = PackedBatch.from_transactions(txns)
        ve, _ = e.detect(pb, now, 0)
        vo, _ = o.detect(pb, now, 0)
        assert (ve == vo).all(), (i, np.nonzero(ve != vo)[0][:10])


@pytest.mark.parametrize("directory,split,gc", [("1", "2", 2), ("1", "1", 2), ("0", "2", 2), ("1", "2", 0)])
def test_radix_directory_slots(engine, oracle_mod, monkeypatch, directory, split, gc):
    """The base tier's radix directory (first two key bytes -> level-0 samples): sparse slots
    counted directly, a crowded slot (one 2-byte prefix holding thousands of boundaries) taking
    the tree, keys at the slot edges (empty key, 0x0000.., 0xffff.., bare 2-byte keys), and
    compactions rebuilding the directory between batches; gc=0 keeps every batch in the delta
    tier, whose directory k_epilogue refills per batch under a new epoch (runs over kDirRun slots
    stay stale and take the tree)."""
    monkeypatch.setenv("FDBCS_DIRECTORY", directory)
    monkeypatch.setenv("FDBCS_SPLIT_CHECK", split)
    rng = np.random.default_rng(4242)
    edges = [b"", b"\x00", b"\x00\x00", b"\x00\x00\x00", b"\x12\x33\xff", b"\x12\x34", b"\x12\x34\x00",
             b"\x12\x35", b"\xff\xfe\xff", b"\xff\xff", b"\xff\xff\x00", b"\xff\xff\xff\xff"]

    def key():
        u = rng.random()
        if u < 0.55:
            return bytes(rng.integers(0, 256, size=int(rng.integers(1, 20))).astype(np.uint8))
        if u < 0.9:
            return b"AB" + bytes(rng.integers(0, 256, size=int(rng.integers(0, 12))).astype(np.uint8))
        e = edges[int(rng.integers(0, len(edges)))]
        return e + bytes(rng.integers(0, 4, size=int(rng.integers(0, 3))).astype(np.uint8))

    hist = sorted({key() for _ in range(60000)} | set(edges[1:]))
    kb = np.frombuffer(b"".join(hist), np.uint8)
    ko = np.zeros(len(hist) + 1, np.int64)
    np.cumsum([len(k) for k in hist], out=ko[1:])
    vers = rng.integers(0, 1000, size=len(hist)).astype(np.int64)
    e = EngineDriver(engine, gc_interval=gc, delta_limit=100000 if gc == 0 else 0)
    o = oracle_mod.SkipListBaseline()
    e.load_history(kb, ko, vers)
    o.load_history(kb, ko, vers)
    now = 1000
    for i in range(8):
        now += 10
        txns = []
        for _ in range(500):
            def rr():
                a, b = key(), key()
                return KeyRange(min(a, b), max(a, b))

            txns.append(CommitTransaction([rr() for _ in range(int(rng.integers(1, 4)))],
                                          [rr() for _ in range(int(rng.integers(0, 3)))],
                                          now - int(rng.integers(0, 600)), False))
        pb = PackedBatch.from_transactions(txns)
        ve, _ = e.detect(pb, now, 0)
        vo, _ = o.detect(pb, now, 0, gc=(i + 1) % 2 == 0)
        assert (ve == vo).all(), (i, np.nonzero(ve != vo)[0][:10])


@pytest.mark.parametrize("split", ["1", "2"])
@pytest.mark.parametrize("plen", [30, 60, 104, 150])
def test_very_long_shared_prefixes(engine, oracle_mod, monkeypatch, plen, split):
    """Keys sharing prefixes of 30-150 bytes, so that tail comparisons end inside the long-key
    probe's first word round (48 bytes), its second (96), and past the query words it holds in
    registers (the rest compared from memory); history and batch keys of every length around them.
    split "1": the split read check (long-key probes in both check launches); "2": the default."""
    monkeypatch.setenv("FDBCS_SPLIT_CHECK", split)
    rng = np.random.default_rng(plen)
    prefixes = [bytes([0x15, 0x2a + i]) + b"x" * (plen - 2) for i in range(2)]

    def key():
        pre = prefixes[int(rng.integers(0, len(prefixes)))]
        cut = int(rng.integers(plen - 20, plen + 1))  # some keys end inside the shared prefix
        return pre[:cut] + bytes(rng.integers(0, 3, size=int(rng.integers(0, 6))).astype(np.uint8))

    hist = sorted({key() for _ in range(6000)})
    kb = np.frombuffer(b"".join(hist), np.uint8)
    ko = np.zeros(len(hist) + 1, np.int64)
    np.cumsum([len(k) for k in hist], out=ko[1:])
    vers = rng.integers(0, 1000, size=len(hist)).astype(np.int64)
    e = EngineDriver(engine, gc_interval=0, delta_limit=1500)
    o = oracle_mod.SkipListBaseline()
    e.load_history(kb, ko, vers)
    o.load_history(kb, ko, vers)
    now = 1000
    for i in range(6):
        now += 10
        txns = []
        for _ in range(300):
            def rr():
                a, b = key(), key()
                return KeyRange(min(a, b), max(a, b))

            txns.append(CommitTransaction([rr() for _ in range(int(rng.integers(1, 4)))],
                                          [rr() for _ in range(int(rng.integers(0, 3)))],
                                          now - int(rng.integers(0, 600)), False))
        pb = PackedBatch.from_transactions(txns)
        ve, _ = e.detect(pb, now, 0)
        vo, _ = o.detect(pb, now, 0)
        assert (ve == vo).all(), (i, np.nonzero(ve != vo)[0][:10])


@pytest.mark.parametrize("alphabet", ["bytes", "digits", "sparse"])
def test_directory_past_shared_prefix(engine, oracle_mod, monkeypatch, alphabet):
    """The radix directories' rank code after the bytes every loaded key shares (MaxLevels::dir_p;
    C4's 9-byte prefix): 120k boundaries under one 10-byte prefix, queries inside it, below and
    above it at every depth, keys shorter than it and the empty key; writes outside the prefix,
    which both tiers' directories file under their end slots (dir_slot), before and after the
    compactions that bring them into the base.  alphabet "digits": the bytes after the prefix are
    decimal digits (C4's user ids), ten ranks per position; "sparse": the history holds only even
    byte values in [0x20, 0x7e] while queries and writes take any value in [0x10, 0x90], so codes
    end at unseen values (the next seen value's rank) and values above every seen one carry into
    the position before."""
    rng = np.random.default_rng(77)
    P = bytes([0x41, 0x42, 0x43, 0x44, 0x00, 0xff, 0x45, 0x46, 0x47, 0x48])
    lo_b, hi_b = {"bytes": (0, 256), "digits": (0x30, 0x3a), "sparse": (0x10, 0x91)}[alphabet]

    long_keys = [False]  # batches alternate: keys up to 21 bytes (short-key lookups), up to 30

    def suffix(n, hist=False):
        if hist and alphabet == "sparse":
            return bytes((2 * rng.integers(0x10, 0x40, size=n)).astype(np.uint8))
        return bytes(rng.integers(lo_b, hi_b, size=n).astype(np.uint8))

    def inside():
        top = 21 if long_keys[0] else 12
        return P + suffix(int(rng.integers(0, top)))

    def any_key(outside_share):
        r = rng.random()
        if r >= outside_share:
            return inside()
        d = int(rng.integers(0, len(P)))  # diverge at byte d, below or above, or stop short of P
        kind = int(rng.integers(0, 3))
        if kind == 0:
            return P[:d]
        x = P[d] - 1 if kind == 1 else P[d] + 1
        if not 0 <= x <= 255:
            return P[:d]
        return P[:d] + bytes([x]) + bytes(rng.integers(0, 256, size=int(rng.integers(0, 8))).astype(np.uint8))

    hist = sorted({P + suffix(6, hist=True) for _ in range(120000)})
    kb = np.frombuffer(b"".join(hist), np.uint8)
    ko = np.zeros(len(hist) + 1, np.int64)
    np.cumsum([len(k) for k in hist], out=ko[1:])
    vers = rng.integers(0, 1000, size=len(hist)).astype(np.int64)
    e = EngineDriver(engine, gc_interval=2, delta_limit=0)  # a compaction every second batch
    o = oracle_mod.SkipListBaseline()
    e.load_history(kb, ko, vers)
    o.load_history(kb, ko, vers)
    now = 1000
    for i in range(8):
        now += 10
        long_keys[0] = i % 2 == 1
        txns = []
        for _ in range(400):
            def rr(share):
                a, b = any_key(share), any_key(share)
                return KeyRange(min(a, b), max(a, b))

            txns.append(CommitTransaction([rr(0.3) for _ in range(int(rng.integers(1, 4)))],
                                          [rr(0.05 if i < 3 else 0.3) for _ in range(int(rng.integers(0, 3)))],
                                          now - int(rng.integers(0, 600)), False))
        pb = PackedBatch.from_transactions(txns)
        ve, _ = e.detect(pb, now, 0)
        vo, _ = o.detect(pb, now, 0)
        assert (ve == vo).all(), (i, np.nonzero(ve != vo)[0][:10])


def test_c1_skiplisttest(engine, oracle_mod):
    seq = list(W.c1_batches(25, seed=7))
    e, o = run_pair(engine, oracle_mod, seq, check_conf=False, ref="skiplist")
    # GC is eager in both (interval 1, full): same step function size
    assert e.cs.history_size() == o.history_size()


def test_c2_reduced(engine, oracle_mod):
    p = W.C2Params(txns=2000, history=200_000)
    kb, ko, vers = W.c2_history(p, seed=1, start_version=10_000_000)
    e = EngineDriver(engine, gc_interval=0, delta_limit=30_000)
    o = oracle_mod.SkipListBaseline()
    e.load_history(kb, ko, vers)
    o.load_history(kb, ko, vers)
    rng = np.random.default_rng(2)
    now = 10_000_000
    for i in range(10):
        now += p.version_step
        pb = W.c2_batch(p, rng, now)
        ve, _ = e.detect(pb, now, now - p.window)
        vo, _ = o.detect(pb, now, now - p.window)
        assert (ve == vo).all(), i


@pytest.mark.parametrize("prepass", ["1", "0"])
def test_c3_zipf_heavy_contention(engine, oracle_mod, monkeypatch, prepass):
    """Zipf hot keys: hundreds of candidate writers per reader, most of them history-aborted.
    Both resolution paths: with the multi-workgroup pre-pass (packed live-writer lists) and
    without it (rounds walk the per-read edge lists)."""
    monkeypatch.setenv("FDBCS_RESOLVE_PREPASS", prepass)
    p = W.C2Params(txns=3000)
    z = W.ZipfGenerator(1_000_000, 0.99)
    rng = np.random.default_rng(3)
    seq = []
    now = 1000
    for _ in range(6):
        now += 1000
        seq.append((W.c3_batch(p, rng, now, z), now, now - 100_000))
    e, o = run_pair(engine, oracle_mod, seq, check_conf=False, ref="skiplist")


@pytest.mark.parametrize("gc_interval,delta_limit,split", [(1, 0, "2"), (0, 3000, "2"), (1, 0, "1"), (0, 3000, "1")])
def test_c4_tuple_keys_window_gc(engine, oracle_mod, monkeypatch, gc_interval, delta_limit, split):
    """BASELINE config C4, reduced: tuple-encoded keys up to ~100 B whose 16-byte prefixes are
    shared by every key of a user (comparisons go to the tail bytes), wide Tuple.range() reads, and
    the window sliding with newOldest = now - window every batch (GC), against the skip-list
    restatement; after a compaction with GC both hold the same boundary count.  split "1": the
    split check (the base tier's long-key lookups on their own launch)."""
    monkeypatch.setenv("FDBCS_SPLIT_CHECK", split)
    p = W.C4Params(txns=1500, users=3000, items=400, history=80_000, window=12_000, staleness=4_000)
    kb, ko, vers = W.c4_history(p, seed=4, start_version=100_000)
    e = EngineDriver(engine, gc_interval=gc_interval, delta_limit=delta_limit)
    o = oracle_mod.SkipListBaseline()
    e.load_history(kb, ko, vers)
    o.load_history(kb, ko, vers)
    rng = np.random.default_rng(5)
    now = 100_000
    seen = set()
    for i in range(10):
        now += p.version_step
        pb = W.c4_batch(p, rng, now)
        ve, _ = e.detect(pb, now, now - p.window)
        vo, _ = o.detect(pb, now, now - p.window)
        assert (ve == vo).all(), (i, np.nonzero(ve != vo)[0][:10])
        seen |= set(np.unique(ve).tolist())
    assert {0, 2} <= seen  # both conflicts and commits
    if gc_interval == 1:
        assert e.cs.history_size() == o.history_size()


def test_compaction_search_modes(engine, oracle_mod, monkeypatch):
    """Both k_compact_search modes (one lane per delta boundary: lane_lower_bound after short-key
    batches, lane_lower_bound_long after long-key ones) place the delta boundaries alike:
    compactions over tails behind a 60-byte shared prefix, over a tiny alphabet, and over C4 tuple
    keys stay verdict-exact.  (The non-temporal copy of bases over 16M boundaries is covered by
    test_async_pipeline_full_c4.)"""
    test_long_shared_prefix_tails(engine, oracle_mod, 0, 40)
    test_delta_tier_configurations(engine, oracle_mod, 0, 25)
    test_c4_tuple_keys_window_gc(engine, oracle_mod, monkeypatch, 0, 3000, "2")


def test_async_pipelined_batches_match_sync(engine):
    rng = np.random.default_rng(4)
    batches = []
    now = 10
    for _ in range(8):
        batches.append((W.random_small_batch(rng, 200, alphabet=4, max_len=4, now=now, staleness=10), now, now - 5))
        now += 2
    sync = EngineDriver(engine)
    want = [sync.detect(pb, n, no)[0] for pb, n, no in batches]
    cs = engine.ConflictSet(0)
    objs = []
    for pb, n, no in batches:
        b = engine.ConflictBatch(cs)
        b.add_packed(pb)
        b.upload()
        b.detect_async(n, no)
        objs.append(b)
    for b, w in zip(objs, want):
        assert (b.wait() == w).all()


def test_gc_interval_is_verdict_neutral(engine):
    rng = np.random.default_rng(6)
    seq = []
    now = 10
    for _ in range(12):
        seq.append((W.random_small_batch(rng, 150, alphabet=3, max_len=4, now=now, staleness=9), now, now - 4))
        now += 3
    a, b = EngineDriver(engine, gc_interval=1), EngineDriver(engine, gc_interval=1000)
    for pb, n, no in seq:
        assert (a.detect(pb, n, no)[0] == b.detect(pb, n, no)[0]).all()
    assert a.cs.history_size() <= b.cs.history_size()


def test_edge_cases(engine):
    e = EngineDriver(engine)
    empty = PackedBatch.from_transactions([])
    v, _ = e.detect(empty, 5, 0)
    assert v.size == 0
    # transactions with no ranges commit; version going backwards is refused
    pb = PackedBatch.from_transactions([CommitTransaction(), CommitTransaction(write_conflict_ranges=[KeyRange(b"a", b"b")])])
    v, _ = e.detect(pb, 10, 0)
    assert v.tolist() == [2, 2]
    with pytest.raises(engine.FdbcsError) as ex:
        e.detect(pb, 9, 0)
    assert ex.value.status == engine.FDBCS_E_VERSION


def _packed(txns, inverted=None):
    """A PackedBatch of (snapshot, reads, writes) with [(begin, end)] byte ranges, built directly so
    that `inverted` = (txn, 'r'|'w', i) can swap one range's ends (KeyRange itself refuses that)."""
    keys, roff, woff, snap = [], [0], [0], []
    for t, (sn, reads, writes) in enumerate(txns):
        snap.append(sn)
        roff.append(roff[-1] + len(reads))
        woff.append(woff[-1] + len(writes))
    rk, wk = [], []
    for t, (_, reads, writes) in enumerate(txns):
        for i, (a, b) in enumerate(reads):
            rk += [b, a] if inverted == (t, "r", i) else [a, b]
        for i, (a, b) in enumerate(writes):
            wk += [b, a] if inverted == (t, "w", i) else [a, b]
    keys = rk + wk
    ko = np.zeros(len(keys) + 1, np.int64)
    ko[1:] = np.cumsum([len(k) for k in keys])
    kb = np.frombuffer(b"".join(keys), np.uint8).copy() if keys else np.zeros(0, np.uint8)
    return PackedBatch(np.array(snap, np.int64), np.zeros(len(txns), np.uint8), np.array(roff, np.int32),
                       np.array(woff, np.int32), kb, ko)


@pytest.mark.parametrize("n_txn", [40, 3000])
def test_add_packed_rejects_inverted_ranges(engine, oracle_mod, n_txn):
    """addTransaction refuses a range with begin > end (KeyRangeRef, FDBTypes.h:288-291) wherever it
    sits -- a read, a write, a TooOld transaction's range, keys tied on the 16-byte prefix and
    ordered by their tails -- all or nothing: the batch stays empty and takes a valid batch
    afterwards.  3000 transactions: the validation runs fused with the normalization over the
    add threads' chunks (FDBCS_ADD_THREADS)."""
    rng = np.random.default_rng(n_txn)
    long = b"p" * 16

    def key():
        return (long if rng.random() < 0.3 else b"") + bytes(rng.integers(0, 4, size=int(rng.integers(1, 6))).tolist())

    def rng_range():
        a, b = sorted([key(), key()])
        return a, b

    txns = [(int(rng.integers(0, 20)), [rng_range() for _ in range(2)], [rng_range() for _ in range(2)])
            for _ in range(n_txn)]
    # a pair tied on the 16-byte prefix, ordered by the tails only
    txns[n_txn // 2] = (15, [(long + b"\x01", long + b"\x02")], [(long + b"\x00\x05", long + b"\x00\x06")])
    cs = engine.ConflictSet(0)
    ora = oracle_mod.OracleConflictSet()
    b0 = engine.ConflictBatch(cs)  # oldest -> 10: snapshots below it are TooOld
    b0.add_packed(_packed([]))
    b0.detect_conflicts(20, 10)
    b0.close()
    ora.detect(_packed([]), 20, 10)
    spots = [(1, "r", 0), (n_txn - 1, "w", 1), (n_txn // 2, "r", 0), (n_txn // 2, "w", 0)]
    old_t = next(t for t, (sn, _, _) in enumerate(txns) if sn < 10)
    spots.append((old_t, "w", 0))  # a TooOld transaction's range is validated too
    now = 30
    for spot in spots:
        t, kind, i = spot
        a, bb = (txns[t][1] if kind == "r" else txns[t][2])[i]
        if a == bb:
            continue
        b = engine.ConflictBatch(cs)
        with pytest.raises(engine.InvertedRange):
            b.add_packed(_packed(txns, inverted=spot))
        assert b.transaction_count == 0
        b.add_packed(_packed(txns))  # the same batch object, now valid
        got = b.detect_conflicts(now, 10)
        b.close()
        want, _ = ora.detect(_packed(txns), now, 10)
        np.testing.assert_array_equal(got, want)
        now += 5
    cs.close()


@pytest.mark.parametrize("bucket,cold", [("3000", "0"), ("600", "0"), ("40", "0"), ("160", "1"), ("64", "1"),
                                         ("8", "0")])
def test_sort_bucket_sizes_match(engine, oracle_mod, monkeypatch, bucket, cold):
    """Buckets past the per-wave capacity (ranked by their workgroup, the overflow list gathered),
    tiny ones, cold-start splitters from the batch's own samples, and warm splitters that no longer
    fit the keys (a plain batch after prefixed ones and back: most endpoints in a few buckets),
    with keys longer than the 16-byte prefix, give the same verdicts and reports."""
    monkeypatch.setenv("FDBCS_SORT_BUCKET", bucket)
    monkeypatch.setenv("FDBCS_SORT_COLD", cold)
    rng = np.random.default_rng(31)
    seq = []
    now = 10
    for i in range(6):
        pb = W.random_small_batch(rng, 700, alphabet=3, max_len=4, now=now, staleness=10, report_frac=0.5)
        if i % 2:  # every key behind a shared 17-byte prefix: prefix ties resolved by the tail bytes
            pb = prefixed(pb, b"\x02tenant\x00orders\x00\x15\x01")
        seq.append((pb, now, now - 3))
        now += 2
    e, _ = run_pair(engine, oracle_mod, seq)
    if bucket in ("3000", "600"):
        assert e.cs.stats()["sort_big_buckets"] > 0  # the workgroup path ran


def prefixed(pb, prefix):
    """The same batch with `prefix` prepended to every key (order and overlaps unchanged)."""
    lens = np.diff(pb.key_offsets)
    parts = [np.frombuffer(prefix, np.uint8)]
    out = []
    for k in range(len(lens)):
        out.append(parts[0])
        out.append(pb.key_bytes[pb.key_offsets[k] : pb.key_offsets[k + 1]])
    kb = np.concatenate(out) if out else np.zeros(0, np.uint8)
    ko = np.concatenate([[0], np.cumsum(lens + len(prefix))]).astype(np.int64)
    return PackedBatch(pb.read_snapshot, pb.report, pb.read_offsets, pb.write_offsets, kb, ko)


def test_sequential_fallback_matches(engine, oracle_mod, monkeypatch):
    """Force the candidate-edge overflow path (sequential MiniConflictSet replay on the GPU)."""
    monkeypatch.setenv("FDBCS_EDGE_CAP", "8")
    rng = np.random.default_rng(8)
    seq = []
    now = 10
    for _ in range(4):
        seq.append((W.random_small_batch(rng, 100, alphabet=2, max_len=3, now=now, staleness=10, report_frac=1.0),
                    now, now - 3))
        now += 2
    run_pair(engine, oracle_mod, seq)


def test_full_size_c2_properties(engine, oracle_mod):
    """BASELINE config C2 at full size (5M-boundary history, 5000 txns x 5R+2W): determinism
    (two engines, identical verdicts), parity with the skip-list restatement on the first
    batches, and history growth bounded by 2 boundaries per committed write."""
    p = W.C2Params()
    kb, ko, vers = W.c2_history(p, seed=1, start_version=10_000_000)
    a, b = EngineDriver(engine, gc_interval=0), EngineDriver(engine, gc_interval=1)
    a.load_history(kb, ko, vers)
    b.load_history(kb, ko, vers)
    o = oracle_mod.SkipListBaseline()
    o.load_history(kb, ko, vers)
    rng = np.random.default_rng(12)
    now = 10_000_000
    n0 = a.cs.history_size()
    assert n0 == len(vers)
    committed_writes = 0
    for i in range(4):
        now += p.version_step
        pb = W.c2_batch(p, rng, now)
        va, _ = a.detect(pb, now, now - p.window)
        vb, _ = b.detect(pb, now, now - p.window)
        assert (va == vb).all()
        vo, _ = o.detect(pb, now, now - p.window)
        assert (va == vo).all(), i
        committed_writes += int((va == 2).sum()) * p.writes
    assert a.cs.history_size() <= n0 + 2 * committed_writes


def test_cpp_shim_driver(tmp_path):
    """The reference-shaped C++ API (conflict_set_shim.hpp) end to end on the GPU."""
    import subprocess

    from tests.test_abi import build_shim_driver

    exe = build_shim_driver(str(tmp_path / "shim_driver"))
    out = subprocess.check_output([exe], text=True, timeout=120)
    assert "b1 commit=2 tooold=0 report1=1" in out, out
    assert "b2 commit=1 first=1" in out, out
    assert "b3 commit=0 report0=1 idx=1 arena=1" in out, out
    assert "b5 commit=2 tooold=1 late=1 late0=0 entries=0" in out, out
    assert "b6 commit=0 first=-1" in out, out


def test_sharded_engines_match_sharded_oracles(engine, oracle_mod):
    """Two key-range shards (two engine handles) fed by the proxy routing, combined by min, equal
    two oracles fed the same way (CommitProxyServer.actor.cpp:118-187, 764-780)."""
    from foundationdb_amd.sharding import KeyRangeSharding

    sh = KeyRangeSharding.uniform(2)
    engines = [EngineDriver(engine) for _ in range(2)]
    oracles = [oracle_mod.OracleConflictSet() for _ in range(2)]
    rng = np.random.default_rng(21)
    now = 10
    for _ in range(8):
        pb = W.random_small_batch(rng, 300, alphabet=256, max_len=3, now=now, staleness=10)
        parts = sh.route(pb)
        ve = [engines[g].detect(parts[g].batch, now, now - 5)[0] for g in range(2)]
        vo = [oracles[g].detect(parts[g].batch, now, now - 5)[0] for g in range(2)]
        for g in range(2):
            assert (ve[g] == vo[g]).all()
        assert (KeyRangeSharding.combine(pb.n_txn, parts, ve) == KeyRangeSharding.combine(pb.n_txn, parts, vo)).all()
        now += 3


def test_batch_outliving_its_set_is_refused_not_corrupting(engine):
    """Batches take pinned staging from a per-set pool; a batch destroyed after its set (garbage
    collection order in a binding) must neither touch the freed set nor crash, and calls on it are
    refused with FDBCS_E_STATE."""
    rng = np.random.default_rng(77)
    for _ in range(3):
        cs = engine.ConflictSet(0)
        done = engine.ConflictBatch(cs)
        done.add_packed(W.random_small_batch(rng, 50, now=10))
        done.detect_conflicts(10, 0)
        pending = engine.ConflictBatch(cs)
        pending.add_packed(W.random_small_batch(rng, 50, now=11))
        cs.close()
        with pytest.raises(engine.FdbcsError) as ex:
            pending.detect_conflicts(11, 0)
        assert ex.value.status == engine.FDBCS_E_STATE
        pending.close()
        done.close()


def test_empty_batches(engine, oracle_mod):
    """A resolver receives a request every batch even when no transaction routed to it has ranges
    there (Resolver.actor.cpp:103-310): empty batches and transactions without ranges must still
    advance the set (oldest version, GC) and agree with the oracle afterwards."""
    from tests.helpers import EngineDriver

    eng = EngineDriver(engine)
    ora = oracle_mod.OracleConflictSet()
    rng = np.random.default_rng(61)
    now = 10
    empty = PackedBatch.from_transactions([])
    no_ranges = PackedBatch.from_transactions([CommitTransaction([], [], now - 1) for _ in range(5)])
    for i in range(12):
        if i % 3 == 0:
            pb = empty
        elif i % 3 == 1:
            pb = no_ranges
        else:
            pb = W.random_small_batch(rng, 200, alphabet=8, max_len=2, now=now, staleness=15)
        ve, ce = eng.detect(pb, now, now - 12)
        vo, co = ora.detect(pb, now, now - 12)
        assert (ve == vo).all()
        assert ce == {t: sorted(v) for t, v in co.items()}
        now += 4


# Every engine knob that selects a different kernel or submission path (DESIGN.md §5 "Engine knobs")
# is parity-tested here; knobs measured slower and not kept were deleted with their code.
@pytest.mark.parametrize("knobs", [{"FDBCS_SPLIT_CHECK": "1"}, {"FDBCS_SPLIT_CHECK": "0"},
                                   {"FDBCS_SORT_COLD": "1"},
                                   {"FDBCS_SUBMIT_THREAD": "0", "FDBCS_SPLIT_CHECK": "1"}, {"FDBCS_SUBMIT_THREAD": "0"},
                                   {"FDBCS_WRITE_GROUPS": "0"}, {"FDBCS_SERIAL": "1"},
                                   {"FDBCS_DIRECTORY": "0"}, {"FDBCS_SKIP_EDGES": "0"}])
def test_pipeline_variants_match_oracle(engine, oracle_mod, knobs):
    """The engine's remaining path-selecting knobs stay exact: the unsplit and split read checks,
    cold-start splitters on every batch, one submitting thread, one candidate edge per writer (the
    production path past 12288 writes), the serial stream layout, base lookups without the radix
    directory, the no-edge launches kept."""
    saved = {k: os.environ.get(k) for k in knobs}
    os.environ.update(knobs)
    try:
        eng = EngineDriver(engine, gc_interval=0, delta_limit=400)  # compactions every few batches
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    ora = oracle_mod.OracleConflictSet()
    rng = np.random.default_rng(71)
    now = 10
    for i in range(20):
        # keys up to 24 bytes (short-key lookups) and up to 40 (long-key lookups) in some batches
        pb = W.random_small_batch(rng, 250, alphabet=6 if i % 2 else 200,
                                  max_len=24 if i % 3 == 0 else (40 if i % 5 == 1 else 3), now=now, staleness=12)
        ve, ce = eng.detect(pb, now, now - 9)
        vo, co = ora.detect(pb, now, now - 9)
        assert (ve == vo).all()
        assert ce == {t: sorted(v) for t, v in co.items()}
        now += 4
    assert eng.cs.history_size() > 0


def test_timing_level_changes_with_batches_in_flight(engine, oracle_mod):
    """Workspace reuse stays ordered when the timing level (and with it the stream layout) changes
    while more batches than workspaces are in flight (ev_b of a level-2 batch)."""
    cs = engine.ConflictSet(0)
    cs.set_gc_interval(3)
    ora = oracle_mod.OracleConflictSet()
    rng = np.random.default_rng(2024)
    now = 10
    levels = [2, 2, 2, 2, 0, 0, 0, 0, 1, 2, 0, 3, 3, 0, 0, 2, 1, 0]
    inflight = []
    for i, lv in enumerate(levels):
        cs.set_timing(lv)
        pb = W.random_small_batch(rng, 300, alphabet=5, max_len=3, now=now, staleness=10)
        b = engine.ConflictBatch(cs)
        b.add_packed(pb)
        b.detect_async(now, now - 8)
        want, _ = ora.detect(pb, now, now - 8)
        inflight.append((b, want, i))
        if len(inflight) > 5:  # keep more batches in flight than there are workspaces (3)
            bb, ww, j = inflight.pop(0)
            assert (bb.wait() == ww).all(), j
            bb.close()
        now += 3
    for bb, ww, j in inflight:
        assert (bb.wait() == ww).all(), j
        bb.close()
    assert cs.kernel_profile(), "timing level 3 recorded per-kernel events"
    cs.close()


def test_conflict_output_rejects_duplicate_ids(engine):
    """fdbcs_batch_set_conflict_output: two batch transactions may not share one global index (a
    duplicate would silently drop a conflict byte from the device combine)."""
    cs = engine.ConflictSet(0)
    pb = PackedBatch.from_transactions([CommitTransaction([KeyRange(b"a", b"b")], [], 5) for _ in range(3)])
    b = engine.ConflictBatch(cs)
    b.add_packed(pb)
    with pytest.raises(engine.FdbcsError):
        b.set_conflict_output(np.array([0, 2, 0], np.int32), 4, 1 << 20)
    b.close()
    cs.close()


def test_verdict_lists_match_oracle_lists(engine, oracle_mod, tmp_path):
    """Both host adapters over the HIP engine fill nonConflicting / tooOld exactly as the oracle's
    restatement of SkipList.cpp:869-876, with a tooOld list (Resolver.actor.cpp:194) and without one
    (skipListTest's call shape, SkipList.cpp:1077): the Python ConflictBatch and the C++ shim
    (tests/cpp/shim_driver.cpp --lists) on the KAT scenarios and random TooOld-heavy sequences.
    GetTooOldTransactions right after the adds (SkipList.cpp:836-842) equals the tooOld list."""
    import subprocess

    from tests.helpers import list_scenarios, oracle_scenario_lists, write_list_file
    from tests.test_abi import build_shim_driver

    scenarios = list_scenarios()
    want = oracle_scenario_lists(oracle_mod, scenarios)
    lines = []
    for steps, res in zip(scenarios, want):
        with_cs, without_cs = engine.ConflictSet(0), engine.ConflictSet(0)
        batches = iter(res)
        for st in steps:
            if st[0] == "clear":
                with_cs.clear(st[1])
                without_cs.clear(st[1])
                continue
            _, pb, now, no = st
            v, nc, to, nc2 = next(batches)
            got_nc, got_to, got_nc2 = [], [], []
            b = engine.ConflictBatch(with_cs)
            b.add_packed(pb)
            early = []
            b.get_too_old_transactions(early)  # GetTooOldTransactions before detect (SkipList.cpp:836-842)
            b.detect_conflicts(now, no, got_nc, got_to)
            b.close()
            assert early == to
            b = engine.ConflictBatch(without_cs)
            b.add_packed(pb)
            b.detect_conflicts(now, no, got_nc2)
            b.close()
            assert (got_nc, got_to, got_nc2) == (nc, to, nc2)
        with_cs.close()
        without_cs.close()
        for i, (v, nc, to, nc2) in enumerate(res):
            lines.append(f"L {i} with nc={','.join(map(str, nc))} to={','.join(map(str, to))}")
            lines.append(f"L {i} without nc={','.join(map(str, nc2))}")
    path = str(tmp_path / "lists.txt")
    write_list_file(scenarios, path)
    exe = build_shim_driver(str(tmp_path / "shim_driver"))
    out = subprocess.check_output([exe, "--lists", path], text=True, timeout=120)
    assert out.split("\n")[:-1] == lines
