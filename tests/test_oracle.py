"""CPU tests: the oracle pinned against the reference's known answers, cross-checked against the
skip-list restatement, and the semantic properties the reference's workloads assert."""
import numpy as np
import pytest

from foundationdb_amd import workloads as W
from foundationdb_amd.packing import CommitTransaction, KeyRange, PackedBatch
from tests.helpers import load_json, nonempty, random_fixture_sequences, scenario_batches


def test_ordering_kats(oracle_built):
    """operatorLessThanTest (SkipList.cpp:973-1005): all four asserts hold in the oracle's order."""
    for kat in load_json("ordering_kats.json"):
        a, b = kat["a"], kat["b"]
        ka, kb = bytes.fromhex(a[0]), bytes.fromhex(b[0])
        assert oracle_built.point_compare(ka, a[1], a[2], kb, b[1], b[2]) == -1, kat["name"]
        assert oracle_built.point_compare(kb, b[1], b[2], ka, a[1], a[2]) == 1, kat["name"]


@pytest.mark.parametrize("impl", ["OracleConflictSet", "SkipListBaseline"])
def test_kat_scenarios(oracle_built, impl):
    for scn in load_json("kat_scenarios.json"):
        cs = getattr(oracle_built, impl)()
        for i, (pb, now, no, expect, conf) in enumerate(scenario_batches(scn)):
            if scn.get("clear_before") == i:
                cs.clear(scn["clear_version"])
            v, c = cs.detect(pb, now, no)
            assert v.tolist() == expect, (scn["name"], i, v.tolist(), expect)
            if conf:
                assert nonempty(c) == conf, (scn["name"], c, conf)


def test_random_fixtures_reproduce(oracle_built):
    """The oracle still produces the committed regression vectors."""
    for s, seq in random_fixture_sequences():
        cs = oracle_built.OracleConflictSet()
        for pb, now, no, verdict, conf in seq:
            v, c = cs.detect(pb, now, no)
            assert (v == verdict).all(), s
            assert nonempty(c) == conf


def _random_sequence(rng, n_batches=6, **kw):
    now = 10
    out = []
    for _ in range(n_batches):
        pb = W.random_small_batch(rng, int(rng.integers(1, 60)), now=now, **kw)
        no = now - int(rng.integers(0, 15))
        out.append((pb, now, no))
        now += int(rng.integers(1, 6))
    return out


def test_oracle_vs_skiplist_random(oracle_built):
    rng = np.random.default_rng(7)
    for trial in range(120):
        a, b = oracle_built.OracleConflictSet(), oracle_built.SkipListBaseline()
        if trial % 4 == 0:
            a.clear(3)
            b.clear(3)
        for pb, now, no in _random_sequence(rng, alphabet=2 + trial % 4, max_len=1 + trial % 4):
            va, ca = a.detect(pb, now, no)
            vb, cb = b.detect(pb, now, no)
            assert (va == vb).all()
            assert ca == cb


def test_oracle_vs_skiplist_c1(oracle_built):
    a, b = oracle_built.OracleConflictSet(), oracle_built.SkipListBaseline()
    for pb, now, no in W.c1_batches(30, seed=3):
        va, _ = a.detect(pb, now, no)
        vb, _ = b.detect(pb, now, no)
        assert (va == vb).all()
    assert a.history_size() == b.history_size()


def test_gc_is_verdict_neutral(oracle_built):
    """removeBefore changes only the history size."""
    rng = np.random.default_rng(11)
    for _ in range(40):
        a, b = oracle_built.OracleConflictSet(), oracle_built.OracleConflictSet()
        for pb, now, no in _random_sequence(rng, n_batches=8):
            va, _ = a.detect(pb, now, no, gc=True)
            vb, _ = b.detect(pb, now, no, gc=False)
            assert (va == vb).all()


def _brute_verdicts(txns, history_fn, oldest):
    """Independent brute force over key space semantics (A.2-A.5) for property checks."""
    T = len(txns)
    status = []
    committed_writes = []
    for t, tr in enumerate(txns):
        if tr.read_snapshot < oldest and tr.read_conflict_ranges:
            status.append(1)
            continue
        hist = any(history_fn(r, tr.read_snapshot) for r in tr.read_conflict_ranges)
        if hist:
            status.append(0)
            continue
        intra = any(
            r.begin < w.end and w.begin < r.end and r.begin < r.end and w.begin < w.end
            for r in tr.read_conflict_ranges
            for w in committed_writes
        )
        if intra:
            status.append(0)
        else:
            status.append(2)
            committed_writes.extend(tr.write_conflict_ranges)
    return status


def test_single_batch_matches_keyspace_bruteforce(oracle_built):
    """Index-space MiniConflictSet == key-space overlap rule on an empty history."""
    rng = np.random.default_rng(5)
    for _ in range(200):
        pb = W.random_small_batch(rng, int(rng.integers(1, 30)), now=100, staleness=10)
        cs = oracle_built.OracleConflictSet()
        v, _ = cs.detect(pb, 100, 0)
        expect = _brute_verdicts(pb.to_transactions(), lambda r, s: False, 0)
        assert v.tolist() == expect


def test_report_conflicting_keys_properties(oracle_built):
    """ReportConflictingKeysWorkload properties (fdbserver/workloads/ReportConflictingKeys.actor.cpp:201-278):
    every reported read range intersects some write committed earlier (history or batch)."""
    rng = np.random.default_rng(9)
    cs = oracle_built.OracleConflictSet()
    written = []  # (range, version)
    now = 10
    for _ in range(10):
        pb = W.random_small_batch(rng, 40, now=now, staleness=8, report_frac=1.0)
        v, conf = cs.detect(pb, now, 0)
        txns = pb.to_transactions()
        batch_committed = []
        for t, tr in enumerate(txns):
            if v[t] == 0:
                assert t in conf and conf[t], "conflicting txn with report flag must report a read"
                for i in conf[t]:
                    r = tr.read_conflict_ranges[i]
                    hit_hist = any(r.intersects(w) and ver > tr.read_snapshot for w, ver in written) or (
                        r.empty() and True
                    )
                    hit_batch = any(r.intersects(w) for w in batch_committed)
                    assert hit_hist or hit_batch
            if v[t] == 2:
                batch_committed.extend(tr.write_conflict_ranges)
        written.extend((w, now) for w in batch_committed)
        now += 3


def test_inverted_range_rejected():
    from foundationdb_amd.packing import InvertedRange

    with pytest.raises(InvertedRange):
        KeyRange(b"b", b"a")


def test_packing_roundtrip():
    rng = np.random.default_rng(1)
    pb = W.random_small_batch(rng, 25)
    again = PackedBatch.from_transactions(pb.to_transactions())
    assert (again.key_bytes == pb.key_bytes).all() and (again.key_offsets == pb.key_offsets).all()
    assert (again.read_offsets == pb.read_offsets).all() and (again.write_offsets == pb.write_offsets).all()


def test_c1_generator_matches_reference_shape():
    """skipListTest data (SkipList.cpp:1023-1065): 2500 txns of 1R+1W, 16-byte setK keys, key2 in key+1..key+10."""
    pb, now, no = next(W.c1_batches(1, seed=1))
    assert pb.n_txn == 2500 and pb.n_reads == 2500 and pb.n_writes == 2500
    assert (np.diff(pb.key_offsets) == 16).all()
    ks = pb.key_bytes.reshape(-1, 16)
    assert (ks[:, :12] == ord(".")).all()
    vals = ks[:, 12:].copy().view(">u4").reshape(-1).astype(np.int64)
    d = vals[1::2] - vals[0::2]
    assert d.min() >= 1 and d.max() <= 10 and vals.max() < 20000000 + 11
    assert (now, no) == (50, 0)


def test_deterministic_random_restatement():
    """DeterministicRandom (flow/DeterministicRandom.cpp:22-53) on std::mt19937(1): gen64 pairs the raw
    words (r0 << 32) ^ r1; raw words of mt19937(1) start 1791095845, 4282876139."""
    g = W.DeterministicRandom(1).gen64(1)[0]
    assert int(g) == (1791095845 << 32) ^ 4282876139


def test_bounded_remove_before_matches_oracle(oracle_built):
    """The skip-list restatement's bounded, resumable removeBefore (SkipList.cpp:880-889: at most
    3 x |combined writes| + 10 nodes per batch, resuming at removalKey) is verdict-neutral and only
    ever shrinks the history toward what a full pass leaves."""
    rng = np.random.default_rng(23)
    for trial in range(30):
        a, b, c = oracle_built.OracleConflictSet(), oracle_built.SkipListBaseline(), oracle_built.SkipListBaseline()
        for pb, now, no in _random_sequence(rng, n_batches=12, alphabet=2 + trial % 3, max_len=2 + trial % 3):
            va, ca = a.detect(pb, now, no, gc=True)
            vb, cb = b.detect(pb, now, no, gc="bounded")
            vc, _ = c.detect(pb, now, no, gc=False)
            assert (va == vb).all() and (va == vc).all()
            assert ca == cb
            assert a.history_size() <= b.history_size() <= c.history_size()


def test_skiplist_restatement_c2_shape(oracle_built):
    """C2-shaped batches (5R+2W, 16-byte keys, prefilled history) through the interleaved CheckMax /
    striped-find restatement with bounded GC, against the semantic oracle."""
    p = W.C2Params(txns=600, history=30_000, staleness=20_000, window=40_000)
    kb, ko, vers = W.c2_history(p, seed=3, start_version=100_000)
    a, b = oracle_built.OracleConflictSet(), oracle_built.SkipListBaseline()
    a.load_history(kb, ko, vers)
    b.load_history(kb, ko, vers)
    rng = np.random.default_rng(4)
    now = 100_000
    seen = set()
    for _ in range(8):
        now += p.version_step
        pb = W.c2_batch(p, rng, now)
        va, _ = a.detect(pb, now, now - p.window, gc=False)
        vb, _ = b.detect(pb, now, now - p.window, gc="bounded")
        assert (va == vb).all()
        seen |= set(np.unique(va).tolist())
    assert {0, 2} <= seen


def test_conflicting_key_map_entries_follow_add_transaction(oracle_built):
    """conflictingKeyRangeMap[t] is created while addTransaction registers a reporting transaction's
    read ranges (SkipList.cpp:777-784): a reporting transaction that only writes gets no entry, a
    reporting reader that commits gets an empty one, a TooOld one none."""
    txns = [
        CommitTransaction([], [KeyRange(b"a", b"b")], 10, True),             # writes only
        CommitTransaction([KeyRange(b"x", b"y")], [], 10, True),             # reads, commits
        CommitTransaction([KeyRange(b"a", b"c")], [], 10, True),             # reads what txn 0 wrote
        CommitTransaction([KeyRange(b"m", b"n")], [], 1, True),              # TooOld below
    ]
    pb = PackedBatch.from_transactions(txns)
    cs = oracle_built.OracleConflictSet()
    cs.set_oldest_version(5)
    v, conf = cs.detect(pb, 10, 5)
    assert v.tolist() == [2, 2, 0, 1]
    assert conf == {1: [], 2: [0]}


def test_verdict_lists_follow_reference_loop(oracle_built):
    """The host adapters' list filling (conflict_set.fill_verdict_lists, mirrored in
    conflict_set_shim.hpp) equals the oracle's restatement of SkipList.cpp:869-876, with and
    without a tooOld list; without one a TooOld transaction lands in neither list (:820,830)."""
    from foundationdb_amd.conflict_set import fill_verdict_lists
    from tests.helpers import list_scenarios, oracle_scenario_lists

    saw_too_old = 0
    for res in oracle_scenario_lists(oracle_built, list_scenarios()):
        for v, nc, to, nc2 in res:
            a, b = [], []
            fill_verdict_lists(v, a, b)
            assert (a, b) == (nc, to)
            c = []
            fill_verdict_lists(v, c, None)
            assert c == nc2
            assert not set(to) & set(nc2)  # TooOld is in neither list without a tooOld list
            assert sorted(nc2 + to + np.flatnonzero(v == 0).tolist()) == list(range(len(v)))
            saw_too_old += len(to)
    assert saw_too_old > 10


@pytest.mark.parametrize("impl", ["OracleConflictSet", "SkipListBaseline"])
def test_add_before_previous_detect(oracle_built, impl):
    """A batch added before the previous batch's detect sees the oldest version from before that
    detect (ConflictBatch::addTransaction reads cs->oldestVersion, SkipList.cpp:770, 880-882): the
    `add_oldest` replay of bench.py's pre-packed batches.  Both restatements agree."""
    tr = lambda snap: CommitTransaction([KeyRange(b"a", b"b")], [KeyRange(b"c", b"d")], snap)  # noqa: E731
    pb = PackedBatch.from_transactions([tr(5), tr(15), tr(25)])
    cs = getattr(oracle_built, impl)()
    cs.detect(PackedBatch.from_transactions([]), 30, 20)  # oldest 0 -> 20
    v, _ = cs.detect(pb, 40, 20)  # added after: snapshots 5 and 15 are TooOld
    assert v.tolist() == [1, 1, 2]
    cs2 = getattr(oracle_built, impl)()
    cs2.detect(PackedBatch.from_transactions([]), 30, 20)
    v, _ = cs2.detect(pb, 40, 20, add_oldest=10)  # added while the oldest was 10: only snapshot 5
    assert v.tolist() == [1, 2, 2]
    v, _ = cs2.detect(pb, 50, 20)  # one-shot: the next batch sees the current oldest (20) again
    assert v.tolist()[:2] == [1, 1]
