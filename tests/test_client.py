"""Client conflict-range production (foundationdb_amd/client.py) against the NativeAPI rules it
restates (fdbclient/NativeAPI.actor.cpp:2597-2629, 2951-2966, 3097-3206, 3208-3316, 3434-3450,
3795-3850), and an end-to-end serializability property: clients doing read-modify-write through
the Transaction API, resolved by the conflict set, never lose an update."""
import numpy as np
import pytest

from foundationdb_amd import client as C
from foundationdb_amd.packing import KeyRange, PackedBatch


def tx(store=None, rv=10, **opts):
    return C.Transaction(store or C.VersionedStore(), rv, np.random.default_rng(0), C.TransactionOptions(**opts))


def test_read_conflict_range_clamp_and_empty_drop():
    t = tx()
    big = b"a" * 20_000
    t.add_read_conflict_range(b"a", big)
    assert t.read_conflict_ranges == [KeyRange(b"a", b"a" * 10_001)]  # limit + 1 bytes (:3185-3188)
    sysk = b"\xff" + b"s" * 40_000
    t.add_write_conflict_range(b"\xff", sysk)
    assert t.write_conflict_ranges == [KeyRange(b"\xff", sysk[:30_001])]
    # both ends clamp to the same key: the range became empty and is dropped (:3192-3194)
    t2 = tx()
    t2.add_read_conflict_range(b"b" * 10_001 + b"a", b"b" * 10_001 + b"b")
    assert t2.read_conflict_ranges == []
    with pytest.raises(AssertionError):
        t2.add_read_conflict_range(b"x", b"x")  # ASSERT(!keys.empty()) (:3178)


def test_point_reads_and_writes():
    s = C.VersionedStore()
    s.apply(5, [(C.SET_VALUE, b"k", b"v")])
    t = tx(s)
    assert t.get(b"k") == b"v"
    assert t.get(b"q", snapshot=True) is None
    assert t.get(b"z" * 10_001) is None  # cannot exist: no read, no conflict range (:2957-2958)
    assert t.read_conflict_ranges == [KeyRange(b"k", b"k\x00")]
    t.set(b"a", b"1")
    t.atomic_op(b"c", b"\x01", C.ADD_VALUE)
    t.atomic_op(b"vs", b"x" * 14, C.SET_VERSIONSTAMPED_KEY)  # no conflict range (:3247)
    t.clear(b"d")
    t.clear(b"e" * 10_001)  # ignored (:3279-3280)
    t.clear_range(b"m", b"m")  # empty: no mutation, no range
    assert t.write_conflict_ranges == [KeyRange(b"a", b"a\x00"), KeyRange(b"c", b"c\x00"), KeyRange(b"d", b"d\x00")]
    with pytest.raises(C.FDBError, match="key_too_large"):
        t.set(b"k" * 10_001, b"")
    with pytest.raises(C.FDBError, match="value_too_large"):
        t.set(b"k", b"v" * 100_001)


def test_read_only_transaction_does_not_commit():
    t = tx()
    t.get(b"a")
    assert t.commit_request() is None
    t2 = tx(read_only=True)
    t2.set(b"a", b"b")
    with pytest.raises(C.FDBError, match="transaction_read_only"):
        t2.commit_request()


def test_blind_write_becomes_self_conflicting():
    t = tx()
    t.get(b"r")
    t.set(b"w", b"1")  # writes do not intersect reads
    ct = t.commit_request()
    sc = [r for r in ct.read_conflict_ranges if r.begin.startswith(b"\xff/SC/")]
    assert len(sc) == 1 and sc[0] in ct.write_conflict_ranges
    assert len(sc[0].begin) == len(b"\xff/SC/") + 16 and sc[0].end == sc[0].begin + b"\x00"
    # causalWriteRisky: no self-conflict (:3844)
    t2 = tx(causal_write_risky=True)
    t2.set(b"w", b"1")
    assert not any(r.begin.startswith(b"\xff/SC/") for r in t2.commit_request().read_conflict_ranges)
    # read-modify-write already intersects: nothing added
    t3 = tx()
    t3.get(b"w")
    t3.set(b"w", b"2")
    assert t3.commit_request().read_conflict_ranges == [KeyRange(b"w", b"w\x00")]


def test_intersects_sorts_ranges_in_place():
    """intersects() sorts the VectorRefs it is given, which alias the transaction's arrays, so
    the read order the resolver (and its conflicting-key indices) sees is by begin."""
    t = tx()
    t.get(b"z")
    t.get(b"b")
    t.get(b"m")
    t.set(b"b", b"1")
    ct = t.commit_request()
    assert [r.begin for r in ct.read_conflict_ranges] == [b"b", b"m", b"z"]


def test_get_range_conflict_ranges():
    s = C.VersionedStore()
    s.apply(5, [(C.SET_VALUE, bytes([c]), b"v") for c in b"bdfhj"])
    fge = C.first_greater_or_equal
    # unlimited forward read: exactly the selector keys
    t = tx(s)
    rows = t.get_range(fge(b"c"), fge(b"i"))
    assert [k for k, _ in rows] == [b"d", b"f", b"h"]
    assert t.extra_conflict_ranges == [(b"c", b"i")]
    # limited forward read: ends just after the last key returned (keyAfter, :2621-2622)
    t = tx(s)
    rows = t.get_range(fge(b"c"), fge(b"i"), limit=2)
    assert [k for k, _ in rows] == [b"d", b"f"]
    assert t.extra_conflict_ranges == [(b"c", b"f\x00")]
    # limited reverse read: begins at the last key returned (:2608)
    t = tx(s)
    rows = t.get_range(fge(b"c"), fge(b"i"), limit=2, reverse=True)
    assert [k for k, _ in rows] == [b"h", b"f"]
    assert t.extra_conflict_ranges == [(b"f", b"i")]
    # reading from the beginning of the database (:2601-2602, 2651-2653)
    t = tx(s)
    t.get_range(fge(b""), fge(b"c"))
    assert t.extra_conflict_ranges == [(b"", b"c")]
    # through the end (:2615-2616)
    t = tx(s)
    t.get_range(fge(b"i"), fge(b"\xff\xff"))
    assert t.extra_conflict_ranges == [(b"i", b"\xff\xff")]
    # snapshot reads add nothing; an inverted request reads nothing
    t = tx(s)
    t.get_range(fge(b"a"), fge(b"z"), snapshot=True)
    assert t.get_range(fge(b"z"), fge(b"a")) == []
    assert t.extra_conflict_ranges == []
    # a ready range with begin < end is added as a read at commit (:3839-3842)
    t = tx(s)
    t.get_range(fge(b"c"), fge(b"i"), limit=1)
    t.set(b"d", b"x")
    ct = t.commit_request()
    assert KeyRange(b"c", b"d\x00") in ct.read_conflict_ranges


def test_get_key_conflict_ranges():
    s = C.VersionedStore()
    s.apply(5, [(C.SET_VALUE, bytes([c]), b"v") for c in b"bdf"])
    t = tx(s)
    assert t.get_key(C.first_greater_or_equal(b"c")) == b"d"
    assert t.get_key(C.last_less_or_equal(b"c")) == b"b"
    assert t.extra_conflict_ranges == [(b"c", b"d\x00"), (b"b", b"c\x00")]  # :3102-3105


def _run_increments(resolve, n_clients=12, rounds=40, keys=4, seed=5):
    """Read-modify-write counters through the Transaction API; every batch is resolved and the
    committed mutations applied at the batch's version.  Returns (store, committed count per key)."""
    rng = np.random.default_rng(seed)
    store = C.VersionedStore()
    store.apply(100, [(C.SET_VALUE, b"ctr%d" % k, (0).to_bytes(8, "little")) for k in range(keys)])
    version = 110
    committed = np.zeros(keys, np.int64)
    for _ in range(rounds):
        txns, reqs = [], []
        for _ in range(n_clients):
            rv = version - int(rng.integers(0, 3))  # some clients read a slightly stale version
            t = C.Transaction(store, rv, rng)
            k = int(rng.integers(0, keys))
            v = int.from_bytes(t.get(b"ctr%d" % k), "little")
            t.set(b"ctr%d" % k, (v + 1).to_bytes(8, "little"))
            if rng.random() < 0.3:
                t.get_range(C.first_greater_or_equal(b"ctr"), C.first_greater_or_equal(b"ctr\xff"), limit=2)
            txns.append((t, k))
            reqs.append(t.commit_request())
        version += 10
        pb = PackedBatch.from_transactions(reqs)
        verdicts = resolve(pb, version, version - 50)
        muts = []
        for (t, k), v in zip(txns, verdicts):
            if v == 2:
                muts.extend(t.mutations)
                committed[k] += 1
        store.apply(version, muts)
    return store, committed


def test_increments_are_serializable(oracle_built):
    """Every committed increment is reflected exactly once: the resolver saw the client's read
    and write conflict ranges, so no two committed increments read the same counter value."""
    cs = oracle_built.OracleConflictSet()

    def resolve(pb, now, no):
        return cs.detect(pb, now, no)[0]

    store, committed = _run_increments(resolve)
    for k in range(len(committed)):
        assert int.from_bytes(store.read(b"ctr%d" % k, store.version), "little") == committed[k]
    assert 0 < committed.sum() < 40 * 12  # some increments commit, some lose their race


def test_increments_without_conflict_ranges_lose_updates(oracle_built):
    """Control: the same clients with their read conflict ranges dropped lose updates, so the
    property above is really enforced by the ranges the client produced."""
    cs = oracle_built.OracleConflictSet()

    def resolve(pb, now, no):
        txns = pb.to_transactions()
        for t in txns:
            t.read_conflict_ranges = []
        return cs.detect(PackedBatch.from_transactions(txns), now, no)[0]

    store, committed = _run_increments(resolve)
    final = sum(int.from_bytes(store.read(b"ctr%d" % k, store.version), "little") for k in range(len(committed)))
    assert final < committed.sum()
