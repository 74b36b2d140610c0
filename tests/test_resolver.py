"""resolveBatch host logic (foundationdb_amd/resolver.py, Resolver.actor.cpp:103-310).

CPU tests inject an oracle-backed ConflictBatch (the checker) so that ordering, duplicates,
state transactions and counters are tested without a GPU; the GPU test runs the same request
stream through the HIP engine and compares replies."""
import numpy as np
import pytest

from foundationdb_amd import workloads as W
from foundationdb_amd.packing import CommitTransaction, KeyRange, PackedBatch, single_key_range
from foundationdb_amd.resolver import (
    Resolver,
    ResolveTransactionBatchRequest as Req,
    TransactionCommitted,
    TransactionConflict,
    TransactionTooOld,
)


class OracleBatch:
    """ConflictBatch-shaped adapter over the CPU oracle (test infrastructure only)."""

    def __init__(self, cs, conflicting_key_range_map=None):
        self.cs, self.map, self.txns = cs, conflicting_key_range_map, []

    def add_transaction(self, t):
        self.txns.append(t)

    def detect_conflicts(self, now, new_oldest, non_conflicting, too_old):
        pb = PackedBatch.from_transactions(self.txns)
        v, conf = self.cs.detect(pb, now, new_oldest)
        for t, x in enumerate(v):
            if x == TransactionTooOld:
                too_old.append(t)
            elif x == TransactionCommitted:
                non_conflicting.append(t)
        if self.map is not None:  # the oracle returns exactly the reference's map entries
            for t, x in conf.items():
                self.map.setdefault(t, []).extend(x)
        return v


def _resolver(oracle_built, **kw):
    from oracle import oracle

    return Resolver(conflict_set=oracle.OracleConflictSet(), batch_factory=OracleBatch, **kw)


def _txn(reads=(), writes=(), snap=0, report=False):
    return CommitTransaction([single_key_range(k) for k in reads], [single_key_range(k) for k in writes], snap, report)


def test_in_order_verdicts_match_conflict_batch(oracle_built):
    from oracle import oracle

    r = _resolver(oracle_built, max_write_transaction_life_versions=3000)
    ref = oracle.OracleConflictSet()
    rng = np.random.default_rng(3)
    prev, v = -1, 1000
    for i in range(6):
        pb = W.random_small_batch(rng, 64, alphabet=5, max_len=4, now=v, staleness=3000)
        txns = pb.to_transactions()
        done = r.submit(Req(prev, v, prev, txns, proxy=None if prev < 0 else "p0"))
        assert len(done) == 1
        want, _ = ref.detect(PackedBatch.from_transactions(txns), v, v - 3000)
        assert done[0][1].committed == want.tolist()
        prev, v = v, v + 1000
    c = r.counters
    assert c["ResolveBatchStart"] == 6 and c["ResolveBatchIn"] == 6 == c["ResolveBatchOut"]
    assert c["TransactionsAccepted"] + c["TransactionsTooOld"] + c["TransactionsConflicted"] == 6 * 64


def test_out_of_order_requests_wait_for_their_predecessor(oracle_built):
    r = _resolver(oracle_built)
    assert [x[0].version for x in r.submit(Req(-1, 10, -1, []))] == [10]
    # v30 (prev 20) arrives before v20 (prev 10): held until v20 runs
    assert r.submit(Req(20, 30, 0, [_txn(reads=[b"a"], snap=20)], proxy="p0")) == []
    assert [q.version for q in r.held] == [30]
    done = r.submit(Req(10, 20, 0, [_txn(writes=[b"a"])], proxy="p0"))
    assert [q.version for q, _ in done] == [20, 30]
    # v20 wrote a at 20; v30's read at snapshot 20 sees no newer write
    assert done[1][1].committed == [TransactionCommitted]
    assert r.version == 30 and not r.held


def test_duplicate_request_gets_cached_reply_until_acknowledged(oracle_built):
    r = _resolver(oracle_built)
    r.submit(Req(-1, 10, -1, []))
    (q1, rep1), = r.submit(Req(10, 20, 0, [_txn(writes=[b"k"])], proxy="p0"))
    r.submit(Req(20, 30, 0, [_txn(reads=[b"k"], snap=10)], proxy="p0"))
    # resend of v20: not re-resolved, same reply
    (qd, repd), = r.submit(Req(10, 20, 0, [_txn(writes=[b"k"])], proxy="p0"))
    assert repd is rep1 and r.counters["ResolveBatchStart"] == 3
    # v40 acknowledges everything up to 30 (lastReceivedVersion): the v20 reply is dropped
    r.submit(Req(30, 40, 30, [], proxy="p0"))
    (_, gone), = r.submit(Req(10, 20, 0, [_txn(writes=[b"k"])], proxy="p0"))
    assert gone is None  # reply.send(Never())


def test_state_transactions_reach_every_proxy_then_prune(oracle_built):
    r = _resolver(oracle_built, commit_proxy_count=2)
    r.submit(Req(-1, 10, -1, []))
    muts = [(b"\xff/conf/x", b"1")]
    (_, ra), = r.submit(Req(10, 20, 0, [_txn(writes=[b"\xff/conf/x"])], [0], {0: muts}, proxy="A"))
    # one (empty) entry per earlier version: the master's v10 (recentStateTransactions[version] is
    # created for every batch, Resolver.actor.cpp:213)
    assert ra.committed == [TransactionCommitted] and ra.state_mutations == [[]]
    assert r.total_state_bytes == len(muts[0][0]) + len(muts[0][1])
    # proxy B has not seen v20: its reply carries A's state transaction
    (_, rb), = r.submit(Req(20, 30, 0, [], proxy="B"))
    assert len(rb.state_mutations) == 2 and rb.state_mutations[1][0].committed
    assert rb.state_mutations[1][0].mutations == muts
    # every proxy has now seen v20: pruned
    assert 20 not in r.recent_state_transactions and r.total_state_bytes == 0


def test_state_memory_back_pressure_holds_a_proxy_that_is_ahead(oracle_built):
    r = _resolver(oracle_built, commit_proxy_count=2, state_memory_limit=4)
    r.submit(Req(-1, 10, -1, []))
    r.submit(Req(10, 20, 0, [_txn()], [0], {0: [(b"\xff/a", b"0123456789")]}, proxy="A"))
    r.submit(Req(20, 30, 0, [], proxy="A"))
    # A is past the oldest unpruned state version and state bytes exceed the limit: held
    assert r.submit(Req(30, 40, 0, [], proxy="A")) == [] and [q.version for q in r.held] == [40]
    r.state_memory_limit = 10**6
    assert [q.version for q, _ in r.poll()] == [40]


def test_back_pressure_is_checked_once_at_arrival(oracle_built):
    """A request that got past the state-memory check while it waited for its predecessor is not
    held again when that predecessor pushes totalStateBytes over the limit: the actor checks
    back-pressure once (Resolver.actor.cpp:126-133), then only waits on the version (:139-150)."""
    r = _resolver(oracle_built, commit_proxy_count=2, state_memory_limit=4)
    r.submit(Req(-1, 10, -1, []))
    assert r.submit(Req(20, 30, 0, [], proxy="A")) == []  # waits for v20, no state bytes yet
    done = r.submit(Req(10, 20, 0, [_txn()], [0], {0: [(b"\xff/a", b"0123456789")]}, proxy="A"))
    assert [q.version for q, _ in done] == [20, 30]
    assert r.total_state_bytes > r.state_memory_limit
    # a request arriving now does meet the back-pressure loop
    assert r.submit(Req(30, 40, 0, [], proxy="A")) == [] and [q.version for q in r.held] == [40]


def test_conflicting_key_map_reported(oracle_built):
    r = _resolver(oracle_built)
    r.submit(Req(-1, 10, -1, []))
    t0 = _txn(writes=[b"x"])
    t1 = CommitTransaction([KeyRange(b"a", b"b"), single_key_range(b"x")], [], 10, True)
    (_, rep), = r.submit(Req(10, 20, 0, [t0, t1], proxy="p0"))
    assert rep.committed == [TransactionCommitted, TransactionConflict]
    assert rep.conflicting_key_range_map == {1: [1]}


@pytest.mark.gpu
def test_resolver_on_gpu_matches_oracle(oracle_built):
    """The same request stream through the HIP conflict set and through the oracle."""
    from foundationdb_amd import conflict_set as C

    gpu = Resolver(conflict_set=C.new_conflict_set(), batch_factory=C.ConflictBatch,
                   max_write_transaction_life_versions=3000)
    ref = _resolver(oracle_built, max_write_transaction_life_versions=3000)
    rng = np.random.default_rng(11)
    prev, v = -1, 1000
    reqs = []
    for i in range(8):
        pb = W.random_small_batch(rng, 200, alphabet=6, max_len=5, now=v, staleness=3000)
        txns = pb.to_transactions()
        for t in txns[::7]:
            t.report_conflicting_keys = True
        reqs.append(Req(prev, v, prev, txns, proxy=None if prev < 0 else "p0"))
        prev, v = v, v + 1000
    # deliver out of order in pairs: both resolvers must hold and release identically
    order = [1, 0, 3, 2, 5, 4, 7, 6]
    for k in order:
        a, b = gpu.submit(reqs[k]), ref.submit(reqs[k])
        assert [q.version for q, _ in a] == [q.version for q, _ in b]
        for (_, ra), (_, rb) in zip(a, b):
            assert ra.committed == rb.committed
            assert {t: sorted(x) for t, x in ra.conflicting_key_range_map.items()} == \
                   {t: sorted(x) for t, x in rb.conflicting_key_range_map.items()}
    assert gpu.version == ref.version == reqs[-1].version
