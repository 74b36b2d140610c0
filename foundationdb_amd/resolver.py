"""The Resolver role's batch handler over the HIP conflict set.

Restates ``resolveBatch`` (fdbserver/Resolver.actor.cpp:103-310) without the flow actor runtime:
requests are submitted as they arrive from commit proxies, and the handler completes them in
version order, the way the actor's ``version.whenAtLeast(prevVersion)`` wait does (:155-163).

What it reproduces:

* Version chaining: a request runs only when the resolver's version equals its ``prev_version``
  (:155-168). Later requests are held and run as soon as their predecessor has run.
* Duplicates: a request whose ``prev_version`` the resolver has already passed gets the reply
  cached for its ``version`` in that proxy's outstanding batches, or no reply when that batch has
  been acknowledged (:167, :290-305; ``reply.send(Never())`` is ``None`` here).
* Verdict bytes: ``ConflictBatch`` over the GPU conflict set with
  ``newOldestVersion = version - MAX_WRITE_TRANSACTION_LIFE_VERSIONS`` (:179-204). Reply bytes use
  the ``ConflictSet.h:40-44`` encoding. The conflicting-key map is filled for transactions that
  ask for it.
* Outstanding batches per proxy, acknowledged through ``last_received_version`` (:171-173).
* State transactions: ``txn_state_transactions`` with their commit flag are kept per version.
  Every reply carries those of versions in ``[firstUnseenVersion, version)``, and they are pruned
  once every proxy has seen them (:213-280).
* State-memory back-pressure: a request is held while the state bytes exceed
  ``RESOLVER_STATE_MEMORY_LIMIT`` under the conditions of :126-131. ``neededVersion`` is raised as
  at :143-146.
* Counters with the reference's names (:60-75).

The conflict set is injected so that the host logic can be tested on CPU against the oracle. The
product default is the HIP conflict set, with no fallback.
"""
from __future__ import annotations

from collections import deque
from dataclasses import dataclass, field
from typing import Callable, Deque, Dict, List, Optional, Tuple

from .packing import CommitTransaction

MAX_WRITE_TRANSACTION_LIFE_VERSIONS = 5_000_000  # fdbserver/Knobs.cpp:41 (5 * VERSIONS_PER_SECOND)
RESOLVER_STATE_MEMORY_LIMIT = 1_000_000  # fdbserver/Knobs.cpp:428

TransactionConflict = 0
TransactionTooOld = 1
TransactionCommitted = 2

MASTER = None  # proxy id of the master's first request (prevVersion < 0, Resolver.actor.cpp:111)


@dataclass
class StateTransaction:
    """StateTransactionRef (ResolverInterface.h:62-77): commit flag + the transaction's mutations."""

    committed: bool
    mutations: list


@dataclass
class ResolveTransactionBatchRequest:
    """ResolveTransactionBatchRequest (ResolverInterface.h:96-111). ``proxy`` names the sending
    commit proxy (the reply endpoint's address in the reference); ``mutations`` of a transaction
    are given per index in ``transaction_mutations`` (only state transactions need them)."""

    prev_version: int
    version: int
    last_received_version: int
    transactions: List[CommitTransaction]
    txn_state_transactions: List[int] = field(default_factory=list)
    transaction_mutations: Dict[int, list] = field(default_factory=dict)
    proxy: object = 0
    debug_id: Optional[object] = None


@dataclass
class ResolveTransactionBatchReply:
    """ResolveTransactionBatchReply (ResolverInterface.h:80-94)."""

    committed: List[int] = field(default_factory=list)
    state_mutations: List[List[StateTransaction]] = field(default_factory=list)
    conflicting_key_range_map: Dict[int, List[int]] = field(default_factory=dict)
    debug_id: Optional[object] = None


@dataclass
class _ProxyRequestsInfo:  # Resolver.actor.cpp:35-41
    outstanding_batches: Dict[int, ResolveTransactionBatchReply] = field(default_factory=dict)
    last_version: int = -1


def _mutation_bytes(mutations: list) -> int:
    """expectedSize() of a mutation list: bytes of its params (MutationRef param1 + param2)."""
    total = 0
    for m in mutations:
        if isinstance(m, (bytes, bytearray)):
            total += len(m)
        elif isinstance(m, tuple):
            total += sum(len(x) for x in m if isinstance(x, (bytes, bytearray)))
    return total


class Resolver:
    """One resolver (Resolver.actor.cpp:43-99) owning one conflict set.

    ``conflict_set`` is the conflict set to resolve against. ``batch_factory(cs, conflict_map)``
    returns an object with ``add_transaction`` and ``detect_conflicts(now, new_oldest,
    non_conflicting, too_old)``: by default the HIP ``ConflictBatch``."""

    def __init__(self, commit_proxy_count: int = 1, resolver_count: int = 1, conflict_set=None,
                 batch_factory: Optional[Callable] = None,
                 max_write_transaction_life_versions: int = MAX_WRITE_TRANSACTION_LIFE_VERSIONS,
                 state_memory_limit: int = RESOLVER_STATE_MEMORY_LIMIT):
        if conflict_set is None or batch_factory is None:
            from . import conflict_set as C  # the product path: HIP engine, raises without a GPU

            conflict_set = conflict_set if conflict_set is not None else C.new_conflict_set()
            batch_factory = batch_factory or C.ConflictBatch
        self.commit_proxy_count = commit_proxy_count
        self.resolver_count = resolver_count
        self.conflict_set = conflict_set
        self._batch_factory = batch_factory
        self.life_versions = max_write_transaction_life_versions
        self.state_memory_limit = state_memory_limit
        self.version = -1  # NotifiedVersion version(-1), :79
        self.needed_version = 0
        self.recent_state_transactions: Dict[int, List[StateTransaction]] = {}
        self.recent_state_transaction_sizes: Deque[Tuple[int, int]] = deque()
        self.total_state_bytes = 0
        self.proxy_info: Dict[object, _ProxyRequestsInfo] = {}
        self.debug_min_recent_state_version = 0
        self._held: List[ResolveTransactionBatchRequest] = []
        self._past_pressure: set = set()  # held requests already through the back-pressure loop (:126-133)
        self.counters = {k: 0 for k in (
            "ResolveBatchIn", "ResolveBatchStart", "ResolvedTransactions", "ResolvedBytes",
            "ResolvedReadConflictRanges", "ResolvedWriteConflictRanges", "TransactionsAccepted",
            "TransactionsTooOld", "TransactionsConflicted", "ResolvedStateTransactions",
            "ResolvedStateMutations", "ResolvedStateBytes", "ResolveBatchOut")}

    # ------------------------------------------------------------------ request flow
    def submit(self, req: ResolveTransactionBatchRequest
               ) -> List[Tuple[ResolveTransactionBatchRequest, Optional[ResolveTransactionBatchReply]]]:
        """Receive one request. Returns every (request, reply) pair that completed as a result,
        in completion order: this request and any held requests it unblocked. A reply of
        ``None`` is the reference's ``reply.send(Never())``."""
        self.counters["ResolveBatchIn"] += 1
        self._held.append(req)
        return self.poll()

    def poll(self) -> List[Tuple[ResolveTransactionBatchRequest, Optional[ResolveTransactionBatchReply]]]:
        """Run every held request that has become ready (the actor's wake-ups on version,
        totalStateBytes and neededVersion changes, :130, :149-151)."""
        done = []
        progress = True
        while progress:
            progress = False
            for r in list(self._held):
                if self._ready(r):
                    self._held.remove(r)
                    self._past_pressure.discard(id(r))
                    done.append((r, self._resolve(r)))
                    progress = True
                    break
        return done

    @property
    def held(self) -> List[ResolveTransactionBatchRequest]:
        """Requests waiting on their predecessor version or on state-memory back-pressure."""
        return list(self._held)

    def _proxy_key(self, req):
        return MASTER if req.prev_version < 0 else req.proxy  # :111

    def _ready(self, req) -> bool:
        info = self.proxy_info.setdefault(self._proxy_key(req), _ProxyRequestsInfo())
        # back-pressure on state-transaction memory (:126-133): checked until the request gets past
        # it once; after that the actor only waits on its predecessor version (:139-150)
        if id(req) not in self._past_pressure:
            if (self.total_state_bytes > self.state_memory_limit and self.recent_state_transaction_sizes
                    and info.last_version > self.recent_state_transaction_sizes[0][0]
                    and req.version > self.needed_version):
                return False
            self._past_pressure.add(id(req))
        # :143-146: a proxy behind the oldest recent state version raises neededVersion
        if self.recent_state_transaction_sizes and info.last_version <= self.recent_state_transaction_sizes[0][0]:
            self.needed_version = max(self.needed_version, req.prev_version)
        return self.version >= req.prev_version  # version.whenAtLeast(prevVersion), :149

    def _resolve(self, req) -> Optional[ResolveTransactionBatchReply]:
        key = self._proxy_key(req)
        info = self.proxy_info[key]
        if self.version == req.prev_version:  # not a duplicate (:167)
            self._run_batch(req, info)
        # a duplicate falls through to the cached reply (:290-305)
        self.counters["ResolveBatchOut"] += 1
        return info.outstanding_batches.get(req.version)

    def _run_batch(self, req, info: _ProxyRequestsInfo) -> None:
        c = self.counters
        c["ResolveBatchStart"] += 1
        c["ResolvedTransactions"] += len(req.transactions)
        c["ResolvedBytes"] += sum(_txn_bytes(t) for t in req.transactions)
        if info.last_version > 0:  # :171-173
            for v in [v for v in info.outstanding_batches if v <= req.last_received_version]:
                del info.outstanding_batches[v]
        first_unseen = info.last_version + 1
        info.last_version = req.version
        reply = ResolveTransactionBatchReply(debug_id=req.debug_id)
        info.outstanding_batches[req.version] = reply

        batch = self._batch_factory(self.conflict_set, reply.conflicting_key_range_map)
        for t in req.transactions:
            batch.add_transaction(t)
            c["ResolvedReadConflictRanges"] += len(t.read_conflict_ranges)
            c["ResolvedWriteConflictRanges"] += len(t.write_conflict_ranges)
        commit_list: List[int] = []
        too_old_list: List[int] = []
        batch.detect_conflicts(req.version, req.version - self.life_versions, commit_list, too_old_list)
        if hasattr(batch, "close"):
            batch.close()

        committed = [TransactionConflict] * len(req.transactions)  # :197-204
        for t in commit_list:
            committed[t] = TransactionCommitted
        for t in too_old_list:
            assert committed[t] == TransactionConflict
            committed[t] = TransactionTooOld
        reply.committed = committed
        c["TransactionsAccepted"] += len(commit_list)
        c["TransactionsTooOld"] += len(too_old_list)
        c["TransactionsConflicted"] += len(req.transactions) - len(commit_list) - len(too_old_list)

        # state transactions (:210-237)
        assert req.prev_version >= 0 or not req.txn_state_transactions  # :210
        states = self.recent_state_transactions.setdefault(req.version, [])
        state_mutations = state_bytes = 0
        for t in req.txn_state_transactions:
            muts = list(req.transaction_mutations.get(t, []))
            state_mutations += len(muts)
            state_bytes += _mutation_bytes(muts)
            states.append(StateTransaction(committed[t] == TransactionCommitted, muts))
        c["ResolvedStateTransactions"] += len(req.txn_state_transactions)
        c["ResolvedStateMutations"] += state_mutations
        c["ResolvedStateBytes"] += state_bytes
        if state_bytes > 0:
            self.recent_state_transaction_sizes.append((req.version, state_bytes))
        assert req.version >= first_unseen
        assert first_unseen >= self.debug_min_recent_state_version
        # every state transaction of versions [firstUnseenVersion, version) this proxy has not seen
        reply.state_mutations = [self.recent_state_transactions[v]
                                 for v in sorted(self.recent_state_transactions) if first_unseen <= v < req.version]

        # prune what every proxy has seen (:254-273)
        oldest_proxy_version = req.version
        for k, pi in self.proxy_info.items():
            if k is not MASTER:
                oldest_proxy_version = min(pi.last_version, oldest_proxy_version)
        if first_unseen <= oldest_proxy_version and len(self.proxy_info) == self.commit_proxy_count + 1:
            for v in [v for v in self.recent_state_transactions if v <= oldest_proxy_version]:
                del self.recent_state_transactions[v]
            self.debug_min_recent_state_version = oldest_proxy_version + 1
            while self.recent_state_transaction_sizes and self.recent_state_transaction_sizes[0][0] <= oldest_proxy_version:
                state_bytes -= self.recent_state_transaction_sizes.popleft()[1]
        self.version = req.version
        self.total_state_bytes += state_bytes


def _txn_bytes(t: CommitTransaction) -> int:
    """expectedSize() of the conflict ranges (the part of CommitTransactionRef this path sees)."""
    n = 0
    for r in list(t.read_conflict_ranges) + list(t.write_conflict_ranges):
        n += len(r.begin) + len(r.end)
    return n
