"""Dynamic resharding of the key space across resolvers.

Three reference pieces, restated without the flow runtime (time is explicit: FDB's ``now()``
seconds; the multi-GPU driver derives it from versions, 1e6 versions per second):

* the resolver's iops sample (fdbserver/Resolver.actor.cpp:178-192, 327-337): every range begin a
  resolver sees is added to a ``TransientStorageMetricSample`` with metric
  SAMPLE_OFFSET_PER_KEY + len(begin), expiring SAMPLE_EXPIRATION_TIME later
  (StorageMetrics.actor.h:35-189), and a resolver answers metrics requests with the sampled total
  and split requests with ``splitEstimate``;
* the master's ``resolutionBalancing`` and ``findRange`` (masterserver.actor.cpp:1073-1179): when
  the busiest and idlest resolvers differ by more than MIN_BALANCE_DIFFERENCE, move about half of
  the smaller excess from the busiest to the idlest, growing an existing border between the two
  first, then creating a new one, splitting ranges at the busiest resolver's sample;
* the proxies' ``keyResolvers`` ownership history that the moves feed
  (sharding.KeyResolvers, CommitProxyServer.actor.cpp:147-174, 622-626, 1284-1297).

Moving a range never moves history: reads whose snapshot predates the move still go to the old
owner, which holds the writes made before it, until MAX_WRITE_TRANSACTION_LIFE_VERSIONS have
passed (sharding.KeyResolvers).  So no GPU-to-GPU copy is needed; only routing changes.
"""
from __future__ import annotations

import bisect
from collections import deque
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

from .packing import PackedBatch

# fdbserver/Knobs.cpp:411-427, fdbclient/Knobs.cpp:74-77
KEY_BYTES_PER_SAMPLE = 20_000
MIN_BALANCE_TIME = 0.2
MIN_BALANCE_DIFFERENCE = 1_000_000
SAMPLE_OFFSET_PER_KEY = 100
SAMPLE_EXPIRATION_TIME = 1.0
SAMPLE_POLL_TIME = 0.1
KEY_SIZE_LIMIT = 10_000
SPLIT_KEY_SIZE_LIMIT = KEY_SIZE_LIMIT // 2
ALL_KEYS_END = b"\xff\xff"  # allKeys = ["", \xff\xff) (SystemData.cpp)
VERSIONS_PER_SECOND = 1_000_000


class OperationFailed(Exception):
    """operation_failed(): findRange has nothing left to move (masterserver.actor.cpp:1120)."""


def key_between(begin: bytes, end: bytes) -> bytes:
    """keyBetween (fdbclient/FDBTypes.h:516-537): the shortest key in [begin, end] (or end),
    within SPLIT_KEY_SIZE_LIMIT."""
    pos = 0
    m = min(len(begin), len(end))
    while pos < m and pos < SPLIT_KEY_SIZE_LIMIT:
        if begin[pos] != end[pos]:
            return end[: pos + 1]
        pos += 1
    if pos < SPLIT_KEY_SIZE_LIMIT and len(begin) < len(end):
        return end[: pos + 1]
    return end


class StorageMetricSample:
    """StorageMetricSample (StorageMetrics.actor.h:35-84): an ordered key -> metric map with
    prefix sums (IndexedSet<Key, int64_t>)."""

    def __init__(self, metric_units_per_sample: int):
        self.metric_units_per_sample = metric_units_per_sample
        self.keys: List[bytes] = []
        self.vals: List[int] = []

    # IndexedSet primitives
    def lower_bound(self, k: bytes) -> int:
        return bisect.bisect_left(self.keys, k)

    def sum_to(self, i: int) -> int:
        return sum(self.vals[:i])

    def index(self, metric: int) -> int:
        """Smallest x such that sumTo(x+1) > metric, or end (IndexedSet.h:269)."""
        s = 0
        for i, v in enumerate(self.vals):
            s += v
            if s > metric:
                return i
        return len(self.keys)

    def add_metric(self, k: bytes, metric: int) -> int:
        """addMetric: add to k's value (inserting it); returns the new value."""
        i = self.lower_bound(k)
        if i < len(self.keys) and self.keys[i] == k:
            self.vals[i] += metric
            return self.vals[i]
        self.keys.insert(i, k)
        self.vals.insert(i, metric)
        return metric

    def erase(self, k: bytes) -> None:
        i = self.lower_bound(k)
        if i < len(self.keys) and self.keys[i] == k:
            del self.keys[i]
            del self.vals[i]

    def insert(self, k: bytes, metric: int) -> None:
        self.erase(k)
        self.add_metric(k, metric)

    # StorageMetricSample
    def get_estimate(self, begin: bytes, end: Optional[bytes]) -> int:
        """sumRange(begin, end) (:41-43); end None = the end of the key space."""
        i0 = self.lower_bound(begin)
        i1 = len(self.keys) if end is None else self.lower_bound(end)
        return sum(self.vals[i0:i1])

    def total(self) -> int:
        return sum(self.vals)

    def split_estimate(self, begin: bytes, end: bytes, offset: int, front: bool = True) -> bytes:
        """splitEstimate (:44-83): the key about `offset` metric units into [begin, end) from the
        front (or back), moved to the shortest key between neighbouring samples, butterfly search."""
        base = self.sum_to(self.lower_bound(begin)) + offset if front else self.sum_to(self.lower_bound(end)) - offset
        fwd = self.index(base)
        n = len(self.keys)
        if fwd == n or self.keys[fwd] >= end:
            return end
        if not front and self.keys[fwd] <= begin:
            return begin
        bck = fwd
        while (fwd != n and self.keys[fwd] < end) or (bck != 0 and self.keys[bck] > begin):
            if bck != 0 and self.keys[bck] > begin:
                it = bck
                bck -= 1
                lo = max(self.keys[bck], begin) if bck != 0 else begin
                split = key_between(lo, self.keys[it])
                if not front or (self.get_estimate(begin, split) > 0 and len(split) <= SPLIT_KEY_SIZE_LIMIT):
                    return split
            if fwd != n and self.keys[fwd] < end:
                it = fwd + 1
                hi = min(self.keys[it], end) if it != n else end
                split = key_between(self.keys[fwd], hi)
                if front or (self.get_estimate(split, end) > 0 and len(split) <= SPLIT_KEY_SIZE_LIMIT):
                    return split
                fwd = it
        return end if front else begin


class TransientStorageMetricSample(StorageMetricSample):
    """TransientStorageMetricSample (StorageMetrics.actor.h:103-189): sampled metric with expiry.
    `rng` supplies random01() (deterministicRandom() in the reference)."""

    def __init__(self, metric_units_per_sample: int, rng: Optional[np.random.Generator] = None):
        super().__init__(metric_units_per_sample)
        self.queue: deque = deque()  # (expiration, key, -delta)
        self.rng = rng if rng is not None else np.random.default_rng(0)

    def _roll(self, metric: int) -> bool:
        return self.rng.random() < metric / self.metric_units_per_sample

    def add(self, key: bytes, metric: int) -> int:
        if not metric:
            return 0
        mag = abs(metric)
        if mag < self.metric_units_per_sample:
            if not self._roll(mag):
                return 0
            metric = -self.metric_units_per_sample if metric < 0 else self.metric_units_per_sample
        if self.add_metric(key, metric) == 0:
            self.erase(key)
        return metric

    def add_and_expire(self, key: bytes, metric: int, expiration: float) -> int:
        x = self.add(key, metric)
        if x:
            self.queue.append((expiration, key, -x))
        return x

    def poll(self, now: float) -> None:
        while self.queue and self.queue[0][0] <= now:
            _, key, delta = self.queue.popleft()
            assert delta != 0
            if self.add_metric(key, delta) == 0:
                self.erase(key)


class ResolverLoad:
    """The resolver side of balancing (Resolver.actor.cpp:58, 178-192, 318-342): the iops sample
    fed by every batch when there is more than one resolver, metrics and split replies."""

    def __init__(self, resolver_count: int, rng: Optional[np.random.Generator] = None,
                 key_bytes_per_sample: int = KEY_BYTES_PER_SAMPLE):
        self.resolver_count = resolver_count
        self.sample = TransientStorageMetricSample(key_bytes_per_sample, rng)
        self.metrics_requests = 0
        self.split_requests = 0

    def add_batch(self, pb: PackedBatch, now: float) -> None:
        """:178-192: write then read range begins of every transaction, expiring at now + 1 s.
        Vectorized roll: a begin key of metric m < 20000 is sampled with probability m/20000."""
        if self.resolver_count <= 1 or pb.n_txn == 0:
            return
        expire = now + SAMPLE_EXPIRATION_TIME
        R = pb.n_reads
        offs = pb.key_offsets
        order = []
        for t in range(pb.n_txn):  # per transaction: its writes, then its reads (:188-191)
            order.extend(2 * (R + w) for w in range(pb.write_offsets[t], pb.write_offsets[t + 1]))
            order.extend(2 * r for r in range(pb.read_offsets[t], pb.read_offsets[t + 1]))
        if not order:
            return
        ks = np.asarray(order, np.int64)
        metric = SAMPLE_OFFSET_PER_KEY + (offs[ks + 1] - offs[ks])
        u = self.sample.rng.random(len(ks))
        big = metric >= self.sample.metric_units_per_sample
        hit = big | (u < metric / self.sample.metric_units_per_sample)
        for i in np.nonzero(hit)[0]:
            m = int(metric[i]) if big[i] else self.sample.metric_units_per_sample
            k = pb.key(int(ks[i]))
            if self.sample.add_metric(k, m) == 0:
                self.sample.erase(k)
            self.sample.queue.append((expire, k, -m))

    def poll(self, now: float) -> None:
        self.sample.poll(now)

    def metrics(self) -> int:
        """ResolutionMetricsRequest (:327-330): the sampled total over allKeys."""
        self.metrics_requests += 1
        return self.sample.get_estimate(b"", ALL_KEYS_END)

    def split(self, begin: bytes, end: Optional[bytes], offset: int, front: bool) -> Tuple[bytes, int]:
        """ResolutionSplitRequest (:331-336): (split key, metric on the moved side)."""
        self.split_requests += 1
        e = ALL_KEYS_END if end is None else end
        key = self.sample.split_estimate(begin, e, offset, front)
        used = self.sample.get_estimate(begin, key) if front else self.sample.get_estimate(key, e)
        return key, used


class KeyResolverMap:
    """CoalescedKeyRangeMap<int> over [b"", end): range i = [bounds[i], bounds[i+1]) -> owner."""

    def __init__(self, owner: int = 0):
        self.bounds: List[bytes] = [b""]
        self.owners: List[int] = [owner]

    def ranges(self) -> List[Tuple[bytes, Optional[bytes], int]]:
        ends = self.bounds[1:] + [None]
        return [(b, e, o) for b, e, o in zip(self.bounds, ends, self.owners)]

    def insert(self, begin: bytes, end: Optional[bytes], owner: int) -> None:
        """insert(range, value), then coalesce equal neighbours."""
        pieces = [(begin, owner)]
        for b, e, o in self.ranges():
            if b < begin:  # [b, min(e, begin)) keeps its owner
                pieces.append((b, o))
            if end is not None and (e is None or e > end):  # [max(b, end), e) keeps its owner
                pieces.append((max(b, end), o))
        pieces.sort(key=lambda x: x[0])
        nb, no = [], []
        for b, o in pieces:
            if no and no[-1] == o:
                continue
            nb.append(b)
            no.append(o)
        self.bounds, self.owners = nb, no

    def owner_of(self, key: bytes) -> int:
        return self.owners[bisect.bisect_right(self.bounds, key) - 1]


Move = Tuple[bytes, Optional[bytes], int]  # ResolverMoveRef: (range begin, range end, dest)


def find_range(key_resolver: KeyResolverMap, moved: Sequence[Move], src: int, dest: int) -> Tuple[Tuple[bytes, Optional[bytes]], bool]:
    """findRange (masterserver.actor.cpp:1073-1121): a range of `src` to move (part of) to
    `dest`, and whether to move its front (True) or back.  Prefers growing an existing src|dest
    border, then a new border next to a range not already bordering dest, then any src range."""
    rs = key_resolver.ranges()

    def moved_to_dest(b, e):
        return (b, e, dest) in moved

    if len(rs) == 1:
        b, e, o = rs[0]
        if o != src or moved_to_dest(b, e):
            raise OperationFailed()
        return (b, e), True
    borders = set()
    for i in range(1, len(rs)):
        prev, it = rs[i - 1], rs[i]
        if it[2] == src and prev[2] == dest and not moved_to_dest(it[0], it[1]):
            return (it[0], it[1]), True
        if it[2] == dest and prev[2] == src and not moved_to_dest(prev[0], prev[1]):
            return (prev[0], prev[1]), False
        if it[2] == dest:
            borders.add(prev[2])
        if prev[2] == dest:
            borders.add(it[2])
    for i in range(1, len(rs)):
        prev, it = rs[i - 1], rs[i]
        if it[2] == src and prev[2] not in borders and not moved_to_dest(it[0], it[1]):
            return (it[0], it[1]), True
        if prev[2] == src and it[2] not in borders and not moved_to_dest(prev[0], prev[1]):
            return (prev[0], prev[1]), False
    for b, e, o in rs:
        if o == src and not moved_to_dest(b, e):
            return (b, e), True
    raise OperationFailed()


class ResolutionBalancer:
    """The master's resolutionBalancing loop body (masterserver.actor.cpp:1123-1179), one
    iteration per call.  `metrics(i)` and `split(i, begin, end, offset, front)` are the resolver
    RPCs (ResolverLoad.metrics / .split)."""

    def __init__(self, resolver_count: int, initial: Optional[KeyResolverMap] = None,
                 min_balance_difference: int = MIN_BALANCE_DIFFERENCE):
        self.n = resolver_count
        self.key_resolver = initial if initial is not None else KeyResolverMap(0)
        self.min_balance_difference = min_balance_difference
        self.moves_made = 0

    def step(self, metrics: Callable[[int], int],
             split: Callable[[int, bytes, Optional[bytes], int, bool], Tuple[bytes, int]]) -> List[Move]:
        vals = [metrics(i) for i in range(self.n)]
        total = sum(vals)
        order = sorted((v, i) for i, v in enumerate(vals))  # IndexedSet<pair<int64,int>>
        (vmin, dest), (vmax, src) = order[0], order[-1]
        if vmax - vmin <= self.min_balance_difference:
            return []
        avg = total // self.n
        amount = min(vmax - avg, avg - vmin) // 2
        moved: List[Move] = []
        try:
            while True:
                (b, e), front = find_range(self.key_resolver, moved, src, dest)
                key, used = split(src, b, e, amount, front)
                move = (b, key, dest) if front else (key, e, dest)
                moved.append(move)
                amount -= used
                if (move[0], move[1]) != (b, e) or amount <= 0:
                    break
        except OperationFailed:
            return []  # the reference discards the partial move list (:1173-1176)
        for b, e, d in moved:
            self.key_resolver.insert(b, e, d)
        self.moves_made += len(moved)
        return moved


class BalancedRouting:
    """Single-process driver of the whole loop for G resolvers (tests and the bench): route each
    batch with the proxies' KeyResolvers, feed every resolver's sample with its sub-batch, and
    every MIN_BALANCE_TIME rebalance; the moves take effect at the next batch's version
    (resolverChangesVersion = master version + 1, :1170) and the proxies coalesce their history
    every RESOLVER_COALESCE_TIME (1 s)."""

    def __init__(self, G: int, key_resolvers=None, seed: int = 0, min_balance_difference: int = MIN_BALANCE_DIFFERENCE,
                 balance_time: float = MIN_BALANCE_TIME, key_bytes_per_sample: int = KEY_BYTES_PER_SAMPLE):
        from .sharding import KeyResolvers

        self.G = G
        self.kr = key_resolvers if key_resolvers is not None else KeyResolvers(G)
        init = KeyResolverMap(self.kr.hist[0][-1][1])
        for b, o in self.kr.current_map()[1:]:
            init.insert(b, None, o)
        self.balancer = ResolutionBalancer(G, init, min_balance_difference)
        rng = np.random.default_rng(seed)
        self.loads = [ResolverLoad(G, np.random.default_rng(rng.integers(1 << 62)), key_bytes_per_sample) for _ in range(G)]
        self.balance_time = balance_time
        self.next_balance = None
        self.next_coalesce = None
        self.pending: List[Move] = []
        self.history: List[Tuple[int, List[Move]]] = []

    def route(self, pb: PackedBatch, version: int):
        """Route the batch at commit version `version` (moves decided earlier apply first)."""
        if self.pending:
            self.kr.apply_changes(self.pending, version)
            self.history.append((version, self.pending))
            self.pending = []
        parts = self.kr.route(pb)
        now = version / VERSIONS_PER_SECOND
        for g in range(self.G):
            self.loads[g].poll(now)
            self.loads[g].add_batch(parts[g].batch, now)
        if self.next_balance is None:
            self.next_balance = now + self.balance_time
            self.next_coalesce = now + 1.0
        if now >= self.next_balance:
            self.next_balance = now + self.balance_time
            self.pending = self.balancer.step(lambda i: self.loads[i].metrics(),
                                              lambda i, b, e, off, fr: self.loads[i].split(b, e, off, fr))
        if now >= self.next_coalesce:
            self.next_coalesce = now + 1.0
            self.kr.coalesce(version)
        return parts
