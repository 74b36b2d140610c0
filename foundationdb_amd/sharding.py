"""Key-range sharding of commit batches across resolvers (one per GPU).

Restates the commit proxy's multi-resolver routing (fdbserver/CommitProxyServer.actor.cpp:118-187):

* ``KeyResolvers`` is ``ProxyCommitData::keyResolvers`` (ProxyCommitData.actor.h:129), a key-range
  map whose value is the ownership history of the range: a deque of (version, resolver), oldest
  first.  It starts as every key owned by resolver 0 at version 0 (:1737-1739) or, for a static
  split, range g owned by resolver g.  ``apply_changes`` appends the master's resolverChanges at
  their version (:622-626); ``coalesce`` drops history no read can need any more (:1284-1297).
* a read range goes, unclipped, to every resolver of every map range it intersects
  (intersectingRanges = [rangeContaining(b), lower_bound(e)), fdbrpc/RangeMap.h:126-129), walking
  each range's history from the newest entry back to the first one older than the transaction's
  read snapshot (:147-164): a read whose snapshot predates a move is checked by the old owner too,
  which holds the writes made before the move.  A write goes only to each range's current owner
  (:166-174).  An empty range at a map boundary has an empty intersection there (the reference
  ASSERTs, :159); it is routed to rangeContaining(b);
* a transaction gets a sub-transaction on a resolver only if that resolver received one of its
  ranges (getOutTransaction, :107-116); its snapshot and report flag are copied (:181-186);
* verdicts combine as the element-wise min over the resolvers that saw the transaction
  (determineCommittedTransactions, :764-780); a transaction routed nowhere commits.  On GPUs this
  is an all-reduce MAX of conflict bytes c = 2 - verdict (0 where not routed);
* conflicting-key reports: for a reporting transaction that did not commit, the proxy concatenates
  each resolver's reported read indices, resolvers in ascending order, mapped back to the
  transaction's own read indices through txReadConflictRangeIndexMap (:144-165, :1243-1261).

``KeyRangeSharding`` is the static split (no version history) with a vectorized fast path for
one-byte split keys; both produce the same ``ShardBatch`` form.
"""
from __future__ import annotations

import bisect
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from .packing import PackedBatch

TransactionConflict, TransactionTooOld, TransactionCommitted = 0, 1, 2  # ConflictSet.h:40-44


@dataclass
class ShardBatch:
    batch: PackedBatch
    txn_ids: np.ndarray  # global transaction index of each sub-transaction
    read_ids: np.ndarray  # original indexInTx of each routed read (txReadConflictRangeIndexMap)


# ---------------------------------------------------------------- vectorized key comparison
def _key_words(pb: PackedBatch, keys: np.ndarray):
    """(hi, lo, lencap, len) of keys `keys`: the 16-byte zero-padded big-endian prefix words and
    min(len, 17) ((prefix, lencap) orders keys unless both exceed 16 bytes)."""
    offs = pb.key_offsets
    start = offs[keys]
    ln = offs[keys + 1] - start
    col = np.arange(16)
    idx = start[:, None] + col[None, :]
    m = col[None, :] < ln[:, None]
    kb = pb.key_bytes
    mat = np.where(m, kb[np.minimum(idx, max(len(kb) - 1, 0))] if len(kb) else 0, 0).astype(np.uint8)
    mat = np.ascontiguousarray(mat)
    w = mat.view(">u8").reshape(-1, 2).astype(np.uint64) if len(keys) else np.zeros((0, 2), np.uint64)
    return w[:, 0], w[:, 1], np.minimum(ln, 17), ln


def _bound_words(b: bytes):
    p = (bytes(b[:16]) + bytes(16))[:16]
    return int.from_bytes(p[:8], "big"), int.from_bytes(p[8:], "big"), min(len(b), 17)


def _cmp_bound(pb: PackedBatch, keys: np.ndarray, words, bound: bytes) -> np.ndarray:
    """sign(key - bound) for each key (int8 array), exact (tails compared where the prefix ties)."""
    hi, lo, lc, ln = words
    bh, bl, blc = _bound_words(bound)
    bh, bl = np.uint64(bh), np.uint64(bl)
    c = np.where(hi < bh, -1, np.where(hi > bh, 1, np.where(lo < bl, -1, np.where(lo > bl, 1,
                 np.where(lc < blc, -1, np.where(lc > blc, 1, 0)))))).astype(np.int8)
    if len(bound) > 16:
        for i in np.nonzero((c == 0) & (ln > 16))[0]:  # both longer than 16 with equal prefixes
            k = pb.key(int(keys[i]))
            c[i] = -1 if k < bound else (1 if k > bound else 0)
    return c


def _range_spans(pb: PackedBatch, kb: np.ndarray, ke: np.ndarray, bounds: Sequence[bytes]):
    """(m0, m1) per range over a map with range starts `bounds` (bounds[0] = b""):
    m0 = rangeContaining(begin), m1 = last map range whose start < end (>= m0)."""
    n = len(kb)
    m0 = np.zeros(n, np.int64)
    m1 = np.zeros(n, np.int64)
    if len(bounds) > 1 and n:
        wb, we = _key_words(pb, kb), _key_words(pb, ke)
        for b in bounds[1:]:
            m0 += _cmp_bound(pb, kb, wb, b) >= 0
            m1 += _cmp_bound(pb, ke, we, b) > 0
    return m0, np.maximum(m1, m0)


def _route_masks(pb: PackedBatch, G: int, rmask: np.ndarray, wmask: np.ndarray) -> List[ShardBatch]:
    """Split a batch by per-range resolver bitmasks (bit g: range goes to resolver g)."""
    T, R, W = pb.n_txn, pb.n_reads, pb.n_writes
    r_idx = np.arange(R)
    w_idx = np.arange(W)
    r_txn = np.repeat(np.arange(T), np.diff(pb.read_offsets))
    w_txn = np.repeat(np.arange(T), np.diff(pb.write_offsets))
    r_in = r_idx - pb.read_offsets[r_txn]
    klen = np.diff(pb.key_offsets)
    out = []
    for g in range(G):
        bit = np.int64(1) << np.int64(g)
        rm = (rmask & bit) != 0
        wm = (wmask & bit) != 0
        has = np.zeros(T, bool)
        has[r_txn[rm]] = True
        has[w_txn[wm]] = True
        txn_ids = np.nonzero(has)[0]
        remap = -np.ones(T, np.int64)
        remap[txn_ids] = np.arange(len(txn_ids))
        rsel = r_idx[rm]
        wsel = w_idx[wm]
        nr = np.bincount(remap[r_txn[rsel]], minlength=len(txn_ids)) if len(rsel) else np.zeros(len(txn_ids), int)
        nw = np.bincount(remap[w_txn[wsel]], minlength=len(txn_ids)) if len(wsel) else np.zeros(len(txn_ids), int)
        roff = np.zeros(len(txn_ids) + 1, np.int32)
        woff = np.zeros(len(txn_ids) + 1, np.int32)
        np.cumsum(nr, out=roff[1:])
        np.cumsum(nw, out=woff[1:])
        keys = np.concatenate(
            [np.stack([2 * rsel, 2 * rsel + 1], 1).reshape(-1), np.stack([2 * (R + wsel), 2 * (R + wsel) + 1], 1).reshape(-1)]
        ).astype(np.int64)
        lens = klen[keys]
        koff = np.zeros(len(keys) + 1, np.int64)
        np.cumsum(lens, out=koff[1:])
        if len(keys):
            starts = pb.key_offsets[keys]
            idx = np.repeat(starts - koff[:-1], lens) + np.arange(int(koff[-1]))
            kbytes = pb.key_bytes[idx]
        else:
            kbytes = np.zeros(0, np.uint8)
        sub = PackedBatch(pb.read_snapshot[txn_ids], pb.report[txn_ids], roff, woff, kbytes, koff)
        out.append(ShardBatch(sub, txn_ids, r_in[rsel]))
    return out


def _span_mask(g0: np.ndarray, g1: np.ndarray) -> np.ndarray:
    """Bitmask of resolvers g0..g1 (inclusive) per range."""
    one = np.int64(1)
    return ((one << (g1 + 1).astype(np.int64)) - one) ^ ((one << g0.astype(np.int64)) - one)


# ---------------------------------------------------------------- combine (proxy side)
def conflict_bytes(T: int, shard: ShardBatch, verdicts: np.ndarray) -> np.ndarray:
    c = np.zeros(T, np.uint8)
    c[shard.txn_ids] = 2 - np.asarray(verdicts).astype(np.uint8)
    return c


def combine(T: int, shards: List[ShardBatch], verdicts: List[np.ndarray]) -> np.ndarray:
    """determineCommittedTransactions (:764-780): min over the resolvers that saw each txn."""
    c = np.zeros(T, np.uint8)
    for s, v in zip(shards, verdicts):
        np.maximum(c, conflict_bytes(T, s, v), out=c)
    return (2 - c).astype(np.uint8)


def combine_conflicting_keys(pb: PackedBatch, shards: List[ShardBatch], maps: List[Dict[int, Sequence[int]]],
                             committed: np.ndarray) -> Dict[int, List[int]]:
    """The proxy's conflictingKRIndices (CommitProxyServer.actor.cpp:1243-1261): for each reporting
    transaction that neither committed nor came back TooOld, the concatenation over the resolvers
    it was routed to (ascending resolver index, transactionResolverMap :181-187) of that
    resolver's conflictingKeyRangeMap entry for its sub-transaction (created empty if absent, as
    std::map::operator[] does), each local read index mapped to the transaction's own index."""
    out: Dict[int, List[int]] = {}
    locs = []
    for s in shards:
        remap = -np.ones(pb.n_txn, np.int64)
        remap[s.txn_ids] = np.arange(len(s.txn_ids))
        locs.append(remap)
    for t in np.nonzero((np.asarray(committed) == TransactionConflict) & (pb.report != 0))[0]:
        t = int(t)
        idx: List[int] = []
        for g, s in enumerate(shards):
            lt = int(locs[g][t])
            if lt < 0:
                continue
            r0 = int(s.batch.read_offsets[lt])
            for i in maps[g].get(lt, ()):
                idx.append(int(s.read_ids[r0 + int(i)]))
        out[t] = idx
    return out


# ---------------------------------------------------------------- static split
class KeyRangeSharding:
    """A static split: shard g owns [split[g-1], split[g]) (split[-1] = "", last shard unbounded),
    i.e. keyResolvers with one history entry per range."""

    def __init__(self, split_keys: Sequence[bytes]):
        self.splits = [bytes(k) for k in split_keys]
        assert all(a < b for a, b in zip(self.splits, self.splits[1:])), "split keys must ascend"
        assert all(self.splits), "split keys must be non-empty"
        self.G = len(self.splits) + 1
        assert self.G <= 62
        self._byte_splits = None
        if all(len(k) == 1 for k in self.splits):
            self._byte_splits = np.array([k[0] for k in self.splits], dtype=np.int64)

    @staticmethod
    def uniform(G: int) -> "KeyRangeSharding":
        """G shards of equal measure over the first key byte."""
        return KeyRangeSharding([bytes([(g * 256) // G]) for g in range(1, G)])

    def shard_bounds(self, g: int):
        lo = self.splits[g - 1] if g > 0 else b""
        hi = self.splits[g] if g < self.G - 1 else None
        return lo, hi

    def _first_bytes(self, pb: PackedBatch, keys: np.ndarray) -> np.ndarray:
        offs = pb.key_offsets
        lens = offs[keys + 1] - offs[keys]
        fb = np.full(len(keys), -1, np.int64)  # empty key sorts before every split
        nz = lens > 0
        fb[nz] = pb.key_bytes[offs[keys[nz]]]
        return fb

    def _shard_span(self, pb: PackedBatch, kb: np.ndarray, ke: np.ndarray):
        """(g0, g1) per range: rangeContaining(begin) .. last shard whose start < end."""
        if self.G == 1:
            z = np.zeros(len(kb), np.int64)
            return z, z
        if self._byte_splits is not None:
            fb = self._first_bytes(pb, kb)
            fe = self._first_bytes(pb, ke)
            g0 = np.searchsorted(self._byte_splits, fb, side="right")
            # shards with start < end: start s (1 byte) < e  <=>  s < e[0] or (s == e[0] and len(e) > 1)
            elen = pb.key_offsets[ke + 1] - pb.key_offsets[ke]
            g1 = np.searchsorted(self._byte_splits, fe, side="left")  # starts strictly below e[0]
            eq = (g1 < len(self._byte_splits)) & (self._byte_splits[np.minimum(g1, len(self._byte_splits) - 1)] == fe)
            g1 = g1 + (eq & (elen > 1)).astype(np.int64)
            return g0, np.maximum(g1, g0)
        return _range_spans(pb, kb, ke, [b""] + self.splits)

    def route(self, pb: PackedBatch) -> List[ShardBatch]:
        R, W = pb.n_reads, pb.n_writes
        r_idx, w_idx = np.arange(R), np.arange(W)
        rg0, rg1 = self._shard_span(pb, 2 * r_idx, 2 * r_idx + 1)
        wg0, wg1 = self._shard_span(pb, 2 * (R + w_idx), 2 * (R + w_idx) + 1)
        return _route_masks(pb, self.G, _span_mask(rg0, rg1), _span_mask(wg0, wg1))

    conflict_bytes = staticmethod(conflict_bytes)
    combine = staticmethod(combine)


# ---------------------------------------------------------------- ownership history
class KeyResolvers:
    """keyResolvers: map ranges [bounds[i], bounds[i+1]) (the last unbounded), each with its
    ownership history [(version, resolver), ...] oldest first."""

    def __init__(self, G: int, splits: Sequence[bytes] = (), owners: Optional[Sequence[int]] = None):
        self.G = G
        assert G <= 62
        self.bounds: List[bytes] = [b""] + [bytes(k) for k in splits]
        assert all(a < b for a, b in zip(self.bounds, self.bounds[1:]))
        owners = list(owners) if owners is not None else (list(range(len(self.bounds))) if splits else [0])
        assert len(owners) == len(self.bounds) and all(0 <= o < G for o in owners)
        self.hist: List[List[Tuple[int, int]]] = [[(0, o)] for o in owners]  # :1737-1739

    @staticmethod
    def from_sharding(sh: KeyRangeSharding) -> "KeyResolvers":
        return KeyResolvers(sh.G, sh.splits)

    # -- map edits (KeyRangeMap::modify splits at the range ends and copies values)
    def _split_at(self, k: bytes) -> int:
        i = bisect.bisect_right(self.bounds, k) - 1
        if self.bounds[i] != k:
            self.bounds.insert(i + 1, k)
            self.hist.insert(i + 1, list(self.hist[i]))
            i += 1
        return i

    def apply_changes(self, moves: Sequence[Tuple[bytes, Optional[bytes], int]], version: int) -> None:
        """versionReply.resolverChanges at resolverChangesVersion (CommitProxyServer.actor.cpp:622-626):
        every map range inside each moved [begin, end) gets (version, dest) appended."""
        for begin, end, dest in moves:
            i0 = self._split_at(bytes(begin))
            i1 = self._split_at(bytes(end)) if end is not None else len(self.bounds)
            for i in range(i0, i1):
                self.hist[i].append((version, dest))

    def coalesce(self, prev_version: int, life_versions: int = 5_000_000) -> None:
        """:1284-1297: drop history entries whose successor is older than oldestVersion, zero an
        older first entry, then merge adjacent ranges with equal histories."""
        oldest = prev_version - life_versions
        for h in self.hist:
            while len(h) > 1 and h[1][0] < oldest:
                h.pop(0)
            if h and h[0][0] < oldest:
                h[0] = (0, h[0][1])
        nb, nh = [self.bounds[0]], [self.hist[0]]
        for b, h in zip(self.bounds[1:], self.hist[1:]):
            if h == nh[-1]:
                continue
            nb.append(b)
            nh.append(h)
        self.bounds, self.hist = nb, nh

    def owner_of(self, key: bytes) -> int:
        return self.hist[bisect.bisect_right(self.bounds, bytes(key)) - 1][-1][1]

    def current_map(self) -> List[Tuple[bytes, int]]:
        """(begin, current owner) per map range."""
        return [(b, h[-1][1]) for b, h in zip(self.bounds, self.hist)]

    # -- routing
    def masks(self, pb: PackedBatch) -> Tuple[np.ndarray, np.ndarray]:
        R, W = pb.n_reads, pb.n_writes
        r_idx, w_idx = np.arange(R), np.arange(W)
        rm0, rm1 = _range_spans(pb, 2 * r_idx, 2 * r_idx + 1, self.bounds)
        wm0, wm1 = _range_spans(pb, 2 * (R + w_idx), 2 * (R + w_idx) + 1, self.bounds)
        snap = np.repeat(pb.read_snapshot, np.diff(pb.read_offsets))
        rmask = np.zeros(R, np.int64)
        wmask = np.zeros(W, np.int64)
        for m, h in enumerate(self.hist):
            rin = (rm0 <= m) & (m <= rm1)
            for i, (_, res) in enumerate(h):
                # :152-157: newest first; entry i is visited iff every newer entry is >= snapshot
                incl = rin if i == len(h) - 1 else rin & (h[i + 1][0] >= snap)
                rmask |= np.where(incl, np.int64(1) << np.int64(res), np.int64(0))
            win = (wm0 <= m) & (m <= wm1)
            wmask |= np.where(win, np.int64(1) << np.int64(h[-1][1]), np.int64(0))  # :169-170
        return rmask, wmask

    def route(self, pb: PackedBatch) -> List[ShardBatch]:
        rmask, wmask = self.masks(pb)
        return _route_masks(pb, self.G, rmask, wmask)

    conflict_bytes = staticmethod(conflict_bytes)
    combine = staticmethod(combine)
