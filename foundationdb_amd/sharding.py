"""Key-range sharding of commit batches across resolvers (one per GPU).

Restates the commit proxy's multi-resolver routing (fdbserver/CommitProxyServer.actor.cpp:118-187)
for a static split (no keyResolvers version history):

* shard g owns [split[g-1], split[g]) (split[-1] = "" and the last shard is unbounded);
* a range [b, e) goes, unclipped, to every shard in intersectingRanges = [rangeContaining(b),
  lower_bound(e)) (fdbrpc/RangeMap.h:126-129).  An empty range at a shard boundary has an empty
  intersection there (the reference ASSERTs, CommitProxyServer.actor.cpp:160); it is routed to
  rangeContaining(b);
* a transaction gets a sub-transaction on a shard only if that shard received one of its ranges
  (getOutTransaction, :107-116); its snapshot and report flag are copied;
* verdicts combine as the element-wise min over the resolvers that saw the transaction
  (determineCommittedTransactions, :764-780); a transaction routed nowhere commits.  On GPUs this
  is an all-reduce MAX of conflict bytes c = 2 - verdict (0 where not routed).
"""
from __future__ import annotations

import bisect
from dataclasses import dataclass
from typing import List, Sequence

import numpy as np

from .packing import PackedBatch


@dataclass
class ShardBatch:
    batch: PackedBatch
    txn_ids: np.ndarray  # global transaction index of each sub-transaction
    read_ids: np.ndarray  # original indexInTx of each routed read (for conflicting-key remap)


class KeyRangeSharding:
    def __init__(self, split_keys: Sequence[bytes]):
        self.splits = [bytes(k) for k in split_keys]
        assert all(a < b for a, b in zip(self.splits, self.splits[1:])), "split keys must ascend"
        assert all(self.splits), "split keys must be non-empty"
        self.G = len(self.splits) + 1
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

    # ---- routing
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
        else:
            g0 = np.array([bisect.bisect_right(self.splits, pb.key(int(k))) for k in kb], np.int64)
            g1 = np.array([bisect.bisect_left(self.splits, pb.key(int(k))) for k in ke], np.int64)
        g1 = np.maximum(g1, g0)
        return g0, g1

    def route(self, pb: PackedBatch) -> List[ShardBatch]:
        T, R, W = pb.n_txn, pb.n_reads, pb.n_writes
        r_idx = np.arange(R)
        w_idx = np.arange(W)
        rg0, rg1 = self._shard_span(pb, 2 * r_idx, 2 * r_idx + 1)
        wg0, wg1 = self._shard_span(pb, 2 * (R + w_idx), 2 * (R + w_idx) + 1)
        r_txn = np.repeat(np.arange(T), np.diff(pb.read_offsets))
        w_txn = np.repeat(np.arange(T), np.diff(pb.write_offsets))
        r_in = r_idx - pb.read_offsets[r_txn]
        out = []
        klen = np.diff(pb.key_offsets)
        for g in range(self.G):
            rm = (rg0 <= g) & (g <= rg1)
            wm = (wg0 <= g) & (g <= wg1)
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

    # ---- combine
    @staticmethod
    def conflict_bytes(T: int, shard: ShardBatch, verdicts: np.ndarray) -> np.ndarray:
        c = np.zeros(T, np.uint8)
        c[shard.txn_ids] = 2 - verdicts.astype(np.uint8)
        return c

    @staticmethod
    def combine(T: int, shards: List[ShardBatch], verdicts: List[np.ndarray]) -> np.ndarray:
        c = np.zeros(T, np.uint8)
        for s, v in zip(shards, verdicts):
            np.maximum(c, KeyRangeSharding.conflict_bytes(T, s, v), out=c)
        return (2 - c).astype(np.uint8)
