"""Host-side packing of commit batches into the flat SoA form the C-ABI takes.

`PackedBatch` mirrors ``fdbcs_packed_batch`` (include/fdb_conflict_set.h): the
fields of ``CommitTransactionRef`` the conflict set reads
(fdbclient/CommitTransaction.h:184-188) flattened into numpy arrays.  Key k of
the batch occupies ``key_bytes[key_offsets[k]:key_offsets[k+1]]``; read range r
uses keys 2r / 2r+1, write range w uses keys 2(R+w) / 2(R+w)+1.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import List, Sequence

import numpy as np


class InvertedRange(ValueError):
    """KeyRangeRef(begin, end) with begin > end throws inverted_range (fdbclient/FDBTypes.h:288-291)."""


@dataclass(frozen=True)
class KeyRange:
    """KeyRangeRef (fdbclient/FDBTypes.h:285-308): half-open [begin, end) of byte strings."""

    begin: bytes
    end: bytes

    def __post_init__(self):
        if bytes(self.begin) > bytes(self.end):
            raise InvertedRange(f"inverted range {self.begin!r} > {self.end!r}")

    def intersects(self, other: "KeyRange") -> bool:  # FDBTypes.h:298
        return self.begin < other.end and other.begin < self.end

    def empty(self) -> bool:
        return self.begin == self.end


def single_key_range(key: bytes) -> KeyRange:
    """singleKeyRange(k) = [k, k + b'\\x00') (fdbclient/FDBTypes.h:499-505)."""
    return KeyRange(key, key + b"\x00")


@dataclass
class CommitTransaction:
    """CommitTransactionRef's conflict-relevant fields (fdbclient/CommitTransaction.h:184-188)."""

    read_conflict_ranges: List[KeyRange] = field(default_factory=list)
    write_conflict_ranges: List[KeyRange] = field(default_factory=list)
    read_snapshot: int = 0
    report_conflicting_keys: bool = False


class _CPackedBatch(ctypes.Structure):
    _fields_ = [
        ("n_txn", ctypes.c_int32),
        ("read_snapshot", ctypes.c_void_p),
        ("report_conflicting_keys", ctypes.c_void_p),
        ("read_offsets", ctypes.c_void_p),
        ("write_offsets", ctypes.c_void_p),
        ("key_bytes", ctypes.c_void_p),
        ("key_offsets", ctypes.c_void_p),
    ]


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data if a.size else 0


@dataclass
class PackedBatch:
    read_snapshot: np.ndarray  # int64[T]
    report: np.ndarray  # uint8[T]
    read_offsets: np.ndarray  # int32[T+1]
    write_offsets: np.ndarray  # int32[T+1]
    key_bytes: np.ndarray  # uint8[...]
    key_offsets: np.ndarray  # int64[2(R+W)+1]

    def __post_init__(self):
        self.read_snapshot = np.ascontiguousarray(self.read_snapshot, dtype=np.int64)
        self.report = np.ascontiguousarray(self.report, dtype=np.uint8)
        self.read_offsets = np.ascontiguousarray(self.read_offsets, dtype=np.int32)
        self.write_offsets = np.ascontiguousarray(self.write_offsets, dtype=np.int32)
        self.key_bytes = np.ascontiguousarray(self.key_bytes, dtype=np.uint8)
        self.key_offsets = np.ascontiguousarray(self.key_offsets, dtype=np.int64)
        T = self.n_txn
        assert self.report.shape == (T,) and self.read_offsets.shape == (T + 1,)
        assert self.write_offsets.shape == (T + 1,)
        assert self.key_offsets.shape == (2 * (self.n_reads + self.n_writes) + 1,)

    @property
    def n_txn(self) -> int:
        return int(self.read_snapshot.shape[0])

    @property
    def n_reads(self) -> int:
        return int(self.read_offsets[-1])

    @property
    def n_writes(self) -> int:
        return int(self.write_offsets[-1])

    @property
    def tail_bytes(self) -> int:
        """Key bytes past the 16-byte prefix over every endpoint (the batch's tail region)."""
        return int(np.maximum(np.diff(self.key_offsets) - 16, 0).sum())

    @property
    def long_endpoints(self) -> int:
        """Endpoints whose key runs past 16 bytes."""
        return int((np.diff(self.key_offsets) > 16).sum())

    def key(self, k: int) -> bytes:
        return self.key_bytes[self.key_offsets[k] : self.key_offsets[k + 1]].tobytes()

    def read_range(self, r: int) -> KeyRange:
        return KeyRange(self.key(2 * r), self.key(2 * r + 1))

    def write_range(self, w: int) -> KeyRange:
        R = self.n_reads
        return KeyRange(self.key(2 * (R + w)), self.key(2 * (R + w) + 1))

    def to_transactions(self) -> List[CommitTransaction]:
        out = []
        for t in range(self.n_txn):
            out.append(
                CommitTransaction(
                    [self.read_range(r) for r in range(self.read_offsets[t], self.read_offsets[t + 1])],
                    [self.write_range(w) for w in range(self.write_offsets[t], self.write_offsets[t + 1])],
                    int(self.read_snapshot[t]),
                    bool(self.report[t]),
                )
            )
        return out

    def slice_txns(self, lo: int, hi: int) -> "PackedBatch":
        """Transactions [lo, hi) as a batch of their own (a commit proxy's share of a global batch)."""
        R, T = self.n_reads, self.n_txn
        assert 0 <= lo <= hi <= T
        r0, r1 = int(self.read_offsets[lo]), int(self.read_offsets[hi])
        w0, w1 = int(self.write_offsets[lo]), int(self.write_offsets[hi])
        ko = self.key_offsets
        # key arena: the reads' key bytes then the writes' (each run contiguous in the source)
        rk = self.key_bytes[ko[2 * r0]: ko[2 * r1]]
        wk = self.key_bytes[ko[2 * (R + w0)]: ko[2 * (R + w1)]]
        rofs = ko[2 * r0: 2 * r1 + 1] - ko[2 * r0]
        wofs = ko[2 * (R + w0): 2 * (R + w1) + 1] - ko[2 * (R + w0)] + len(rk)
        return PackedBatch(self.read_snapshot[lo:hi].copy(), self.report[lo:hi].copy(),
                           (self.read_offsets[lo: hi + 1] - r0).astype(np.int32),
                           (self.write_offsets[lo: hi + 1] - w0).astype(np.int32),
                           np.concatenate([rk, wk]), np.concatenate([rofs, wofs[1:]]).astype(np.int64))

    def c_struct(self) -> _CPackedBatch:
        """ctypes view; the numpy arrays must outlive the returned struct."""
        return _CPackedBatch(
            self.n_txn,
            _ptr(self.read_snapshot),
            _ptr(self.report),
            _ptr(self.read_offsets),
            _ptr(self.write_offsets),
            _ptr(self.key_bytes),
            _ptr(self.key_offsets),
        )

    @staticmethod
    def from_transactions(txns: Sequence[CommitTransaction]) -> "PackedBatch":
        T = len(txns)
        snap = np.array([t.read_snapshot for t in txns], dtype=np.int64)
        rep = np.array([1 if t.report_conflicting_keys else 0 for t in txns], dtype=np.uint8)
        roff = np.zeros(T + 1, dtype=np.int32)
        woff = np.zeros(T + 1, dtype=np.int32)
        for i, t in enumerate(txns):
            roff[i + 1] = roff[i] + len(t.read_conflict_ranges)
            woff[i + 1] = woff[i] + len(t.write_conflict_ranges)
        keys: List[bytes] = []
        for t in txns:
            for rr in t.read_conflict_ranges:
                keys += [bytes(rr.begin), bytes(rr.end)]
        for t in txns:
            for wr in t.write_conflict_ranges:
                keys += [bytes(wr.begin), bytes(wr.end)]
        lens = np.array([len(k) for k in keys], dtype=np.int64)
        koff = np.zeros(len(keys) + 1, dtype=np.int64)
        np.cumsum(lens, out=koff[1:])
        kb = np.frombuffer(b"".join(keys), dtype=np.uint8).copy() if keys else np.zeros(0, np.uint8)
        return PackedBatch(snap, rep, roff, woff, kb, koff)

    @staticmethod
    def from_key_matrix(
        read_snapshot: np.ndarray,
        read_offsets: np.ndarray,
        write_offsets: np.ndarray,
        key_mat: np.ndarray,
        key_len: np.ndarray,
        report: np.ndarray | None = None,
    ) -> "PackedBatch":
        """Vectorised constructor: key k = key_mat[k, :key_len[k]] (keys in packed order)."""
        key_mat = np.ascontiguousarray(key_mat, dtype=np.uint8)
        key_len = np.asarray(key_len, dtype=np.int64)
        n, width = key_mat.shape
        assert key_len.shape == (n,) and (key_len <= width).all()
        mask = np.arange(width)[None, :] < key_len[:, None]
        kb = key_mat[mask]
        koff = np.zeros(n + 1, dtype=np.int64)
        np.cumsum(key_len, out=koff[1:])
        T = len(read_snapshot)
        if report is None:
            report = np.zeros(T, dtype=np.uint8)
        return PackedBatch(read_snapshot, report, read_offsets, write_offsets, kb, koff)


def pack_keys(keys: Sequence[bytes]):
    """(key_bytes, key_offsets) for a list of keys, e.g. a sorted history to bulk-load."""
    lens = np.array([len(k) for k in keys], dtype=np.int64)
    koff = np.zeros(len(keys) + 1, dtype=np.int64)
    np.cumsum(lens, out=koff[1:])
    kb = np.frombuffer(b"".join(keys), dtype=np.uint8).copy() if keys else np.zeros(0, np.uint8)
    return kb, koff


def keys_from_matrix(key_mat: np.ndarray, key_len: np.ndarray):
    """(key_bytes, key_offsets) for keys given as rows of a matrix with lengths."""
    key_mat = np.ascontiguousarray(key_mat, dtype=np.uint8)
    key_len = np.asarray(key_len, dtype=np.int64)
    mask = np.arange(key_mat.shape[1])[None, :] < key_len[:, None]
    koff = np.zeros(len(key_len) + 1, dtype=np.int64)
    np.cumsum(key_len, out=koff[1:])
    return key_mat[mask], koff
