"""Client-side conflict-range production.

Restates how NativeAPI's ``Transaction`` turns reads and writes into the read/write conflict
ranges of the ``CommitTransactionRef`` the resolver checks (fdbclient/NativeAPI.actor.cpp), so the
engine sees the inputs a real client produces and the guarantees it may rely on:

* ``get`` adds ``singleKeyRange(key)`` unless it is a snapshot read; a key longer than the key-size
  limit cannot exist and reads nothing (:2951-2966);
* ``get_range`` / ``get_key`` add the range they actually observed once the result is known
  (extraConflictRanges, :3097-3165; getRangeFinished :2597-2629), computed here by
  ``get_range_conflict_range`` / ``get_key_conflict_range`` from the result;
* ``set`` / ``atomic_op`` add ``singleKeyRange(key)`` (not for SetVersionstampedKey), ``clear`` adds
  the cleared range; oversized keys are rejected (set, atomicOp) or clamped / ignored (clear)
  (:3208-3293);
* ``add_read_conflict_range`` / ``add_write_conflict_range`` clamp keys to limit + 1 bytes (a
  longer key cannot exist) and drop ranges that became empty (:3177-3197, :3294-3316): **the
  engine never receives an empty range from NativeAPI**;
* ``commit_request`` applies commitMutations (:3795-3850): a transaction without writes or
  mutations does not commit at all; ready extra conflict ranges with begin < end are appended as
  reads; unless CAUSAL_WRITE_RISKY, a transaction whose writes do not intersect its reads becomes
  self-conflicting (a random ``\\xff/SC/<uid>`` key read and written, :3199-3206) — and the
  ``intersects`` test sorts both range lists by begin in place (:3434-3446), which fixes the read
  order the conflicting-key indices refer to; with checkWrites (1 %), writes are also read.

A small multi-version key-value store stands in for the storage servers so reads have results.
"""
from __future__ import annotations

import bisect
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from .packing import CommitTransaction, KeyRange

KEY_SIZE_LIMIT = 10_000  # fdbclient/Knobs.cpp:74
SYSTEM_KEY_SIZE_LIMIT = 30_000  # :75
VALUE_SIZE_LIMIT = 100_000  # :76
TRANSACTION_SIZE_LIMIT = 10_000_000  # :73
ALL_KEYS_BEGIN = b""
ALL_KEYS_END = b"\xff\xff"
SYSTEM_PREFIX = b"\xff"

# MutationRef::Type values used here (fdbclient/CommitTransaction.h)
SET_VALUE, CLEAR_RANGE, ADD_VALUE, SET_VERSIONSTAMPED_KEY, SET_VERSIONSTAMPED_VALUE = 0, 1, 2, 14, 15


class FDBError(Exception):
    def __init__(self, name: str):
        super().__init__(name)
        self.name = name


def key_limit(key: bytes) -> int:
    return SYSTEM_KEY_SIZE_LIMIT if key.startswith(SYSTEM_PREFIX) else KEY_SIZE_LIMIT


def clamp_key(key: bytes) -> bytes:
    """A key over the limit cannot exist: keep limit + 1 bytes, an equivalent bound (:3185-3188)."""
    lim = key_limit(key)
    return key[: lim + 1] if len(key) > lim else key


def key_after(key: bytes) -> bytes:
    """keyAfter (fdbclient/FDBTypes.h:481-490): key + \\0, except \\xff\\xff stays."""
    return key if key == ALL_KEYS_END else key + b"\x00"


def single_key_range(key: bytes) -> KeyRange:
    """singleKeyRange (FDBTypes.h:500-508): [key, key + \\0) (always appends)."""
    return KeyRange(key, key + b"\x00")


@dataclass(frozen=True)
class KeySelector:
    """KeySelectorRef (FDBTypes.h:539-602): the last key < key (<= if or_equal), then `offset`
    items forward.  The key is clamped like setKey (:565-572)."""

    key: bytes
    or_equal: bool
    offset: int

    def __post_init__(self):
        k = bytes(self.key)
        lim = SYSTEM_KEY_SIZE_LIMIT if k.startswith(b"\xff") else KEY_SIZE_LIMIT
        object.__setattr__(self, "key", k[: lim + 1] if len(k) > lim else k)

    def remove_or_equal(self) -> "KeySelector":
        return KeySelector(key_after(self.key), False, self.offset) if self.or_equal else self

    def is_first_greater_or_equal(self) -> bool:
        return not self.or_equal and self.offset == 1

    def is_first_greater_than(self) -> bool:
        return self.or_equal and self.offset == 1


def first_greater_or_equal(k: bytes) -> KeySelector:
    return KeySelector(k, False, 1)


def first_greater_than(k: bytes) -> KeySelector:
    return KeySelector(k, True, 1)


def last_less_than(k: bytes) -> KeySelector:
    return KeySelector(k, False, 0)


def last_less_or_equal(k: bytes) -> KeySelector:
    return KeySelector(k, True, 0)


# ------------------------------------------------------------------ conflict ranges of results
def get_range_conflict_range(begin: KeySelector, end: KeySelector, result_keys: Sequence[bytes], more: bool,
                             read_to_begin: bool, read_through_end: bool, reverse: bool) -> Tuple[bytes, bytes]:
    """getRangeFinished's conflict range (NativeAPI.actor.cpp:2597-2629); `result_keys` in the
    order returned (descending when reverse)."""
    n = len(result_keys)
    if read_to_begin:
        rb = ALL_KEYS_BEGIN
    elif ((not reverse or not more or begin.offset > 1) and begin.offset > 0) or n == 0:
        rb = begin.key
    else:
        rb = result_keys[-1] if reverse else result_keys[0]
    if end.offset > begin.offset and end.key < rb:
        rb = end.key
    if read_through_end:
        re_ = ALL_KEYS_END
    elif ((reverse or not more or end.offset <= 0) and end.offset <= 1) or n == 0:
        re_ = end.key
    else:
        re_ = key_after(result_keys[0] if reverse else result_keys[-1])
    if begin.offset < end.offset and begin.key > re_:
        re_ = begin.key
    return rb, re_


def get_key_conflict_range(sel: KeySelector, resolved: bytes) -> Tuple[bytes, bytes]:
    """getKeyAndConflictRange (NativeAPI.actor.cpp:3097-3111)."""
    if sel.offset <= 0:
        return resolved, key_after(sel.key) if sel.or_equal else sel.key
    return (key_after(sel.key) if sel.or_equal else sel.key), key_after(resolved)


# ------------------------------------------------------------------ a storage stand-in
class VersionedStore:
    """Committed key -> value history; reads see the latest value at or below a read version."""

    def __init__(self):
        self.keys: List[bytes] = []
        self.hist: Dict[bytes, List[Tuple[int, Optional[bytes]]]] = {}
        self.version = 0

    def read(self, key: bytes, version: int) -> Optional[bytes]:
        h = self.hist.get(key)
        if not h:
            return None
        i = bisect.bisect_right([v for v, _ in h], version) - 1
        return h[i][1] if i >= 0 else None

    def live_keys(self, version: int) -> List[bytes]:
        return [k for k in self.keys if self.read(k, version) is not None]

    def resolve(self, sel: KeySelector, version: int) -> bytes:
        """Key a selector resolves to (allKeys.begin / allKeys.end past the ends)."""
        ks = self.live_keys(version)
        base = (bisect.bisect_right(ks, sel.key) if sel.or_equal else bisect.bisect_left(ks, sel.key)) - 1
        i = base + sel.offset
        if i < 0:
            return ALL_KEYS_BEGIN
        if i >= len(ks):
            return ALL_KEYS_END
        return ks[i]

    def apply(self, version: int, mutations: Sequence[Tuple[int, bytes, bytes]]) -> None:
        assert version > self.version
        self.version = version
        for typ, p1, p2 in mutations:
            if typ == SET_VALUE:
                self._put(p1, version, p2)
            elif typ == ADD_VALUE:
                old = self.read(p1, version) or b""
                a = int.from_bytes(old, "little") if old else 0
                w = max(len(old), len(p2))
                self._put(p1, version, ((a + int.from_bytes(p2, "little")) % (1 << (8 * w))).to_bytes(w, "little"))
            elif typ == CLEAR_RANGE:
                for k in [k for k in self.keys if p1 <= k < p2]:
                    self._put(k, version, None)

    def _put(self, key: bytes, version: int, value: Optional[bytes]) -> None:
        if key not in self.hist:
            bisect.insort(self.keys, key)
            self.hist[key] = []
        self.hist[key].append((version, value))


# ------------------------------------------------------------------ the transaction
@dataclass
class TransactionOptions:
    causal_write_risky: bool = False
    read_only: bool = False
    check_writes_enabled: bool = False
    report_conflicting_keys: bool = False
    size_limit: int = TRANSACTION_SIZE_LIMIT


class Transaction:
    """NativeAPI Transaction's conflict bookkeeping over a VersionedStore at `read_version`.
    `rng` supplies randomUniqueID() and the checkWrites roll."""

    def __init__(self, store: VersionedStore, read_version: int, rng: Optional[np.random.Generator] = None,
                 options: Optional[TransactionOptions] = None):
        self.store = store
        self.read_version = read_version
        self.rng = rng if rng is not None else np.random.default_rng()
        self.options = options or TransactionOptions()
        self.read_conflict_ranges: List[KeyRange] = []
        self.write_conflict_ranges: List[KeyRange] = []
        self.mutations: List[Tuple[int, bytes, bytes]] = []
        self.extra_conflict_ranges: List[Tuple[bytes, bytes]] = []  # ready futures of range reads

    # ---- reads
    def get(self, key: bytes, snapshot: bool = False) -> Optional[bytes]:
        if len(key) > key_limit(key):
            return None
        if not snapshot:
            self.read_conflict_ranges.append(single_key_range(key))
        return self.store.read(key, self.read_version)

    def get_key(self, sel: KeySelector, snapshot: bool = False) -> bytes:
        k = self.store.resolve(sel, self.read_version)
        if not snapshot:
            self.extra_conflict_ranges.append(get_key_conflict_range(sel, k))
        return k

    def get_range(self, begin: KeySelector, end: KeySelector, limit: int = 0, snapshot: bool = False,
                  reverse: bool = False) -> List[Tuple[bytes, bytes]]:
        """Transaction::getRange (:3124-3165) over getRangeFallback's read model (:2533-2566):
        resolve both selectors, read the exact range with a row limit (0 = none)."""
        b, e = begin.remove_or_equal(), end.remove_or_equal()
        if b.offset >= e.offset and b.key >= e.key:
            return []
        read_to_begin = b.key == ALL_KEYS_BEGIN and b.offset < 1  # :2651-2653
        bk, ek = self.store.resolve(b, self.read_version), self.store.resolve(e, self.read_version)
        rows: List[Tuple[bytes, bytes]] = []
        more = False
        if bk < ek:
            ks = [k for k in self.store.live_keys(self.read_version) if bk <= k < ek]
            if reverse:
                ks = ks[::-1]
            if limit and len(ks) > limit:
                ks, more = ks[:limit], True
            rows = [(k, self.store.read(k, self.read_version)) for k in ks]
            read_to_begin |= bk == ALL_KEYS_BEGIN and (not reverse or not more)  # :2562-2565
        read_through_end = bk < ek and ek == ALL_KEYS_END and (reverse or not more)
        if not snapshot:
            self.extra_conflict_ranges.append(
                get_range_conflict_range(b, e, [k for k, _ in rows], more, read_to_begin, read_through_end, reverse))
        return rows

    # ---- writes
    def set(self, key: bytes, value: bytes, add_conflict_range: bool = True) -> None:
        if len(key) > key_limit(key):
            raise FDBError("key_too_large")
        if len(value) > VALUE_SIZE_LIMIT:
            raise FDBError("value_too_large")
        r = single_key_range(key)
        self.mutations.append((SET_VALUE, key, value))
        if add_conflict_range:
            self.write_conflict_ranges.append(r)

    def atomic_op(self, key: bytes, operand: bytes, op: int, add_conflict_range: bool = True) -> None:
        if len(key) > key_limit(key):
            raise FDBError("key_too_large")
        if len(operand) > VALUE_SIZE_LIMIT:
            raise FDBError("value_too_large")
        self.mutations.append((op, key, operand))
        if add_conflict_range and op != SET_VERSIONSTAMPED_KEY:
            self.write_conflict_ranges.append(single_key_range(key))

    def clear_range(self, begin: bytes, end: bytes, add_conflict_range: bool = True) -> None:
        r = KeyRange(clamp_key(begin), clamp_key(end))
        if r.empty():
            return
        self.mutations.append((CLEAR_RANGE, r.begin, r.end))
        if add_conflict_range:
            self.write_conflict_ranges.append(r)

    def clear(self, key: bytes, add_conflict_range: bool = True) -> None:
        if len(key) > key_limit(key):
            return
        self.mutations.append((CLEAR_RANGE, key, key + b"\x00"))
        if add_conflict_range:
            self.write_conflict_ranges.append(KeyRange(key, key + b"\x00"))

    # ---- explicit conflict ranges
    def add_read_conflict_range(self, begin: bytes, end: bytes) -> None:
        assert begin < end, "addReadConflictRange of an empty range"  # :3178
        r = KeyRange(clamp_key(begin), clamp_key(end))
        if not r.empty():
            self.read_conflict_ranges.append(r)

    def add_write_conflict_range(self, begin: bytes, end: bytes) -> None:
        assert begin < end, "addWriteConflictRange of an empty range"  # :3295
        r = KeyRange(clamp_key(begin), clamp_key(end))
        if not r.empty():
            self.write_conflict_ranges.append(r)

    def make_self_conflicting(self) -> None:
        """:3199-3206: a fresh \\xff/SC/<randomUniqueID> key, read and written."""
        uid = self.rng.integers(0, 1 << 63, size=2, dtype=np.int64).astype("<u8").tobytes()
        r = single_key_range(b"\xff/SC/" + uid)
        self.read_conflict_ranges.append(r)
        self.write_conflict_ranges.append(r)

    # ---- commit
    def size(self) -> int:
        """getSize (:4405-4411): mutations + both conflict range lists."""
        m = sum(len(a) + len(b) for _, a, b in self.mutations)
        return m + sum(len(r.begin) + len(r.end) for r in self.read_conflict_ranges + self.write_conflict_ranges)

    def commit_request(self) -> Optional[CommitTransaction]:
        """commitMutations (:3795-3850): the CommitTransactionRef sent to the proxy, or None for a
        transaction with nothing to commit."""
        if not self.write_conflict_ranges and not self.mutations:
            return None  # read-only: no commit version (:3797-3804)
        if self.options.read_only:
            raise FDBError("transaction_read_only")
        if self.size() > self.options.size_limit:
            raise FDBError("transaction_too_large")
        checking_writes = self.options.check_writes_enabled and self.rng.random() < 0.01
        for b, e in self.extra_conflict_ranges:  # :3839-3842
            if b < e:
                self.read_conflict_ranges.append(KeyRange(b, e))
        if not self.options.causal_write_risky and intersects(self.write_conflict_ranges, self.read_conflict_ranges) is None:
            self.make_self_conflicting()
        if checking_writes:
            self.read_conflict_ranges.extend(self.write_conflict_ranges)
        return CommitTransaction(list(self.read_conflict_ranges), list(self.write_conflict_ranges), self.read_version,
                                 self.options.report_conflicting_keys)


def intersects(lhs: List[KeyRange], rhs: List[KeyRange]) -> Optional[KeyRange]:
    """intersects (NativeAPI.actor.cpp:3434-3450): sorts both lists by begin IN PLACE (the
    VectorRefs alias the transaction's arrays), then a merge walk; returns a range inside the
    intersection, or None.  (std::sort leaves equal begins in an unspecified order; this sort is
    stable.)"""
    if lhs and rhs:
        lhs.sort(key=lambda r: r.begin)
        rhs.sort(key=lambda r: r.begin)
        l = r = 0
        while l < len(lhs) and r < len(rhs):
            if lhs[l].end <= rhs[r].begin:
                l += 1
            elif rhs[r].end <= lhs[l].begin:
                r += 1
            else:
                return KeyRange(max(lhs[l].begin, rhs[r].begin), min(lhs[l].end, rhs[r].end))
    return None
