"""Synthetic commit-batch generators for the configurations BASELINE.json names.

All generators are deterministic in their seed and emit ``PackedBatch`` objects
(flat SoA, the C-ABI input).  They restate the reference's own generators:

* ``DeterministicRandom`` — flow/DeterministicRandom.cpp:22-53: a mt19937 seeded
  with the seed, ``gen64 = (r() << 32) ^ r()`` with one step of look-ahead, and
  ``randomInt(a, b) = a + gen64() % (b - a)``.  numpy's legacy ``RandomState``
  seeding is ``std::mt19937(seed)``'s init_genrand, so raw words match.
* ``ZipfGenerator`` — the YCSB Zipfian of fdbclient/zipf.c:27-110.
* ``tuple_pack`` — Tuple encoding of (bytes, str, int) (fdbclient/Tuple.cpp:72-117).

Configurations (SURVEY.md §8 shorthand):
  C1  skipListTest (fdbserver/SkipList.cpp:1008-1077): 2500 txns/batch, 1 read + 1 write,
      keys setK(i) = 12 x '.' + big-endian int32 (SkipList.cpp:942-953), k in [0, 2e7),
      range [k, k + 1 + U[0,10]], snapshot v, now v + 50, newOldest v.
  C2  5000 txns/batch, 5 reads + 2 writes, 16-byte uniform keys, 5M-boundary history.
  C3  C2 shape, keys from YCSB Zipf(theta=0.99) over 1M Mako-style keys.
  C4  tuple-encoded keys (subspace, str, int) <= 100 B, wide Tuple.range() reads.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Iterator, List, Tuple

import numpy as np

from .packing import PackedBatch, keys_from_matrix


class DeterministicRandom:
    """flow/DeterministicRandom.cpp:22-53 (mt19937, gen64 with look-ahead)."""

    def __init__(self, seed: int):
        assert seed != 0  # DeterministicRandom.cpp:31 — mersenne twister needs x0 > 0
        self._bg = np.random.RandomState(seed)._bit_generator
        self._buf = np.zeros(0, np.uint64)
        self._pos = 0

    def _raw(self, n: int) -> np.ndarray:
        return self._bg.random_raw(n).astype(np.uint64)

    def gen64(self, n: int) -> np.ndarray:
        r = self._raw(2 * n)
        return (r[0::2] << np.uint64(32)) ^ r[1::2]

    def random_int(self, lo: int, hi: int, n: int) -> np.ndarray:
        """n draws of randomInt(lo, hi) for 0 <= lo < hi (DeterministicRandom.cpp:34-48)."""
        assert 0 <= lo < hi
        return (self.gen64(n) % np.uint64(hi - lo)).astype(np.int64) + lo


# --------------------------------------------------------------------------- C1
def setk(vals: np.ndarray) -> np.ndarray:
    """setK (SkipList.cpp:942-953): 12 x '.' then the int32 big-endian -> (n, 16) uint8."""
    vals = np.asarray(vals, dtype=np.int64)
    out = np.full((len(vals), 16), ord("."), dtype=np.uint8)
    be = vals.astype(">u4").view(np.uint8).reshape(-1, 4)
    out[:, 12:] = be
    return out


def c1_batches(n_batches: int = 500, seed: int = 1, data_per_batch: int = 5000) -> Iterator[Tuple[PackedBatch, int, int]]:
    """skipListTest data (SkipList.cpp:1023-1077): yields (batch, now, newOldest)."""
    rng = DeterministicRandom(seed)
    T = data_per_batch // 2
    for v in range(n_batches):
        g = rng.gen64(2 * data_per_batch)
        key = (g[0::2] % np.uint64(20000000)).astype(np.int64)
        key2 = key + 1 + (g[1::2] % np.uint64(10)).astype(np.int64)
        # ranges j = 0..4999: txn t reads data[2t], writes data[2t+1] (readCount = writeCount = 1)
        kb = setk(key)
        ke = setk(key2)
        R = T
        mat = np.zeros((4 * T, 16), np.uint8)
        mat[0 : 2 * R : 2] = kb[0::2]
        mat[1 : 2 * R : 2] = ke[0::2]
        mat[2 * R :: 2] = kb[1::2]
        mat[2 * R + 1 :: 2] = ke[1::2]
        lens = np.full(4 * T, 16, np.int64)
        offs = np.arange(T + 1, dtype=np.int32)
        pb = PackedBatch.from_key_matrix(np.full(T, v, np.int64), offs, offs, mat, lens)
        yield pb, v + 50, v


# --------------------------------------------------------------------------- C2
def _add_be128(keys: np.ndarray, delta: np.ndarray) -> np.ndarray:
    """keys (n,16) uint8 as big-endian 128-bit integers + small delta, saturating at 2^128-1."""
    hi = keys[:, :8].copy().view(">u8").reshape(-1).astype(np.uint64)
    lo = keys[:, 8:].copy().view(">u8").reshape(-1).astype(np.uint64)
    d = np.asarray(delta, dtype=np.uint64)
    nlo = lo + d
    carry = (nlo < lo).astype(np.uint64)
    nhi = hi + carry
    over = (nhi < hi) | ((hi == np.uint64(0xFFFFFFFFFFFFFFFF)) & (carry > 0))
    nlo[over] = np.uint64(0xFFFFFFFFFFFFFFFF)
    nhi[over] = np.uint64(0xFFFFFFFFFFFFFFFF)
    out = np.empty_like(keys)
    out[:, :8] = nhi.astype(">u8").view(np.uint8).reshape(-1, 8)
    out[:, 8:] = nlo.astype(">u8").view(np.uint8).reshape(-1, 8)
    return out


@dataclass
class C2Params:
    txns: int = 5000
    reads: int = 5
    writes: int = 2
    history: int = 5_000_000
    version_step: int = 1000  # versions between batches
    window: int = 5_000_000  # MAX_WRITE_TRANSACTION_LIFE_VERSIONS (fdbserver/Knobs.cpp:41)
    staleness: int = 100_000  # snapshot = now - U[0, staleness)
    # share of transactions whose snapshot sits at the MVCC window's edge, now - window +
    # U[-2 step, 2 step): about half of them are TooOld (SkipList.cpp:770) once the oldest version
    # follows now - window (Resolver.actor.cpp:194)
    too_old_frac: float = 0.0
    range_write_frac: float = 0.5  # fraction of writes that are short ranges (rest single-key)


def c2_history(p: C2Params, seed: int, start_version: int):
    """5M random 16-B boundaries, versions uniform over the MVCC window below start_version.
    Returns (key_bytes, key_offsets, versions) sorted by key."""
    rng = np.random.default_rng(seed + 1000003)
    keys = rng.integers(0, 256, size=(p.history, 16), dtype=np.uint8)
    hi = keys[:, :8].copy().view(">u8").reshape(-1)
    lo = keys[:, 8:].copy().view(">u8").reshape(-1)
    keys = keys[np.lexsort((lo, hi))]
    # drop duplicates (vanishingly rare)
    if len(keys) > 1:
        keep = np.ones(len(keys), bool)
        keep[1:] = (keys[1:] != keys[:-1]).any(axis=1)
        keys = keys[keep]
    vers = rng.integers(max(0, start_version - p.window), start_version, size=len(keys), dtype=np.int64)
    kb = keys.reshape(-1)
    ko = np.arange(len(keys) + 1, dtype=np.int64) * 16
    return kb, ko, vers


def window_edge_snapshots(p, rng: np.random.Generator, now: int, snap: np.ndarray) -> np.ndarray:
    """p.too_old_frac of the snapshots moved to the window's edge (no draws when it is 0, so the
    default workloads' streams are unchanged)."""
    if p.too_old_frac <= 0:
        return snap
    T = len(snap)
    edge = rng.random(T) < p.too_old_frac
    snap = snap.copy()
    snap[edge] = now - p.window + rng.integers(-2 * p.version_step, 2 * p.version_step, size=int(edge.sum()))
    return snap


def c2_batch(p: C2Params, rng: np.random.Generator, now: int) -> PackedBatch:
    T, nr, nw = p.txns, p.reads, p.writes
    R, W = T * nr, T * nw
    rb = rng.integers(0, 256, size=(R, 16), dtype=np.uint8)
    re = _add_be128(rb, rng.integers(1, 17, size=R))
    wb = rng.integers(0, 256, size=(W, 16), dtype=np.uint8)
    is_range = rng.random(W) < p.range_write_frac
    we = np.zeros((W, 17), np.uint8)
    we[:, :16] = wb  # single key: [k, k + b"\0")
    wr = _add_be128(wb, rng.integers(1, 17, size=W))
    we[is_range, :16] = wr[is_range]
    wlen = np.where(is_range, 16, 17)
    mat = np.zeros((2 * (R + W), 17), np.uint8)
    mat[0 : 2 * R : 2, :16] = rb
    mat[1 : 2 * R : 2, :16] = re
    mat[2 * R :: 2, :16] = wb
    mat[2 * R + 1 :: 2] = we
    lens = np.full(2 * (R + W), 16, np.int64)
    lens[2 * R + 1 :: 2] = wlen
    snap = window_edge_snapshots(p, rng, now, now - rng.integers(0, p.staleness, size=T))
    return PackedBatch.from_key_matrix(
        snap, np.arange(T + 1, dtype=np.int32) * nr, np.arange(T + 1, dtype=np.int32) * nw, mat, lens
    )


# --------------------------------------------------------------------------- C3
class ZipfGenerator:
    """YCSB zipfian (fdbclient/zipf.c:27-110), vectorised; items in [0, n)."""

    def __init__(self, n: int, theta: float = 0.99):
        self.n, self.theta = n, theta
        i = np.arange(1, n + 1, dtype=np.float64)
        self.zetan = float(np.sum(1.0 / i**theta))
        self.zeta2 = 1.0 + 1.0 / 2**theta
        self.alpha = 1.0 / (1.0 - theta)
        self.eta = (1 - (2.0 / n) ** (1 - theta)) / (1 - self.zeta2 / self.zetan)

    def sample(self, rng: np.random.Generator, size: int) -> np.ndarray:
        u = rng.random(size)
        uz = u * self.zetan
        out = (self.n * np.power(self.eta * u - self.eta + 1, self.alpha)).astype(np.int64)
        out[uz < 1.0 + 0.5**self.theta] = 1
        out[uz < 1.0] = 0
        return np.minimum(out, self.n - 1)


def mako_keys(idx: np.ndarray, width: int = 16) -> np.ndarray:
    """Mako-style key: 'mako' + zero-padded decimal index, padded with 'x' (workloads/Mako.actor.cpp:252-256)."""
    out = np.full((len(idx), width), ord("x"), np.uint8)
    out[:, :4] = np.frombuffer(b"mako", np.uint8)
    digits = 8
    v = np.asarray(idx, np.int64).copy()
    for d in range(digits - 1, -1, -1):
        out[:, 4 + d] = ord("0") + (v % 10)
        v //= 10
    return out


def c3_batch(p: C2Params, rng: np.random.Generator, now: int, zipf: ZipfGenerator) -> PackedBatch:
    T, nr, nw = p.txns, p.reads, p.writes
    R, W = T * nr, T * nw
    rk = mako_keys(zipf.sample(rng, R))
    wk = mako_keys(zipf.sample(rng, W))
    mat = np.zeros((2 * (R + W), 17), np.uint8)
    mat[0 : 2 * R : 2, :16] = rk
    mat[1 : 2 * R : 2, :16] = rk
    mat[2 * R :: 2, :16] = wk
    mat[2 * R + 1 :: 2, :16] = wk
    lens = np.full(2 * (R + W), 16, np.int64)
    lens[1::2] = 17  # every range is singleKeyRange(k) = [k, k\0)
    snap = window_edge_snapshots(p, rng, now, now - rng.integers(0, p.staleness, size=T))
    return PackedBatch.from_key_matrix(
        snap, np.arange(T + 1, dtype=np.int32) * nr, np.arange(T + 1, dtype=np.int32) * nw, mat, lens
    )


# --------------------------------------------------------------------------- C4
def tuple_pack(subspace: bytes, s: str, i: int) -> bytes:
    """Tuple encoding (fdbclient/Tuple.cpp:72-117): 0x01 bytes\\0 (0x00 -> 0x00 0xFF), 0x02 str\\0,
    int: 0x14 for zero, 0x14+n / 0x14-n with n big-endian magnitude bytes (one's complement if negative)."""
    out = bytearray(subspace)

    def enc_bytes(code, b):
        out.append(code)
        out.extend(b.replace(b"\x00", b"\x00\xff"))
        out.append(0)

    enc_bytes(0x02, s.encode())
    if i == 0:
        out.append(0x14)
    else:
        n = (abs(i).bit_length() + 7) // 8
        mag = abs(i).to_bytes(n, "big")
        if i > 0:
            out.append(0x14 + n)
            out.extend(mag)
        else:
            out.append(0x14 - n)
            out.extend(bytes(255 - x for x in mag))
    return bytes(out)


def tuple_range(prefix: bytes) -> Tuple[bytes, bytes]:
    """Tuple::range() = [p\\x00, p\\xff) (fdbclient/Tuple.cpp:240-255)."""
    return prefix + b"\x00", prefix + b"\xff"


@dataclass
class C4Params:
    """Tuple-key workload (BASELINE.json configs[3]).

    Keys are ``subspace + pack((str user, int item))``: a 2-byte directory-layer style subspace
    (the tuple encoding of a small int, as the directory layer's allocator hands out), the user
    string ``"user" + 8 digits + filler`` (filler 0..max_filler bytes of 'x', fixed per user, so
    keys run up to ~100 B) and a positive int item.  The first 16 bytes distinguish users, so
    every comparison between keys of one user goes to the tail bytes (SURVEY §7 hard parts).
    Each transaction reads one whole user (``Tuple.range()`` of the user prefix, a wide read)
    plus ``point_reads`` single keys, and writes ``writes`` single keys."""

    txns: int = 5000
    point_reads: int = 4
    writes: int = 2
    users: int = 1_000_000
    items: int = 50_000
    history: int = 50_000_000  # boundaries (two per prefilled key: k and k + b"\0")
    max_filler: int = 70
    version_step: int = 1000
    window: int = 5_000_000
    staleness: int = 100_000
    too_old_frac: float = 0.0  # as C2Params.too_old_frac
    subspace: bytes = b"\x15\x2a"  # tuple-encoded int 42

    @property
    def reads(self) -> int:
        return 1 + self.point_reads


C4_WIDTH = 112  # row width of the key matrices (longest key is < 100 bytes)


def c4_filler_len(p: C4Params, user: np.ndarray) -> np.ndarray:
    """Per-user filler length: a fixed hash of the user id (Knuth multiplicative)."""
    h = (np.asarray(user, np.uint64) * np.uint64(2654435761)) & np.uint64(0xFFFFFFFF)
    return (h % np.uint64(p.max_filler + 1)).astype(np.int64)


def c4_user_string(p: C4Params, user: int) -> str:
    return f"user{user:08d}" + "x" * int(c4_filler_len(p, np.array([user]))[0])


def c4_user_split(p: C4Params, user: int) -> bytes:
    """A key below every key of `user` and above every key of smaller users (shard split point)."""
    return p.subspace + b"\x02" + f"user{user:08d}".encode()


def c4_keys(p: C4Params, user: np.ndarray, item: np.ndarray, kind: np.ndarray):
    """Key matrix (n, C4_WIDTH) and lengths, one row per (user, item, kind):
    0 = pack(user, item);  1 = pack(user, item) + b"\\0" (keyAfter);
    2 = Tuple.range(user).begin = prefix(user) + b"\\0";  3 = Tuple.range(user).end = prefix(user) + b"\\xff".
    Items must lie in [1, 65536) (one or two magnitude bytes)."""
    user = np.asarray(user, np.int64)
    item = np.asarray(item, np.int64)
    kind = np.asarray(kind, np.int64)
    n = len(user)
    sub = np.frombuffer(p.subspace, np.uint8)
    S = len(sub)
    mat = np.zeros((n, C4_WIDTH), np.uint8)
    mat[:, :S] = sub
    mat[:, S] = 0x02  # string type code (Tuple.cpp:72-117)
    mat[:, S + 1 : S + 5] = np.frombuffer(b"user", np.uint8)
    v = user.copy()
    for d in range(7, -1, -1):
        mat[:, S + 5 + d] = ord("0") + (v % 10)
        v //= 10
    f0 = S + 13  # filler start
    L = c4_filler_len(p, user)
    cols = np.arange(C4_WIDTH)[None, :]
    mat[(cols >= f0) & (cols < (f0 + L)[:, None])] = ord("x")
    rows = np.arange(n)
    pe = f0 + L  # string terminator; prefix(user) = bytes [0, pe]
    mat[rows, pe] = 0x00
    nb = np.where(item >= 256, 2, 1)
    length = np.empty(n, np.int64)
    wide = kind >= 2
    mat[rows[wide], pe[wide] + 1] = np.where(kind[wide] == 2, 0x00, 0xFF)
    length[wide] = pe[wide] + 2
    pt = ~wide
    r, q, it, nbp = rows[pt], pe[pt], item[pt], nb[pt]
    mat[r, q + 1] = 0x14 + nbp  # positive int code (Tuple.cpp:72-117)
    two = nbp == 2
    mat[r[two], q[two] + 2] = (it[two] >> 8).astype(np.uint8)
    mat[r[two], q[two] + 3] = (it[two] & 0xFF).astype(np.uint8)
    mat[r[~two], q[~two] + 2] = it[~two].astype(np.uint8)
    klen = q + 2 + nbp
    suf = kind[pt] == 1
    mat[r[suf], klen[suf]] = 0x00  # keyAfter(k) = k + b"\0"
    length[pt] = klen + suf
    return mat, length


def c4_history(p: C4Params, seed: int, start_version: int, users: Tuple[int, int] | None = None,
               chunk: int = 2_000_000):
    """Prefilled history of about p.history boundaries: random distinct (user, item) keys (users
    in [users[0], users[1]) when given), each a boundary k and its keyAfter k + b"\\0", with versions
    spread over the window (the step function single-key writes leave).  Sorted by construction:
    tuple order is (user, item) because the user digits are fixed width and positive ints encode
    order-preservingly (Tuple.cpp:72-117).  Returns (key_bytes, key_offsets, versions).

    Same bytes as c4_keys row by row, built from a per-user prefix table (the user prefix is the
    long shared part of every key) so the 50M-boundary window generates in seconds."""
    rng = np.random.default_rng(seed + 4000037)
    u0, u1 = users if users is not None else (0, p.users)
    span = p.items - 1
    code = np.unique(rng.integers(u0 * span, u1 * span, size=p.history // 2, dtype=np.int64))
    user = code // span
    item = code % span + 1
    n = 2 * len(code)
    ulo = int(user.min()) if len(user) else 0
    uids = np.arange(ulo, int(user.max()) + 1 if len(user) else 0)
    # prefix(user) = subspace 0x02 "user" 8 digits filler 0x00 (c4_keys without the item)
    S = len(p.subspace)
    f0 = S + 13
    PW = f0 + p.max_filler + 1
    ptab = np.zeros((len(uids), PW), np.uint8)
    ptab[:, :S] = np.frombuffer(p.subspace, np.uint8)
    ptab[:, S] = 0x02
    ptab[:, S + 1 : S + 5] = np.frombuffer(b"user", np.uint8)
    v = uids.copy()
    for d in range(7, -1, -1):
        ptab[:, S + 5 + d] = ord("0") + (v % 10)
        v //= 10
    Lf = c4_filler_len(p, uids)
    cols = np.arange(PW)[None, :]
    ptab[(cols >= f0) & (cols < (f0 + Lf)[:, None])] = ord("x")
    plen = f0 + Lf + 1
    lens = np.empty(n, np.int64)
    nb = np.where(item >= 256, 2, 1)
    parts = []
    wcols = np.arange(PW + 4)[None, :]
    for a in range(0, len(code), chunk):
        ur = np.repeat(user[a : a + chunk] - ulo, 2)
        m2 = len(ur)
        tab = np.zeros((m2, PW + 4), np.uint8)
        tab[:, :PW] = ptab[ur]
        pl = plen[ur]
        rows = np.arange(m2)
        nbr = np.repeat(nb[a : a + chunk], 2)
        itr = np.repeat(item[a : a + chunk], 2)
        tab[rows, pl] = (0x14 + nbr).astype(np.uint8)  # positive int code (Tuple.cpp:72-117)
        two = nbr == 2
        tab[rows[two], pl[two] + 1] = (itr[two] >> 8).astype(np.uint8)
        tab[rows[two], pl[two] + 2] = (itr[two] & 0xFF).astype(np.uint8)
        tab[rows[~two], pl[~two] + 1] = itr[~two].astype(np.uint8)
        ln = pl + 1 + nbr + np.tile(np.array([0, 1], np.int64), m2 // 2)  # keyAfter: trailing 0x00
        lens[2 * a : 2 * a + m2] = ln
        parts.append(tab[wcols < ln[:, None]])
    kb = np.concatenate(parts) if parts else np.zeros(0, np.uint8)
    ko = np.zeros(n + 1, np.int64)
    np.cumsum(lens, out=ko[1:])
    vers = rng.integers(max(0, start_version - p.window), start_version, size=n, dtype=np.int64)
    return kb, ko, vers


def c4_batch(p: C4Params, rng: np.random.Generator, now: int) -> PackedBatch:
    """One C4 batch: per transaction one wide read of a user, p.point_reads point reads and
    p.writes point writes, the point ranges single-key [k, k + b"\\0") (FDBTypes.h:499-505)."""
    T, nr, nw = p.txns, p.reads, p.writes
    R, W = T * nr, T * nw
    user = rng.integers(0, p.users, size=R + W)
    item = rng.integers(1, p.items, size=R + W)
    wide = np.zeros(R + W, bool)
    wide[0:R:nr] = True  # each transaction's first read covers the whole user
    kind = np.tile(np.array([0, 1], np.int64), R + W) + 2 * np.repeat(wide, 2)
    mat, lens = c4_keys(p, np.repeat(user, 2), np.repeat(item, 2), kind)
    snap = window_edge_snapshots(p, rng, now, now - rng.integers(0, p.staleness, size=T))
    return PackedBatch.from_key_matrix(
        snap, np.arange(T + 1, dtype=np.int32) * nr, np.arange(T + 1, dtype=np.int32) * nw, mat, lens
    )


# --------------------------------------------------------------------------- tests
def random_small_batch(
    rng: np.random.Generator,
    txns: int,
    max_reads: int = 3,
    max_writes: int = 3,
    alphabet: int = 4,
    max_len: int = 3,
    now: int = 100,
    staleness: int = 20,
    report_frac: float = 0.5,
) -> PackedBatch:
    """Short keys over a tiny alphabet so ranges collide, touch, nest and repeat; includes
    empty keys, empty ranges and equal keys of different lengths (SURVEY §7 hard parts)."""
    from .packing import CommitTransaction, KeyRange

    def key():
        n = int(rng.integers(0, max_len + 1))
        return bytes(int(x) for x in rng.integers(0, alphabet, size=n))

    out: List[CommitTransaction] = []
    for _ in range(txns):
        def rng_range():
            a, b = key(), key()
            if rng.random() < 0.1:
                b = a  # empty range
            if a > b:
                a, b = b, a
            return KeyRange(a, b)

        t = CommitTransaction(
            [rng_range() for _ in range(int(rng.integers(0, max_reads + 1)))],
            [rng_range() for _ in range(int(rng.integers(0, max_writes + 1)))],
            int(now - rng.integers(0, staleness)),
            bool(rng.random() < report_frac),
        )
        out.append(t)
    return PackedBatch.from_transactions(out)
