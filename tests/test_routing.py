"""Multi-resolver routing on the device, host side: the proxy share's wire layout
(fdbcs_share_pack, engine.h ShareHeader) and PackedBatch.slice_txns.  No GPU needed: the packing
is host code of the C-ABI library.  The device split itself is checked against the host routing
(sharding.KeyRangeSharding.route, CommitProxyServer.actor.cpp:118-187) in tests/test_gpu_multi.py."""
import numpy as np
import pytest

from foundationdb_amd import build, conflict_set as C
from foundationdb_amd import workloads as W
from foundationdb_amd.packing import PackedBatch


@pytest.fixture(scope="module")
def lib():
    build.build()
    return C.load_library()


def _header(buf):
    h = np.frombuffer(buf[:128].tobytes(), dtype=np.int64)
    T, R = np.frombuffer(buf[:8].tobytes(), dtype=np.int32)
    Wn = int(np.frombuffer(buf[8:12].tobytes(), dtype=np.int32)[0])
    names = ["bytes", "off_keys", "off_snap", "off_roff", "off_woff", "off_report", "off_tail", "tail_bytes", "off_owner"]
    return int(T), int(R), Wn, dict(zip(names, (int(x) for x in h[2:11])))


def _dkey(buf, off, k):
    rec = buf[off + 24 * k: off + 24 * k + 24].tobytes()
    hi, lo = np.frombuffer(rec[:16], dtype=np.uint64)
    ln, tail = np.frombuffer(rec[16:], dtype=np.uint32)
    return int(hi), int(lo), int(ln), int(tail)


@pytest.mark.parametrize("long_keys", [False, True])
def test_share_pack_layout(lib, long_keys):
    rng = np.random.default_rng(3)
    if long_keys:
        pb = W.c4_batch(W.C4Params(txns=64, history=0), rng, 10_000)
    else:
        pb = W.c2_batch(W.C2Params(txns=64, history=0), rng, 10_000)
    buf = C.share_pack(pb)
    T, R, Wn, h = _header(buf)
    assert (T, R, Wn) == (pb.n_txn, pb.n_reads, pb.n_writes)
    assert h["bytes"] == len(buf) and all(h[k] % 64 == 0 for k in h if k.startswith("off_"))
    np.testing.assert_array_equal(np.frombuffer(buf[h["off_snap"]: h["off_snap"] + 8 * T].tobytes(), np.int64),
                                  pb.read_snapshot)
    np.testing.assert_array_equal(np.frombuffer(buf[h["off_roff"]: h["off_roff"] + 4 * (T + 1)].tobytes(), np.int32),
                                  pb.read_offsets)
    np.testing.assert_array_equal(np.frombuffer(buf[h["off_woff"]: h["off_woff"] + 4 * (T + 1)].tobytes(), np.int32),
                                  pb.write_offsets)
    tails = buf[h["off_tail"]:]
    for k in range(2 * (R + Wn)):
        key = pb.key(k)
        hi, lo, ln, tail = _dkey(buf, h["off_keys"], k)
        pre = (key[:16] + bytes(16))[:16]
        assert (hi, lo, ln) == (int.from_bytes(pre[:8], "big"), int.from_bytes(pre[8:], "big"), len(key))
        if len(key) > 16:
            assert tails[tail: tail + len(key) - 16].tobytes() == key[16:]
    assert sum(max(0, len(pb.key(k)) - 16) for k in range(2 * (R + Wn))) == h["tail_bytes"]
    owner = np.frombuffer(buf[h["off_owner"]: h["off_owner"] + 4 * (R + Wn)].tobytes(), np.int32)
    np.testing.assert_array_equal(owner[:R], np.repeat(np.arange(T), np.diff(pb.read_offsets)))
    np.testing.assert_array_equal(owner[R:], np.repeat(np.arange(T), np.diff(pb.write_offsets)))


def test_share_pack_rejects_inverted_range_and_small_buffer(lib):
    pb = PackedBatch(np.array([5], np.int64), np.zeros(1, np.uint8), np.array([0, 1], np.int32),
                     np.array([0, 0], np.int32), np.frombuffer(b"ba", np.uint8).copy(), np.array([0, 1, 2], np.int64))
    with pytest.raises(Exception):
        C.share_pack(pb)
    ok = PackedBatch(np.array([5], np.int64), np.zeros(1, np.uint8), np.array([0, 1], np.int32),
                     np.array([0, 0], np.int32), np.frombuffer(b"ab", np.uint8).copy(), np.array([0, 1, 2], np.int64))
    with pytest.raises(ValueError):
        C.share_pack(ok, np.zeros(64, np.uint8))


def test_slice_txns_concatenates_back():
    rng = np.random.default_rng(4)
    pb = W.c2_batch(W.C2Params(txns=90, history=0), rng, 1000)
    parts = [pb.slice_txns(a, b) for a, b in ((0, 30), (30, 30), (30, 90))]
    assert sum(p.n_txn for p in parts) == 90 and parts[1].n_txn == 0
    keys = [p.key(2 * r + e) for p in parts for r in range(p.n_reads) for e in (0, 1)]
    assert keys == [pb.key(2 * r + e) for r in range(pb.n_reads) for e in (0, 1)]
    wkeys = [p.key(2 * (p.n_reads + w) + e) for p in parts for w in range(p.n_writes) for e in (0, 1)]
    assert wkeys == [pb.key(2 * (pb.n_reads + w) + e) for w in range(pb.n_writes) for e in (0, 1)]
