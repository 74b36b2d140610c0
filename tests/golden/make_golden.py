"""Generate the committed golden fixtures under tests/golden/.

1. ordering_kats.json — the four known-answer asserts of operatorLessThanTest
   (fdbserver/SkipList.cpp:973-1005), transcribed as data.
2. kat_scenarios.json — hand-derived multi-batch scenarios.  Every expected verdict is
   derived from reading SkipList.cpp (line cited per case), NOT computed by the oracle;
   tests check both the oracle and the HIP engine against them.
3. random_batches.npz — oracle-generated regression vectors (small random batches over a
   tiny alphabet) so GPU parity is checked against frozen outputs, not only a live oracle.

Run:  python tests/golden/make_golden.py   (needs oracle/liboracle.so: `make -C oracle`)
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

C, TOO_OLD, OK = 0, 1, 2


def h(b: bytes) -> str:
    return b.hex()


def ordering_kats():
    # (keyA, beginA, writeA) < (keyB, beginB, writeB) must hold; SkipList.cpp:975-1003
    return [
        {"name": "longer strings after shorter", "a": [h(b"hello"), False, True], "b": [h(b"hello\x00"), False, False],
         "line": "SkipList.cpp:975-980"},
        {"name": "read end before write end", "a": [h(b"hello"), False, False], "b": [h(b"hello"), False, True],
         "line": "SkipList.cpp:983-988"},
        {"name": "write end before read begin", "a": [h(b"hello"), False, True], "b": [h(b"hello"), True, False],
         "line": "SkipList.cpp:991-996"},
        {"name": "write end before write begin", "a": [h(b"hello"), False, True], "b": [h(b"hello"), True, True],
         "line": "SkipList.cpp:999-1004"},
    ]


def txn(reads=(), writes=(), snap=0, report=False):
    return {"reads": [[h(a), h(b)] for a, b in reads], "writes": [[h(a), h(b)] for a, b in writes],
            "snapshot": snap, "report": report}


def scenarios():
    S = []
    S.append({
        "name": "write at version == snapshot does not conflict",
        "why": "CheckMax compares maxVersion > version strictly (SkipList.cpp:664,671,690)",
        "batches": [
            {"now": 10, "new_oldest": 0, "txns": [txn(writes=[(b"a", b"b")])], "expect": [OK]},
            {"now": 20, "new_oldest": 0, "txns": [txn(reads=[(b"a", b"b")], snap=10),
                                                   txn(reads=[(b"a", b"b")], snap=9)], "expect": [OK, C]},
        ]})
    S.append({
        "name": "touching ranges do not conflict with history",
        "why": "segment ending at b is excluded (SkipList.cpp:690-697); segment starting at e excluded",
        "batches": [
            {"now": 10, "new_oldest": 0, "txns": [txn(writes=[(b"b", b"c")])], "expect": [OK]},
            {"now": 20, "new_oldest": 0, "txns": [txn(reads=[(b"a", b"b")], snap=5),
                                                   txn(reads=[(b"c", b"d")], snap=5),
                                                   txn(reads=[(b"a", b"b\x00")], snap=5),
                                                   txn(reads=[(b"b\x00", b"b\x01")], snap=5)],
             "expect": [OK, OK, C, C]},
        ]})
    S.append({
        "name": "intra-batch: later reader of an earlier committed write aborts; touching does not",
        "why": "MiniConflictSet over point indices with class order (SkipList.cpp:812-834, 89-91)",
        "batches": [
            {"now": 10, "new_oldest": 0, "txns": [
                txn(writes=[(b"k", b"k\x00")], snap=0),
                txn(reads=[(b"k", b"k\x00")], snap=0),
                txn(reads=[(b"k\x00", b"z")], snap=0),
                txn(reads=[(b"a", b"k")], snap=0),
            ], "expect": [OK, C, OK, OK]},
        ]})
    S.append({
        "name": "intra-batch: only earlier transactions' writes count",
        "why": "writes join the MiniConflictSet after the transaction is decided (SkipList.cpp:831-832)",
        "batches": [
            {"now": 10, "new_oldest": 0, "txns": [
                txn(reads=[(b"x", b"x\x00")], writes=[(b"y", b"y\x00")]),
                txn(reads=[(b"y", b"y\x00")], writes=[(b"x", b"x\x00")]),
            ], "expect": [OK, C]},
        ]})
    S.append({
        "name": "intra-batch chain: an aborted writer does not kill later readers",
        "why": "only non-conflicting transactions set their writes (SkipList.cpp:830-832)",
        "batches": [
            {"now": 10, "new_oldest": 0, "txns": [
                txn(writes=[(b"a", b"a\x00")]),
                txn(reads=[(b"a", b"a\x00")], writes=[(b"b", b"b\x00")]),
                txn(reads=[(b"b", b"b\x00")], writes=[(b"c", b"c\x00")]),
                txn(reads=[(b"c", b"c\x00")]),
            ], "expect": [OK, C, OK, C]},
        ]})
    S.append({
        "name": "too old: snapshot below oldestVersion with reads; write-only is never too old",
        "why": "tooOld = read_snapshot < oldestVersion && reads (SkipList.cpp:770); oldest raised after verdicts (:880-882)",
        "batches": [
            {"now": 100, "new_oldest": 50, "txns": [txn(reads=[(b"q", b"r")], snap=40)], "expect": [OK]},
            {"now": 110, "new_oldest": 50, "txns": [txn(reads=[(b"q", b"r")], snap=40),
                                                     txn(writes=[(b"q", b"r")], snap=40),
                                                     txn(reads=[(b"s", b"t")], snap=50),
                                                     txn(reads=[(b"q", b"q\x00")], snap=50)],
             "expect": [TOO_OLD, OK, OK, C]},
        ]})
    S.append({
        "name": "degenerate empty read [b,b) checks the segment of the greatest boundary < b",
        "why": "start/end fingers never diverge; level-0 finger is the predecessor (SkipList.cpp:650-666)",
        "batches": [
            {"now": 10, "new_oldest": 0, "txns": [txn(writes=[(b"k", b"m")])], "expect": [OK]},
            {"now": 20, "new_oldest": 0, "txns": [txn(reads=[(b"k", b"k")], snap=5),
                                                   txn(reads=[(b"m", b"m")], snap=5),
                                                   txn(reads=[(b"l", b"l")], snap=5),
                                                   txn(reads=[(b"m", b"m")], snap=10)],
             "expect": [OK, C, C, OK]},
        ]})
    S.append({
        "name": "empty key and header version",
        "why": "header node holds key '' and the initial version, never rewritten (SkipList.cpp:398-404, 591-610)",
        "batches": [
            {"now": 10, "new_oldest": 0, "txns": [txn(writes=[(b"", b"a")])], "expect": [OK]},
            {"now": 20, "new_oldest": 0, "txns": [txn(reads=[(b"", b"")], snap=5),
                                                   txn(reads=[(b"", b"\x00")], snap=5),
                                                   txn(reads=[(b"a", b"b")], snap=5)],
             "expect": [OK, C, OK]},
        ]})
    S.append({
        "name": "keys equal up to zero padding are distinct",
        "why": "compare(): shorter key first (SkipList.cpp:53-60); end boundary keeps old version (:419)",
        "batches": [
            {"now": 10, "new_oldest": 0, "txns": [txn(writes=[(b"ab", b"ab\x00")])], "expect": [OK]},
            {"now": 20, "new_oldest": 0, "txns": [txn(reads=[(b"ab\x00", b"ab\x00\x00")], snap=5),
                                                   txn(reads=[(b"a", b"ab\x00")], snap=5),
                                                   txn(reads=[(b"ab\x00\x00", b"ac")], snap=5)],
             "expect": [OK, C, OK]},
        ]})
    S.append({
        "name": "long keys compare on their tails",
        "why": "byte-lexicographic order over the whole key (flow/Arena.h:692-697)",
        "batches": [
            {"now": 10, "new_oldest": 0, "txns": [txn(writes=[(b"P" * 20 + b"m", b"P" * 20 + b"n")])], "expect": [OK]},
            {"now": 20, "new_oldest": 0, "txns": [txn(reads=[(b"P" * 20 + b"a", b"P" * 20 + b"m")], snap=5),
                                                   txn(reads=[(b"P" * 20 + b"a", b"P" * 20 + b"m\x00")], snap=5),
                                                   txn(reads=[(b"P" * 20 + b"n", b"P" * 20 + b"z")], snap=5),
                                                   txn(reads=[(b"P" * 20 + b"mz" * 10, b"P" * 20 + b"mz" * 11)], snap=5)],
             "expect": [OK, C, OK, C]},
        ]})
    S.append({
        "name": "clearConflictSet resets every version but keeps oldestVersion",
        "why": "SkipList(v).swap(versionHistory) (SkipList.cpp:742-744)",
        "clear_before": 1, "clear_version": 100,
        "batches": [
            {"now": 50, "new_oldest": 30, "txns": [txn(writes=[(b"a", b"b")])], "expect": [OK]},
            {"now": 150, "new_oldest": 30, "txns": [txn(reads=[(b"x", b"y")], snap=99),
                                                     txn(reads=[(b"x", b"y")], snap=100),
                                                     txn(reads=[(b"x", b"y")], snap=20)],
             "expect": [C, OK, TOO_OLD]},
        ]})
    S.append({
        "name": "conflicting keys: every conflicting read for history, first for intra-batch",
        "why": "CheckMax::conflict pushes indexInTx (SkipList.cpp:641-645); intra pushes the first (:821-828)",
        "batches": [
            {"now": 10, "new_oldest": 0, "txns": [txn(writes=[(b"a", b"b"), (b"c", b"d")])], "expect": [OK]},
            {"now": 20, "new_oldest": 0, "txns": [
                txn(reads=[(b"a", b"a\x00"), (b"x", b"y"), (b"c", b"c\x00")], snap=5, report=True),
                txn(writes=[(b"m", b"n"), (b"p", b"q")], snap=15),
                txn(reads=[(b"e", b"f"), (b"p", b"p\x00"), (b"m", b"m\x00")], snap=15, report=True),
                txn(reads=[(b"e", b"f")], snap=15, report=True),
            ], "expect": [C, OK, C, OK], "conflicting": {"0": [0, 2], "2": [1]}},
        ]})
    S.append({
        "name": "union of committed writes: adjacent and overlapping writes merge, aborted writes do not",
        "why": "combineWriteConflictRanges counts only non-conflicting writers (SkipList.cpp:926-939)",
        "batches": [
            {"now": 10, "new_oldest": 0, "txns": [
                txn(writes=[(b"a", b"c")]),
                txn(writes=[(b"c", b"e"), (b"b", b"d")]),
                txn(reads=[(b"b", b"b\x00")], writes=[(b"x", b"z")]),
            ], "expect": [OK, OK, C]},
            {"now": 20, "new_oldest": 0, "txns": [txn(reads=[(b"d", b"e")], snap=9),
                                                   txn(reads=[(b"e", b"f")], snap=9),
                                                   txn(reads=[(b"y", b"y\x00")], snap=9)],
             "expect": [C, OK, OK]},
        ]})
    return S


def random_fixtures(path):
    from foundationdb_amd import workloads as W
    from oracle.oracle import OracleConflictSet

    rng = np.random.default_rng(20261015)
    out = {}
    seqs = 12
    for s in range(seqs):
        cs = OracleConflictSet()
        now = 10
        for b in range(5):
            pb = W.random_small_batch(rng, int(rng.integers(1, 48)), alphabet=3 + s % 3, max_len=3, now=now,
                                      staleness=12)
            no = now - int(rng.integers(0, 10))
            v, conf = cs.detect(pb, now, no)
            p = f"s{s}b{b}_"
            out[p + "snap"] = pb.read_snapshot
            out[p + "report"] = pb.report
            out[p + "roff"] = pb.read_offsets
            out[p + "woff"] = pb.write_offsets
            out[p + "kb"] = pb.key_bytes
            out[p + "ko"] = pb.key_offsets
            out[p + "now"] = np.array([now, no], np.int64)
            out[p + "verdict"] = v
            ct = sorted(conf)
            out[p + "conf_txn"] = np.array(ct, np.int32)
            out[p + "conf_off"] = np.cumsum([0] + [len(conf[t]) for t in ct]).astype(np.int32)
            out[p + "conf_idx"] = np.array([i for t in ct for i in conf[t]], np.int32)
            now += int(rng.integers(1, 6))
    out["meta"] = np.array([seqs, 5], np.int32)
    np.savez_compressed(path, **out)


def main():
    with open(os.path.join(HERE, "ordering_kats.json"), "w") as f:
        json.dump(ordering_kats(), f, indent=1)
    with open(os.path.join(HERE, "kat_scenarios.json"), "w") as f:
        json.dump(scenarios(), f, indent=1)
    random_fixtures(os.path.join(HERE, "random_batches.npz"))
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
