"""Randomized parity stress of the HIP engine against the skip-list restatement (run on the GPU box).

Each round draws a key alphabet (arbitrary bytes, decimal digits, a sparse byte set, a tiny
alphabet), a shared prefix, key lengths around 16 and 24 bytes, a loaded history, engine knobs
read at set creation (directory slot budget, split check, stream layout, submitting threads),
compaction and GC cadence, and a sequence of batches whose snapshots straddle the oldest version; verdicts and
conflicting-read reports must match oracle/skiplist_baseline.cpp batch by batch.

    python3 scripts/stress_parity.py [seconds] [first_seed]

Exit status 1 and the failing seed on the first mismatch."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from foundationdb_amd import conflict_set as C  # noqa: E402
from foundationdb_amd.packing import CommitTransaction, KeyRange, PackedBatch  # noqa: E402
from oracle import oracle  # noqa: E402
from tests.helpers import EngineDriver  # noqa: E402

KNOBS = {
    "FDBCS_DIR_BITS": ["0", "0", "16", "18"],
    "FDBCS_SPLIT_CHECK": ["2", "1"],
    "FDBCS_SERIAL": ["0", "0", "0", "1"],
    "FDBCS_SKIP_EDGES": ["1", "0"],
    "FDBCS_SUBMIT_THREAD": ["1", "1", "0"],
}


def one(seed):
    rng = np.random.default_rng(seed)
    for k, vals in KNOBS.items():
        os.environ[k] = vals[int(rng.integers(0, len(vals)))]
    kind = ["bytes", "digits", "sparse", "tiny"][int(rng.integers(0, 4))]
    prefix = bytes(rng.integers(0, 256, size=int(rng.integers(0, 20))).astype(np.uint8))
    top = int(rng.choice([8, 16, 30]))

    def suffix(n, hist):
        if kind == "bytes":
            return bytes(rng.integers(0, 256, size=n).astype(np.uint8))
        if kind == "digits":
            return bytes(rng.integers(0x30, 0x3a, size=n).astype(np.uint8))
        if kind == "tiny":
            return bytes(rng.integers(0, 3, size=n).astype(np.uint8))
        if hist:  # sparse: even values in the history, any value in the batches
            return bytes((2 * rng.integers(0x10, 0x40, size=n)).astype(np.uint8))
        return bytes(rng.integers(0x10, 0x91, size=n).astype(np.uint8))

    def key(hist=False):
        k = prefix + suffix(int(rng.integers(0, top)), hist)
        if rng.random() < 0.05:  # outside the shared prefix
            k = bytes(rng.integers(0, 256, size=int(rng.integers(0, 6))).astype(np.uint8))
        return k

    n_hist = int(rng.integers(0, 40000))
    hist = sorted({key(True) for _ in range(n_hist)})
    kb = np.frombuffer(b"".join(hist), np.uint8) if hist else np.zeros(0, np.uint8)
    ko = np.zeros(len(hist) + 1, np.int64)
    if hist:
        np.cumsum([len(k) for k in hist], out=ko[1:])
    vers = rng.integers(0, 1000, size=len(hist)).astype(np.int64)
    e = EngineDriver(C, gc_interval=int(rng.integers(0, 4)), delta_limit=int(rng.choice([0, 2000, 20000])))
    o = oracle.SkipListBaseline()
    e.load_history(kb, ko, vers)
    o.load_history(kb, ko, vers)
    now, oldest = 1000, 0
    for i in range(int(rng.integers(3, 10))):
        now += int(rng.integers(1, 200))
        txns = []
        for _ in range(int(rng.integers(1, 1500))):
            def rr():
                a, b = key(), key()
                return KeyRange(min(a, b), max(a, b))

            txns.append(CommitTransaction([rr() for _ in range(int(rng.integers(0, 4)))],
                                          [rr() for _ in range(int(rng.integers(0, 3)))],
                                          now - int(rng.integers(0, 700)), bool(rng.random() < 0.3)))
        pb = PackedBatch.from_transactions(txns)
        if rng.random() < 0.5:
            oldest = max(oldest, now - int(rng.integers(100, 600)))
        ve, ce = e.detect(pb, now, oldest)
        vo, co = o.detect(pb, now, oldest)
        if not (ve == vo).all():
            return f"verdicts batch {i}: {int((ve != vo).sum())} differ, first {np.nonzero(ve != vo)[0][:5].tolist()}"
        ce = {t: v for t, v in ce.items() if v}
        co = {t: sorted(v) for t, v in co.items() if v}
        if ce != co:
            return f"conflicting reads batch {i}"
    e.cs.close()
    return None


def main():
    budget = float(sys.argv[1]) if len(sys.argv) > 1 else 120.0
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    oracle.build()
    t0 = time.time()
    n = 0
    while time.time() - t0 < budget:
        err = one(seed)
        knobs = {k: os.environ[k] for k in KNOBS}
        if err:
            print(f"MISMATCH seed {seed} knobs {knobs}: {err}", flush=True)
            sys.exit(1)
        n += 1
        if n % 10 == 0:
            print(f"{n} rounds ok ({time.time() - t0:.0f} s), last seed {seed}", flush=True)
        seed += 1
    print(f"stress: {n} random rounds, every batch exact ({time.time() - t0:.0f} s)")


if __name__ == "__main__":
    main()
