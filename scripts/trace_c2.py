"""C2 (or C3 / C4: third argument "c3" / "c4") batches run one at a time with FDBCS_TRACE=1: prints device
timestamps of kernel sections."""
import os
import sys

os.environ["FDBCS_TRACE"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from foundationdb_amd import build, conflict_set as C, workloads as W  # noqa: E402

build.build()
wl = sys.argv[3] if len(sys.argv) > 3 else "c2"
if wl == "c4":
    p = W.C4Params(txns=int(sys.argv[2]) if len(sys.argv) > 2 else 5000,
                   history=int(os.environ.get("HISTORY", 50_000_000)))
    kb, ko, vers = W.c4_history(p, seed=1000, start_version=10_000_000)
else:
    p = W.C2Params(txns=int(sys.argv[2]) if len(sys.argv) > 2 else 5000)
    kb, ko, vers = W.c2_history(p, seed=1, start_version=10_000_000)
cs = C.ConflictSet(0)
cs.load_history(kb, ko, vers, 0)
rng = np.random.default_rng(5)
zipf = W.ZipfGenerator(1_000_000, 0.99) if len(sys.argv) > 3 and sys.argv[3] == "c3" else None
now = 10_000_000
for i in range(int(sys.argv[1]) if len(sys.argv) > 1 else 12):
    now += p.version_step
    pb = W.c4_batch(p, rng, now) if wl == "c4" else (W.c3_batch(p, rng, now, zipf) if zipf else W.c2_batch(p, rng, now))
    b = C.ConflictBatch(cs)
    b.add_packed(pb)
    b.upload()
    b.detect_async(now, now - p.window)
    b.wait()
    b.close()
