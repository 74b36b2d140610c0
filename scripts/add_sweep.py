"""addTransaction host cost per C2 / C4 batch under FDBCS_ADD_THREADS and FDBCS_PIN_IN (one
process per setting; run on the GPU box).  Prints ms per batch of fdbcs_batch_add_packed."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

torch.cuda.is_available()
from foundationdb_amd import conflict_set as C  # noqa: E402
from foundationdb_amd import workloads as W  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "c2"
p = W.C4Params(history=0) if wl == "c4" else W.C2Params(history=0)
rng = np.random.default_rng(1)
bs = [(W.c4_batch(p, rng, 1000 + i) if wl == "c4" else W.c2_batch(p, rng, 1000 + i)) for i in range(40)]
cs = C.ConflictSet(0)
cs.reserve(1 << 20, 1 << 26, p.txns, p.txns * 8, p.txns * 4)
ts = []
for i, pb in enumerate(bs):
    b = C.ConflictBatch(cs)
    t = time.perf_counter()
    b.add_packed(pb)
    ts.append(time.perf_counter() - t)
    b.close()
st = cs.stats()
print(f"{wl} threads={os.environ.get('FDBCS_ADD_THREADS', 'default')} pin={os.environ.get('FDBCS_PIN_IN', 'coherent')}: "
      f"python-timed median {np.median(ts[8:]) * 1e3:.4f} ms, engine {st['host_ms_add'] / max(1, st['added_txns']) * p.txns:.4f} ms per batch",
      flush=True)
cs.close()
