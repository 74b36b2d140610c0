"""Shared test helpers: golden fixture loading and a uniform driver over the oracle / HIP engine."""
import json
import os

import numpy as np

from foundationdb_amd.packing import CommitTransaction, KeyRange, PackedBatch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_json(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def scenario_batches(scn):
    """Yield (PackedBatch, now, new_oldest, expect, conflicting) per batch of a KAT scenario."""
    for b in scn["batches"]:
        txns = []
        for t in b["txns"]:
            txns.append(
                CommitTransaction(
                    [KeyRange(bytes.fromhex(x), bytes.fromhex(y)) for x, y in t["reads"]],
                    [KeyRange(bytes.fromhex(x), bytes.fromhex(y)) for x, y in t["writes"]],
                    t["snapshot"],
                    t["report"],
                )
            )
        conf = {int(k): v for k, v in b.get("conflicting", {}).items()}
        yield PackedBatch.from_transactions(txns), b["now"], b["new_oldest"], b["expect"], conf


def random_fixture_sequences():
    z = np.load(os.path.join(GOLDEN, "random_batches.npz"))
    seqs, nb = (int(x) for x in z["meta"])
    for s in range(seqs):
        seq = []
        for b in range(nb):
            p = f"s{s}b{b}_"
            pb = PackedBatch(z[p + "snap"], z[p + "report"], z[p + "roff"], z[p + "woff"], z[p + "kb"], z[p + "ko"])
            now, no = (int(x) for x in z[p + "now"])
            ct = z[p + "conf_txn"]
            co = z[p + "conf_off"]
            ci = z[p + "conf_idx"]
            conf = {int(ct[i]): ci[co[i] : co[i + 1]].tolist() for i in range(len(ct))}
            seq.append((pb, now, no, z[p + "verdict"], conf))
        yield s, seq


class EngineDriver:
    """Runs packed batches through the HIP engine's Python mirror of ConflictBatch."""

    def __init__(self, cs_module, device=0, gc_interval=1, delta_limit=0):
        self.C = cs_module
        self.cs = cs_module.ConflictSet(device)
        self.cs.set_gc_interval(gc_interval)
        self.cs.set_delta_limit(delta_limit)

    def clear(self, v):
        self.cs.clear(v)

    def load_history(self, kb, ko, vers, header=0):
        self.cs.load_history(kb, ko, vers, header)

    def detect(self, pb, now, new_oldest):
        m = {}
        b = self.C.ConflictBatch(self.cs, m)
        b.add_packed(pb)
        v = b.detect_conflicts(now, new_oldest)
        b.close()
        return v, {t: sorted(x) for t, x in m.items()}


def nonempty(conf):
    return {t: sorted(v) for t, v in conf.items() if v}
