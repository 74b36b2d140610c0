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


def list_scenarios():
    """Scenarios for the verdict-list tests (SkipList.cpp:869-876): every KAT scenario plus random
    sequences whose snapshots straddle the oldest version (TooOld transactions in most batches).
    Each scenario is a list of steps ("clear", version) or ("batch", PackedBatch, now, new_oldest)."""
    from foundationdb_amd import workloads as W

    out = []
    for scn in load_json("kat_scenarios.json"):
        steps = []
        for i, (pb, now, no, _, _) in enumerate(scenario_batches(scn)):
            if scn.get("clear_before") == i:
                steps.append(("clear", scn["clear_version"]))
            steps.append(("batch", pb, now, no))
        out.append(steps)
    rng = np.random.default_rng(869)
    for s in range(4):
        steps, now = [], 20
        for _ in range(6):
            pb = W.random_small_batch(rng, int(rng.integers(5, 40)), alphabet=3, max_len=2, now=now, staleness=25)
            steps.append(("batch", pb, now, now - 10))
            now += 4
        out.append(steps)
    return out


def write_list_file(scenarios, path):
    """The scenarios in tests/cpp/shim_driver.cpp's --lists format."""
    lines = []
    for steps in scenarios:
        lines.append("S")
        for st in steps:
            if st[0] == "clear":
                lines.append(f"C {st[1]}")
                continue
            _, pb, now, no = st
            txns = pb.to_transactions()
            lines.append(f"B {now} {no} {len(txns)}")
            for t in txns:
                keys = []
                for r in list(t.read_conflict_ranges) + list(t.write_conflict_ranges):
                    keys += [bytes(r.begin).hex() or "-", bytes(r.end).hex() or "-"]
                lines.append(f"T {t.read_snapshot} {int(bool(t.report_conflicting_keys))} "
                             f"{len(t.read_conflict_ranges)} {len(t.write_conflict_ranges)} " + " ".join(keys))
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


def oracle_scenario_lists(oracle_mod, scenarios):
    """Per batch: (nonConflicting, tooOld) with a tooOld list and nonConflicting without one, from
    the oracle's restatement of SkipList.cpp:869-876."""
    out = []
    for steps in scenarios:
        cs = oracle_mod.OracleConflictSet()
        res = []
        for st in steps:
            if st[0] == "clear":
                cs.clear(st[1])
                continue
            _, pb, now, no = st
            v, _ = cs.detect(pb, now, no)
            nc, to = cs.last_lists(True)
            nc2, _ = cs.last_lists(False)
            res.append((v, nc, to, nc2))
        out.append(res)
    return out
