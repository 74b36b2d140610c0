#!/usr/bin/env python3
"""Join the engine's host spans (FDBCS_HOST_TRACE csv: D detect call, A / X / Y issue of a batch's
stage A / X half / Y half, W wait for its flag) with a rocprofv3 kernel trace of the same run (both
in CLOCK_MONOTONIC ns).  Per chain head (A: k_sort_partition, X: k_check_lanes, Y: k_seg_prep), how
long after its issue began the kernel started, and how often the chain's stream was idle waiting
for the host (the head's issue began after the chain's previous kernel had ended).

    python3 scripts/host_trace.py host.csv kernel_trace.csv [--skip 30]"""
import argparse
import csv
import statistics
from collections import defaultdict


def med(v):
    return statistics.median(v) if v else float("nan")


def q(v, f):
    v = sorted(v)
    return v[min(len(v) - 1, int(f * len(v)))] if v else float("nan")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("host")
    ap.add_argument("kernels")
    ap.add_argument("--skip", type=int, default=30)
    a = ap.parse_args()
    spans = defaultdict(dict)  # kind -> seq -> (t0, t1)
    for r in csv.DictReader(open(a.host)):
        spans[r["kind"]][int(r["seq"])] = (int(r["t0"]), int(r["t1"]))
    ks = defaultdict(list)
    for r in csv.DictReader(open(a.kernels)):
        n = r["Kernel_Name"]
        for key in ("k_sort_partition", "k_sort_bucket", "EdgePairScan", "k_edge_fill", "k_check_lanes", "k_resolve_pre",
                    "k_resolve<", "k_combine", "k_seg_prep", "BatchIns", "k_epilogue"):
            if key in n:
                ks[key].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
                break
    for k in ks:
        ks[k].sort()
    # launches before the first batch's sort belong to the history load (epilogue, directory)
    t_first = ks["k_sort_partition"][0][0] if ks.get("k_sort_partition") else 0
    for k in ks:
        ks[k] = [x for x in ks[k] if x[0] >= t_first]
    seqs = sorted(spans["D"])
    print(f"host spans: {len(seqs)} detect calls; kernels: " + ", ".join(f"{k} {len(v)}" for k, v in ks.items()))
    # the n-th launch of a per-batch kernel belongs to the n-th detected batch
    first = seqs[0]

    def kern(name, seq):
        i = seq - first
        v = ks.get(name, [])
        return v[i] if 0 <= i < len(v) else None

    steady = seqs[a.skip:-5]
    rows = defaultdict(list)
    for s in steady:
        d = spans["D"].get(s)
        for kind, head, prev in (("A", "k_sort_partition", "k_edge_fill"), ("X", "k_check_lanes", "k_combine"),
                                 ("Y", "k_seg_prep", "k_epilogue")):
            sp = spans[kind].get(s)
            kh = kern(head, s)
            kp = kern(prev, s - 1)
            if not sp or not kh:
                continue
            rows[kind + " issue-begin -> head start"].append((kh[0] - sp[0]) / 1e3)
            rows[kind + " issue span"].append((sp[1] - sp[0]) / 1e3)
            if kp:
                rows[kind + " prev chain end -> head start"].append((kh[0] - kp[1]) / 1e3)
                rows[kind + " host-late (issue after prev end)"].append(1.0 if sp[0] > kp[1] else 0.0)
                rows[kind + " host-late by"].append(max(0.0, (sp[0] - kp[1]) / 1e3))
            if d:
                rows[kind + " detect call begin -> issue begin"].append((sp[0] - d[0]) / 1e3)
        w = spans["W"].get(s)
        ke = kern("k_epilogue", s)
        if w and ke:
            rows["W span"].append((w[1] - w[0]) / 1e3)
            rows["W flag seen - epilogue end"].append((w[1] - ke[1]) / 1e3)
            rows["W begin - epilogue end (neg: waited)"].append((w[0] - ke[1]) / 1e3)
        if d:
            rows["D span"].append((d[1] - d[0]) / 1e3)
        dn = spans["D"].get(s + 1)
        if d and dn:
            rows["D period"].append((dn[0] - d[0]) / 1e3)
    for k, v in rows.items():
        if "host-late (" in k:
            print(f"  {k:45s} share {sum(v) / len(v):6.2f}")
        else:
            print(f"  {k:45s} median {med(v):8.1f}  p10 {q(v, 0.1):8.1f}  p90 {q(v, 0.9):8.1f}")
    # stream idle per chain: gaps between consecutive kernels of the chain's stream
    for chain, names in (("A", ["k_sort_partition", "k_sort_bucket", "EdgePairScan", "k_edge_fill"]),
                         ("X", ["k_check_lanes", "k_resolve_pre", "k_resolve<", "k_combine"]),
                         ("Y", ["k_seg_prep", "BatchIns", "k_epilogue"])):
        busy, span = 0.0, 0.0
        for s in steady:
            kk = [kern(n, s) for n in names]
            if all(kk):
                busy += sum(e - b for b, e in kk) / 1e3
        t0 = kern(names[0], steady[0])
        t1 = kern(names[-1], steady[-1])
        if t0 and t1:
            span = (t1[1] - t0[0]) / 1e3
            print(f"  chain {chain}: kernel-busy {busy / span:5.2f} of its span ({span / len(steady):.1f} us per batch)")


if __name__ == "__main__":
    main()
