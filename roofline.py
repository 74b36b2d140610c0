"""Algorithmic bytes per launch of the hot kernels, for the bench roofline.

The §8(d) model prices the work, not this implementation's traffic: a kernel's `achieved` GB/s is
these bytes divided by its measured average launch time, and `frac` = achieved / 8 TB/s (MI355X
HBM3E, /opt/skills/guides/MI355X_MICROARCH.md).  PMC counters (scripts/gpu_pmc.sh) give the
bytes a kernel really moved; the two side by side show wasted re-reads.

Notation (§8(d)): P = 16 (key prefix bytes), L = 4 (length/offset bytes), V = 8 (version bytes),
N = live history boundaries, F = 9 (fan-out of a 128-byte node holding 8 keys), l = search-tree
levels resident in LDS (not fetched from HBM per lookup), R / W = read / write ranges, T = txns,
E = 2 (R + W) endpoints.

* D.CheckRead (k_check_tier<true>: the base tier, N = base boundaries; k_check_reads over both
  tiers when the check is not split), per launch:
    search    2R(P+L) + 2R*4 + 2R*128*max(0, ceil(log_F N) - l)
    range-max R*2V + T
* D.Sort (k_bucket_sort): one read and one write of every 32-byte sort item: 2 * 32 * E.
* D.MergeWrite copy (k_merge_copy<BatchIns>) and compaction copy (k_merge_copy<CompactIns>):
  32 B (key 16 + length/tail 8 + version 8) per kept boundary read, per inserted boundary read,
  and per boundary of the result written; counted exactly by the engine from the device scalars
  (fdbcs_stats.merge_bytes / compact_bytes).
"""
from __future__ import annotations

import math

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
P, L, V, F = 16, 4, 8, 9
NODE = 128


def search_levels(n: float) -> int:
    return max(1, math.ceil(math.log(max(n, 2.0), F)))


def check_bytes(reads: float, txns: float, n: float, lds_levels: int = 0) -> float:
    """Algorithmic bytes of one read-check launch over `reads` ranges and a history of n boundaries."""
    lv = max(0, search_levels(n) - lds_levels)
    search = 2 * reads * (P + L) + 2 * reads * 4 + 2 * reads * NODE * lv
    rmax = reads * 2 * V + txns
    return search + rmax


def sort_bytes(items: float) -> float:
    return 2 * 32 * items


def kernel_entry(name: str, ms_total: float, launches: int, bytes_total: float) -> dict:
    launches = max(1, int(launches))
    avg_ms = ms_total / launches
    per = bytes_total / launches
    ach = per / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    return {
        "kernel": name,
        "launches": launches,
        "total_ms": ms_total,
        "avg_launch_ms": avg_ms,
        "algorithmic_bytes_per_launch": per,
        "achieved_GBps": ach,
        "frac": ach / HBM_PEAK_GBS,
    }


def kernels_from_stats(st: dict, lds_levels: int = 0) -> dict:
    """Per-kernel roofline entries from fdbcs_stats accumulated at timing level >= 1."""
    out = {}
    if st.get("check_launches", 0) > 0:
        n = st["check_launches"]
        avg_reads = st["check_reads"] / n
        avg_hist = st["check_history"] / n
        avg_txn = st["transactions"] / max(1, st["batches"])
        out["check"] = kernel_entry("D.CheckRead: k_check_reads (both tiers) or k_check_tier<base> (split), search + range max",
                                    st["ms_check_kernel"], n,
                                    n * check_bytes(avg_reads, avg_txn, avg_hist, lds_levels))
        out["check"]["model"] = {"reads": avg_reads, "history": avg_hist, "lds_levels": lds_levels,
                                 "search_levels": search_levels(avg_hist)}
    if st.get("sort_launches", 0) > 0:
        out["sort"] = kernel_entry("k_bucket_sort (D.Sort)", st["ms_sort_kernel"], st["sort_launches"],
                                   sort_bytes(st["sort_items"]))
    if st.get("merge_launches", 0) > 0 and st.get("ms_merge_kernel", 0) > 0:
        out["merge"] = kernel_entry("k_merge_copy<BatchIns> (D.MergeWrite delta-tier copy)", st["ms_merge_kernel"],
                                    st["merge_launches"], st["merge_bytes"])
    if st.get("compactions", 0) > 0 and st.get("ms_compact_kernel", 0) > 0:
        out["compact"] = kernel_entry("k_merge_copy<CompactIns> (base-tier compaction copy)",
                                      st["ms_compact_kernel"], st["compactions"], st["compact_bytes"])
    return out


def dominant(kernels: dict) -> str | None:
    """The kernel with the largest total device time."""
    if not kernels:
        return None
    return max(kernels, key=lambda k: kernels[k]["total_ms"])
