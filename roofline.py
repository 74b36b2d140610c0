"""Algorithmic bytes per launch of every pipeline kernel, for the bench roofline.

The model prices the work the kernel must do, at element granularity (no sector, line or
memory-side-atomic rounding: those are this implementation's traffic, which PMC measures), not
this implementation's traffic: `achieved` GB/s
is these bytes divided by the kernel's measured average launch time (HIP events around the
kernel on the stream it runs on), and `frac` = achieved / 8 TB/s (MI355X HBM3E,
/opt/skills/guides/MI355X_MICROARCH.md).  PMC counters (scripts/gpu_pmc.sh) give the bytes a
kernel really moved (`traffic`); the two side by side show wasted re-reads.

Notation (§8(d)): P = 16 (key prefix bytes), V = 8 (version bytes), D = 24 (a batch key record:
prefix, length, tail offset), I = 32 (a sort item), N / Nd = base / delta history boundaries,
R / W = read / write ranges, T = transactions, E = 2 (R + W) endpoints, G = R + W ranges,
U = union segments of committed writes, X = candidate intra-batch edges.

A lookup in a tier is priced by the nodes it must read: a 128-byte node per search-tree level
(8 sampled keys), ceil(log_8(N / 64)) levels above the 64-boundary block plus the skey8 line and
the 8 boundaries of the final group (3 lines); a lookup whose first two key bytes fall in a sparse
slot of the tier's radix directory starts at level 0 (the directory entry, the level-0 group, the
skey8 line and the boundary group: `dir_levels`).  Which path a lookup takes depends on the key
distribution: the bench estimates the directory share from the prefilled history (shape_of).
"""
from __future__ import annotations

import json
import math
import os

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
P, V, D, I = 16, 8, 24, 32
NODE = 128


def tree_levels(n: float) -> int:
    """128-byte nodes one lookup reads descending the full tree over n boundaries."""
    if n <= 0:
        return 0
    return max(1, math.ceil(math.log(max(n / 64.0, 2.0), 8))) + 2


def lookup_bytes(n: float, dir_share: float) -> float:
    if n <= 0:
        return 0.0
    direct = 8 + 3 * NODE
    return dir_share * direct + (1 - dir_share) * tree_levels(n) * NODE


def shape_of(batches, st: dict, history: int, dir_share: float = 1.0) -> dict:
    """Average batch shape of the measured batches plus per-batch history sizes from the engine's
    stats (fdbcs_stats: base_sum / delta_sum / segments_sum / intra_edges over `batches`)."""
    nb = max(1, len(batches))
    b = max(1, st.get("batches", 0))
    T = sum(x.n_txn for x in batches) / nb
    R = sum(x.n_reads for x in batches) / nb
    W = sum(x.n_writes for x in batches) / nb
    return {
        "T": T, "R": R, "W": W, "E": 2 * (R + W), "G": R + W,
        "N": st.get("base_sum", 0) / b if st.get("base_sum") else float(history),
        "Nd": st.get("delta_sum", 0) / b,
        "U": st.get("segments_sum", 0) / b,
        "X": st.get("intra_edges", 0) / max(1, b - st.get("intra_fallbacks", 0)),
        "merge_bytes": st.get("merge_bytes_all", 0) / b,
        "compact_bytes": st.get("compact_bytes_all", 0) / max(1, st.get("compactions", 0)),
        "dir_share": dir_share,
        # tail bytes per batch and the share of endpoints whose keys run past 16 bytes
        "tail_bytes": sum(x.tail_bytes for x in batches) / nb,
        "long_share": sum(x.long_endpoints for x in batches) / max(1.0, sum(2 * (x.n_reads + x.n_writes) for x in batches)),
    }


def kernel_bytes(name: str, s: dict):
    """(bytes per launch, model text) of kernel `name` (engine demangled name) at shape s."""
    T, R, W, E, G, N, Nd, U, X = (s[k] for k in ("T", "R", "W", "E", "G", "N", "Nd", "U", "X"))
    S = min(E, max(1024.0, min(8192.0, 4 * math.ceil(E / 128))))
    nb = min(2048.0, math.ceil(E / 128))
    look_b, look_d = lookup_bytes(N, s["dir_share"]), lookup_bytes(Nd, 0.5)
    if name == "k_check_lanes" or name.startswith("k_check_lanes<") or name.startswith("k_check_reads"):  # both tiers
        return (2 * R * (D + look_b + look_d) + R * (4 + V) + 2 * R * V + T,
                "2R(D + base lookup + delta lookup) + R(owner + snapshot) + range-max ends 2RV + T")
    if name.startswith("k_check_tier<true") or name.startswith("k_check_lanes_tier<true"):
        return (2 * R * (D + look_b) + R * (4 + V) + R * V + T, "base tier: 2R(D + lookup) + R(4+V) + RV + T")
    if name.startswith("k_check_tier<false") or name.startswith("k_check_lanes_tier<false"):
        return (2 * R * (D + look_d) + R * (4 + V) + R * V + T, "delta tier: 2R(D + lookup) + R(4+V) + RV + T")
    if name == "k_sample":
        return S * (D + I + 4), "S samples: key read, item written, rank"
    if name == "k_quant_cold":
        # kQuant (4096) quantiles: rank inverse of the S samples, each quantile's item read and its
        # SplitKey (8 words, length, meta: 72 B) written
        return S * 8 + 4096 * (I + 72), "cold start: sample ranks inverted, 4096 quantile items read and splitters written"
    if name == "k_lvl3_reset":
        return 8 * (N / (64.0 ** 3) + N / (64.0 ** 2) + 2), "range-max levels 2 and 3 of a tier reset before a rebuild"
    if name == "k_bucket_count":
        return E * (D + 2) + nb * (I + 4), "E keys read, E bucket ids written, splitters"
    if name == "k_bucket_scatter":
        return E * (2 + D + I) + nb * 8, "E (bucket id + key) read, E items written"
    if name.startswith("k_bucket_sort"):
        return 2 * I * E, "one read and one write of every 32-byte item"
    if name == "k_sort_partition":
        # E·(D + I) -- every endpoint's key record read once and its sort item
        # written once.  Keys over 16 bytes add their tail bytes (read once).  The slot atomics and
        # the write keys' tail copy are this implementation's traffic (PMC `traffic`), not the model.
        tl = s.get("tail_bytes", 0.0)
        return (E * (D + I) + tl,
                "SURVEY 8(d): E(D + I), every endpoint's key record read and its item written once; + tail bytes of "
                "keys over 16 B")
    if name.startswith("k_sort_bucket"):
        # SURVEY §8(d) intra term: one sort pass = 2·E·(P + 8) (every endpoint's prefix and its
        # 8-byte length/class/owner word read and written once).  Scattered stores, sectors and
        # lines are `traffic`, not algorithmic bytes.
        tl = s.get("tail_bytes", 0.0)
        return (2 * E * (P + 8) + tl,
                "SURVEY 8(d): one sort pass 2E(P + 8), every endpoint's prefix and 8-byte word read and written once; "
                "+ tail bytes of keys over 16 B")
    if name.startswith("k_scan<3, fdbcs::PosScan"):
        return E * (4 + 4 + 4 + 12) + G * 4, "E metas read; pos, pmeta, 3 class prefixes written; R+W begin lists"
    if name.startswith("k_scan<3, fdbcs::EdgePairScan"):
        # per range its two sorted positions, the three 4-byte class prefixes at both, its slot / pair
        # offsets; writes also place their sorted endpoint records and keys for D.Combine
        return (G * (8 + 6 * 4 + 8) + W * (2 * 8 + 2 * D + 8),
                "per range: 2 positions, 3 class prefixes at both (6 x 4 B), slot/pair offsets; per write its two "
                "sorted endpoint records and keys, group lead and owner")
    if name == "k_edge_fill":
        return X * (4 + 4 + 4 + 4) + G * 8, "per edge: partner, owner, slot atomic, edge; range offsets"
    if name == "k_resolve_pre":
        if X > 0:
            return (T * (1 + 1 + 4 + 1 + 4) + X * (4 + 1 + 1 + 4) + T * 12,
                    "pre-pass: per transaction its flags and edge runs, per edge the writer and its flags, packed live "
                    "writers, resume pointers")
        return (T * (1 + 1 + 1 + 4 + 1) + 2 * W * (8 + 1 + 1 + 1) + U * (2 * D + 8),
                "statuses (hist flag, tooOld flag, status, first conflict, verdict); D.Combine: per write endpoint its "
                "record, owner's flags, segment flag; per segment 2 keys and 2 positions")
    if name.startswith("k_resolve<") or name == "k_resolve":
        if X == 0:
            return 8, "no candidate edges: the pre-pass decided and combined; one scalar"
        return (T * (1 + 1 + 8 + 4 + 1) + X * (4 + 1) + W * 16,
                "statuses, flags, resume pointers, edges and writer states, write-group members, verdicts")
    if name == "k_combine":
        if X == 0:
            return 8, "no candidate edges: the pre-pass combined; one scalar"
        return (2 * W * (8 + 1 + 1 + 1) + U * (2 * D + 8),
                "D.Combine: per write endpoint its record, owner's status, segment flag; per segment 2 keys and 2 positions")
    if name == "k_intra_report":
        return R * 12, "per read: edge range, first conflict"
    if name.startswith("k_seg_prep"):
        return (U * 2 * (D + look_d) + U * (8 + 8 + 1 + 8 + 24 + 4),
                "per segment: 2 keys + 2 delta lookups; lo, hi, end flag, inherited version, 3 prefixes, tile index")
    if name.startswith("k_merge_copy<fdbcs::BatchIns"):
        return s["merge_bytes"], "32 B per kept and inserted boundary read and per result boundary written (device scalars)"
    if name.startswith("k_merge_copy<fdbcs::CompactIns"):
        return s["compact_bytes"], "32 B per kept base / inserted delta boundary read and per result boundary written"
    if name.startswith("k_compact_search"):
        return Nd * (P + 8 + lookup_bytes(N, s["dir_share"]) + 17), "per delta boundary: key + lookup in the base, 2 words"
    if name.startswith("k_scan<2, fdbcs::CompactSumScan"):
        return Nd * (8 + 8 + 1 + 24), "per delta boundary: lo, version, exact flag; 3 words written"
    if name.startswith("k_scan<2, fdbcs::GcScan"):
        return N * (2 * V + 8) + N * 32, "versions (own + predecessor) and lengths read, kept boundaries rewritten"
    if name.startswith("k_epilogue"):
        # the levels and sample index of the tier that changed: the delta after a merge
        # (k_epilogue<false>), the whole base after a compaction (k_epilogue<true>); per boundary its
        # version read, per 8 boundaries the sampled key read and its skey8 entry written, per 64 the
        # level-1 maximum and the level-0 sample key written
        n = N if name.startswith("k_epilogue<true") or Nd <= 0 else Nd
        return (n * (V + 2 * P / 8 + (V + P) / 64) + T * 2 + R * 6,
                "levels and sample index of the changed tier (the delta after a merge; the base after a compaction, "
                "k_epilogue<true>): versions, per 8 boundaries a sampled key read and its skey8 entry written, per 64 "
                "the level-1 max and sample key; verdicts; re-zeroed flags and edge counts")
    if name == "k_directory":
        return 65537 * (4 + 17 * P), "65537 slots: binary search over level-0 samples"
    if name == "k_conflict_output":
        return T * 6, "per global transaction: map entry, status, conflict byte"
    if name == "k_copy_bytes":
        return T * 2, "report side outputs"
    if name == "k_validate_sort":
        return E * (I + 8), "sorted items and positions re-read"
    return None, "no model"


def entry(name: str, ms_total: float, launches: int, s: dict, st: dict = None) -> dict:
    launches = max(1, int(launches))
    avg_ms = ms_total / launches
    b, model = kernel_bytes(name, s)
    out = {"kernel": name, "launches": launches, "total_ms": ms_total, "avg_launch_ms": avg_ms,
           "algorithmic_bytes_per_launch": b, "model": model}
    if b is not None and avg_ms > 0:
        ach = b / (avg_ms * 1e-3) / 1e9
        out["achieved_GBps"] = ach
        out["frac"] = ach / HBM_PEAK_GBS
    else:
        out["achieved_GBps"] = out["frac"] = None
    return out


def kernel_table(kprof: dict, s: dict, st: dict = None) -> dict:
    """Every kernel of the profile pass with its roofline entry, largest total device time first."""
    rows = {k: entry(k, v["ms"], v["launches"], s, st) for k, v in kprof.items() if not k.startswith("k_hold")}
    return dict(sorted(rows.items(), key=lambda kv: -kv[1]["total_ms"]))


SORT_KERNELS = ("k_sample", "k_quant_cold", "k_bucket_count", "k_bucket_scatter", "k_bucket_sort", "k_sort_")


def sort_phase(table: dict) -> dict | None:
    """D.Sort as one unit: the sort kernels' average launch times summed per batch."""
    ks = {k: v for k, v in table.items() if k.startswith(SORT_KERNELS)}
    if not ks:
        return None
    per_batch = sum(v["total_ms"] for v in ks.values()) / max(v["launches"] for v in ks.values())
    return {"kernels": sorted(ks), "ms_per_batch": per_batch}


# Sources whose content defines the kernels a profile measured: a profile whose build id differs
# from the running tree's describes other code and is not used.
BUILD_SOURCES = ("foundationdb_amd/csrc/kernels.hip", "foundationdb_amd/csrc/engine.cpp",
                 "foundationdb_amd/csrc/engine.h", "foundationdb_amd/csrc/scan.h", "foundationdb_amd/csrc/launch.h",
                 "foundationdb_amd/csrc/dkey.h", "foundationdb_amd/csrc/lane_xor.h",
                 "include/fdb_conflict_set.h")


def build_id(root: str) -> str:
    """Content hash of the engine sources (the GPU box has no .git: the tree itself is the identity)."""
    import hashlib

    h = hashlib.sha256()
    for rel in BUILD_SOURCES:
        with open(os.path.join(root, rel), "rb") as f:
            h.update(rel.encode() + b"\0" + f.read())
    return h.hexdigest()[:16]


def _profile(root: str, prefix: str, workload: str, txns: int, history: int, build: str):
    f = os.path.join(root, "profiles", f"{prefix}_{workload}_{txns}_{history}.json")
    if not os.path.exists(f):
        return None, f"no {os.path.basename(f)}"
    try:
        with open(f) as fh:
            d = json.load(fh)
    except Exception as e:  # noqa: BLE001
        return None, f"{os.path.basename(f)} unreadable: {e}"
    if d.get("build_id") != build:
        return None, f"{os.path.basename(f)} measured build {d.get('build_id')}, running build {build}"
    return d, f"profiles/{os.path.basename(f)} (build {build}, git {d.get('git_head')})"


def pmc_traffic(root: str, workload: str, kernel: str, txns: int, history: int, build: str):
    """(HBM bytes per launch of `kernel`, source note) from the PMC passes of the SAME configuration
    and the SAME build (profiles/pmc_<workload>_<txns>_<history>.json, written by
    scripts/pmc_summary.py: FETCH_SIZE x2 gfx950 correction + WRITE_SIZE, each in its own
    rocprofv3 pass); None when the file is absent or measured other code."""
    d, note = _profile(root, "pmc", workload, txns, history, build)
    if d is None:
        return None, note
    return d.get("bytes_per_launch", {}).get(kernel), note


def rocprof_kernels(root: str, workload: str, txns: int, history: int, build: str):
    """({kernel: {"calls", "avg_us", "total_ms"}}, source note) from the rocprofv3 kernel-trace
    summary of the same configuration and build (profiles/rocprof_<workload>_<txns>_<history>.json,
    scripts/rocprof_rank.py), or (None, why not)."""
    d, note = _profile(root, "rocprof", workload, txns, history, build)
    if d is None:
        return None, note
    return d.get("kernels"), note
