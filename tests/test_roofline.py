"""The bench line's bookkeeping (roofline.py), on CPU: every kernel the committed rocprof rankings
name has a byte model, the whole-tier epilogue is priced on the base and the per-batch one on the
delta, and profile files of another build are refused."""
import glob
import json
import os
import shutil

import roofline

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHAPE = {"T": 5000.0, "R": 25000.0, "W": 10000.0, "E": 70000.0, "G": 35000.0, "N": 5e6, "Nd": 2e5, "U": 9000.0,
         "X": 0.0, "merge_bytes": 1e7, "compact_bytes": 3e8, "dir_share": 1.0, "tail_bytes": 0.0, "long_share": 0.0}


def test_every_ranked_kernel_has_a_model():
    files = glob.glob(os.path.join(ROOT, "profiles", "rocprof_*.json"))
    assert files
    for f in files:
        with open(f) as fh:
            d = json.load(fh)
        for name in d["kernels"]:
            b, model = roofline.kernel_bytes(name, SHAPE)
            assert b is not None and b >= 0, (os.path.basename(f), name, model)


def test_epilogue_priced_on_the_tier_it_rebuilds():
    per_batch, _ = roofline.kernel_bytes("k_epilogue<false>", SHAPE)
    whole, _ = roofline.kernel_bytes("k_epilogue<true>", SHAPE)
    # versions (8 B), a sampled key read and its skey8 entry written per 8 boundaries, the level-1
    # max and level-0 sample per 64 (element bytes: no line rounding)
    per_boundary = 8 + 2 * 16 / 8 + (8 + 16) / 64
    fixed = SHAPE["T"] * 2 + SHAPE["R"] * 6
    assert abs(per_batch - (SHAPE["Nd"] * per_boundary + fixed)) < 1e-6
    assert abs(whole - (SHAPE["N"] * per_boundary + fixed)) < 1e-6


def test_profiles_of_another_build_are_refused(tmp_path):
    src = os.path.join(ROOT, "profiles", "rocprof_c2_5000_5000000.json")
    os.makedirs(tmp_path / "profiles")
    shutil.copy(src, tmp_path / "profiles")
    with open(src) as fh:
        measured = json.load(fh)["build_id"]
    kern, note = roofline.rocprof_kernels(str(tmp_path), "c2", 5000, 5000000, measured)
    assert kern and "k_sort_bucket<false>" in kern
    kern, note = roofline.rocprof_kernels(str(tmp_path), "c2", 5000, 5000000, "0" * 16)
    assert kern is None and "measured build" in note
    traffic, note = roofline.pmc_traffic(str(tmp_path), "c2", "k_sort_bucket<false>", 5000, 5000000, measured)
    assert traffic is None and note.startswith("no pmc_")


def test_sort_priced_by_survey_8d():
    """one sort pass is 2E(P + 8); the partition E(D + I) -- no sector or atomic terms."""
    b, model = roofline.kernel_bytes("k_sort_bucket<false>", SHAPE)
    assert b == 2 * SHAPE["E"] * (16 + 8) and "8(d)" in model
    b, model = roofline.kernel_bytes("k_sort_partition", SHAPE)
    assert b == SHAPE["E"] * (24 + 32) and "8(d)" in model
