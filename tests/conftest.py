import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session")
def oracle_built():
    from oracle import oracle

    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def engine():
    """The HIP engine; GPU tests only.  Builds in-tree if needed and fails loudly without a device."""
    import torch

    # torch ships its own HIP runtime: let it probe the device before the engine's runtime
    # initializes (the order bench.py uses), so tests can hand torch device memory to the engine
    torch.cuda.is_available()
    from foundationdb_amd import build, conflict_set

    os.environ.setdefault("FDBCS_VALIDATE", "1")  # device-side sort/permutation invariant checks
    build.build()
    conflict_set.load_library()
    return conflict_set
