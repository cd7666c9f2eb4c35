import os
import pathlib
import sys

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def orbx_lib():
    """liborbx.so, rebuilt in-tree when missing or stale (hipcc cross-compiles without a GPU).
    Staleness is by content: the library carries a hash of the sources it was built from, so
    a library that does not match the tree under test is never tested."""
    from my_orb_slam2_amd import build as b
    if b.stale():
        print(f"{b.LIB} is missing or stale: rebuilding", file=sys.stderr, flush=True)
        b.build()
    from my_orb_slam2_amd import _lib
    L = _lib.load()
    assert b.source_hash() in L.orbx_version().decode(), "loaded library is not this tree's"
    return L


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no GPU is visible")
    return torch.device("cuda", 0)
