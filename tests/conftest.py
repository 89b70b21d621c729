import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(Path(__file__).resolve().parent))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running CPU test")
    config.addinivalue_line("markers", "config: full-size BASELINE config parity (runs first)")


def pytest_collection_modifyitems(session, config, items):
    """Full-size BASELINE config tests (tests/test_gpu_configs.py) run before everything
    else, so that under `-x` a failure elsewhere cannot leave a config unexercised."""
    items.sort(key=lambda it: 0 if it.get_closest_marker("config") else 1)  # stable


@pytest.fixture(scope="session")
def oracle():
    """The CPU checker (oracle/, test infrastructure only)."""
    import _oracle
    return _oracle.load()


@pytest.fixture(scope="session")
def lib():
    from subspace_amd import _lib
    if not _lib.LIB_PATH.exists():
        subprocess.run(["make", "-C", str(ROOT)], check=True)
    return _lib.load()


@pytest.fixture(scope="session")
def gpu_ctx():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from subspace_amd.gpu import CrcContext
    ctx = CrcContext(0)
    yield ctx
    ctx.close()


@pytest.fixture(scope="session")
def gpu_ctx_c():
    """A context on the CRC-32C (Castagnoli) polynomial."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from subspace_amd.gpu import POLY_CASTAGNOLI, CrcContext
    ctx = CrcContext(0, poly=POLY_CASTAGNOLI)
    yield ctx
    ctx.close()


@pytest.fixture(autouse=True)
def _release_cached_device_memory(request):
    """After every GPU test, hand torch's cached blocks back to the driver: the full-size
    tests (config C holds 118 GB, the 2^31-message test 52 GB) check torch.cuda.mem_get_info,
    which counts cached blocks as used."""
    yield
    if request.node.get_closest_marker("gpu"):
        torch = sys.modules.get("torch")
        if torch is not None and torch.cuda.is_available():
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
