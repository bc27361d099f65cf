"""Shared fixtures.  `gpu` tests run the HIP engine on an MI355X; everything else runs on CPU."""
import ctypes
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from testground_amd import abi  # noqa: E402
from testground_amd.build import build_oracle  # noqa: E402
from testground_amd.engine import CABIEngine  # noqa: E402


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X; drives libtgsim.so through its C ABI")


def pytest_collection_finish(session):
    """torch ships its own HIP runtime: when the run holds GPU tests, let it initialise the device
    before any engine library does, whatever the order the selected tests run in."""
    if not any(item.get_closest_marker("gpu") for item in session.items):
        return
    try:
        import torch
    except ImportError:  # pragma: no cover
        return
    if torch.cuda.is_available():
        torch.cuda.init()


@pytest.fixture(scope="session")
def oracle_lib():
    """The CPU golden model (oracle/), the checker for every parity test."""
    lib = ctypes.CDLL(str(build_oracle()))
    abi.declare(lib, "tgo_")
    lib.tgo_percentage2u32.restype = ctypes.c_uint32
    lib.tgo_percentage2u32.argtypes = [ctypes.c_float]
    return lib


@pytest.fixture
def make_oracle(oracle_lib):
    def _make(n_peers, **kw):
        return CABIEngine(oracle_lib, "tgo_", n_peers, **kw)
    return _make


def pytest_sessionfinish(session, exitstatus):
    """With TGSIM_LIB naming a TGSIM_CHECK build (scripts/check_build.sh), report the cross-lane
    exec-mask guard violations the run's kernels counted."""
    import os

    lib = os.environ.get("TGSIM_LIB", "")
    if not lib.endswith("_check.so"):
        return
    from testground_amd.engine import load_library

    n = load_library().tgsim_debug_exec_faults()
    print(f"\nTGSIM_CHECK exec-mask guard violations: {n}")
