import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

REFERENCE = "/root/reference"
SCENES = os.path.join(ROOT, "sspp_amd", "scenes")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:  # pragma: no cover
        return False


@pytest.fixture(scope="session")
def golden():
    import numpy as np
    return np.load(os.path.join(ROOT, "tests", "golden", "bsplines_golden.npz"))


@pytest.fixture(scope="session")
def cuda():
    if not gpu_available():
        pytest.skip("no GPU visible (run with -m gpu on an MI355X)")
    import torch
    return torch.device("cuda:0")


def arc_err(got, want):
    """Max |got - want| over finite entries; +inf when the +inf patterns differ (collision-free
    candidates carry an arc length, colliding ones +inf — findBestPath semantics)."""
    import numpy as np
    got, want = np.asarray(got, np.float64), np.asarray(want, np.float64)
    if not np.array_equal(np.isinf(got), np.isinf(want)):
        return float("inf")
    fin = np.isfinite(want)
    return float(np.abs(got[fin] - want[fin]).max()) if fin.any() else 0.0
