import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "split-learning-k8s_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

FIXTURES = ["split_step_b4.npz", "split_step_b1.npz", "split_step_b12.npz", "split_step_b13.npz",
            "split_step_ties_b2.npz", "split_step_b14.npz"]
PARAMS = ["W1", "b1", "W2", "b2", "W3", "b3"]


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm) GPU and the built libslk.so")


def load_fixture(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def rel_err(got, want):
    """max |got - want| / max |want| (norm-free, elementwise worst case scaled by the tensor's range)."""
    got = np.asarray(got, dtype=np.float64)
    want = np.asarray(want, dtype=np.float64)
    if got.shape != want.shape and got.size == want.size:
        got = got.reshape(want.shape)
    assert got.shape == want.shape, (got.shape, want.shape)
    scale = max(np.abs(want).max(), 1e-30)
    return float(np.abs(got - want).max() / scale)


def weight_ok(got, want, init, rtol=1e-4):
    """Post-step weights: |got - want| <= rtol * max|want - init| + 2 ulp(fp32, |want|) elementwise.
    The reference stores fp32 weights, so its own rounding (~3e-8 at |w| ~ 0.3) is comparable to
    rtol x a 0.01-lr update; comparing raw deltas at 1e-4 would test fp32 rounding, not the step."""
    got = np.asarray(got, dtype=np.float64)
    want = np.asarray(want, dtype=np.float64)
    init = np.asarray(init, dtype=np.float64)
    tol = rtol * np.abs(want - init).max() + 2 * np.finfo(np.float32).eps * np.abs(want)
    return bool((np.abs(got - want) <= tol).all())


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no ROCm GPU")
    from splitcnn import _lib
    _lib.load()  # fail loudly if the HIP library is missing
    return torch.device("cuda:0")
