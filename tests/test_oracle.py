"""The oracle (oracle/split_step.py, numpy float64) pinned against the reference's golden fixtures
(tests/golden/, produced by importing the reference src/model_def.py — make_golden.py)."""
import numpy as np
import pytest

from conftest import FIXTURES, PARAMS, load_fixture, rel_err, weight_ok
from oracle import split_step as O


def _params(fx, prefix):
    return {k: fx[prefix + k].astype(np.float64) for k in PARAMS}


@pytest.mark.parametrize("name", FIXTURES)
def test_oracle_matches_reference_fixture(name):
    fx = load_fixture(name)
    P = _params(fx, "init_")
    for s in range(1, int(fx["nsteps"]) + 1):
        new, rec = O.split_step(P, fx[f"x_{s}"], fx[f"y_{s}"])
        assert rel_err(rec["act"], fx[f"act_{s}"]) <= 1e-6
        assert rel_err(rec["logits"], fx[f"logits_{s}"]) <= 1e-5
        assert abs(rec["loss"] - float(fx[f"loss_{s}"])) <= 2e-6 * abs(float(fx[f"loss_{s}"]))
        assert rel_err(rec["cut_grad"], fx[f"cut_grad_{s}"]) <= 1e-5
        if s == 1:
            for k in PARAMS:
                assert rel_err(rec["grads"][k], fx[f"grad_{k}_1"]) <= 1e-5, k
        if f"post_W1_{s}" in fx:
            for k in PARAMS:
                assert weight_ok(new[k], fx[f"post_{k}_{s}"], P[k], rtol=1e-5), k
        P = new


def test_oracle_ties_route_to_first_max():
    fx = load_fixture("split_step_ties_b2.npz")
    P = _params(fx, "init_")
    _, rec = O.split_step(P, fx["x_1"], fx["y_1"])
    idx = rec["idx"]
    pooled = rec["pooled"]
    # constant images -> every window is a 4-way tie: the argmax must be position 0 everywhere
    assert (idx[pooled > 0] == 0).all()
    assert rel_err(rec["cut_grad"], fx["cut_grad_1"]) <= 1e-5


def test_oracle_loss_curve_prefix():
    """The first 30 steps of the 1k-step reference loss curve at B=64."""
    import torch  # noqa: F401  (SyntheticMNIST uses torch's CPU generator)
    from splitcnn.data import SyntheticMNIST
    fx = load_fixture("loss_curve_b64.npz")
    fx1 = load_fixture("split_step_b4.npz")
    P = _params(fx1, "init_")  # seed-0 init, same as the curve's
    data = SyntheticMNIST(42)
    for s in range(30):
        x, y = data.batch(64)
        P, rec = O.split_step(P, x.numpy(), y.numpy())
        assert abs(rec["loss"] - float(fx["losses"][s])) <= 1e-4 * float(fx["losses"][s]), s


def test_maxpool_first_max_semantics():
    r = np.zeros((1, 1, 2, 2))
    r[0, 0] = [[1.0, 3.0], [3.0, 2.0]]
    p, idx = O.maxpool2(r)
    assert p[0, 0, 0, 0] == 3.0 and idx[0, 0, 0, 0] == 1
    d = O.maxpool2_bwd(np.ones((1, 1, 1, 1)), idx, r.shape)
    assert d[0, 0].tolist() == [[0.0, 1.0], [0.0, 0.0]]
