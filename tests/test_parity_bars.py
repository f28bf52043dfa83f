"""CPU tests of the parity bars themselves (oracle/parity.py): they pass at the errors the GPU runs
measure and fail on the regressions they exist to catch."""
import numpy as np
import pytest

from oracle import parity as PAR


def _case(P=1000, H=32, W=48, seed=0):
    rng = np.random.default_rng(seed)
    color = rng.uniform(0, 1, (3, H, W)).astype(np.float32)
    depth = rng.uniform(2, 10, (1, H, W)).astype(np.float32)
    grads = [rng.normal(0, 1, (P, 3)).astype(np.float32), rng.normal(0, 1, (P, 16, 3)).astype(np.float32)]
    return color, depth, grads, np.zeros((H, W), np.uint8), np.zeros(P, np.uint8)


def _run(color, depth, grads, o_color, o_depth, o_grads, pflag, gflag, **kw):
    return PAR.check(color, depth, grads, o_color, o_depth, o_grads, pflag, gflag, names=["a", "b"], **kw)


def test_measured_errors_pass():
    color, depth, grads, pflag, gflag = _case()
    rep = _run(color + 1e-6, depth + 1e-6, [g * (1 + 1e-6) for g in grads], color, depth, grads, pflag, gflag)
    assert rep["a"][1] < 0.01


def test_ten_times_regressions_fail():
    color, depth, grads, pflag, gflag = _case()
    with pytest.raises(AssertionError, match="colour"):
        _run(color + 3e-5, depth, grads, color, depth, grads, pflag, gflag)
    # a relative error of 2e-3 on one small element: far below 1e-3 of the tensor's max, above its own bar
    g = [x.copy() for x in grads]
    i = int(np.argmin(np.abs(grads[0][:, 0])))
    g[0][i, 0] = grads[0][i, 0] + 2e-3 * abs(grads[0][i, 0]) + 2e-5 * np.abs(grads[0]).max()
    with pytest.raises(AssertionError, match="per-element|bar"):
        _run(color, depth, g, color, depth, grads, pflag, gflag)


def test_flagged_elements_are_bounded_and_counted():
    color, depth, grads, pflag, gflag = _case()
    g = [x.copy() for x in grads]
    gflag = gflag.copy()
    gflag[:3] = 1
    g[0][:3] *= 1.0005                          # a flip-sized error on flagged Gaussians passes
    _run(color, depth, g, color, depth, grads, pflag, gflag)
    g[0][0] += 0.1 * np.abs(grads[0]).max()     # beyond FLIP_GRAD_MAX fails
    with pytest.raises(AssertionError, match="flagged Gaussian"):
        _run(color, depth, g, color, depth, grads, pflag, gflag)
    gflag[:100] = 1                             # 10 % of the Gaussians flagged: over the cap
    with pytest.raises(AssertionError, match="Gaussians flagged"):
        _run(color, depth, grads, color, depth, grads, pflag, gflag)
