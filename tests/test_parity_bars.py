"""CPU tests of the parity bars themselves (oracle/parity.py): they pass at the errors the GPU runs
measure and fail on the regressions they exist to catch, including on elements with a flip bound."""
import numpy as np
import pytest

from oracle import parity as PAR


def _case(P=1000, H=32, W=48, seed=0):
    rng = np.random.default_rng(seed)
    color = rng.uniform(0, 1, (3, H, W)).astype(np.float32)
    depth = rng.uniform(2, 10, (1, H, W)).astype(np.float32)
    grads = [rng.normal(0, 1, (P, 3)).astype(np.float32), rng.normal(0, 1, (P, 16, 3)).astype(np.float32)]
    bounds = dict(pflag=np.zeros((H, W), np.uint8), gflag=np.zeros(P, np.uint8), pix_rad=np.zeros((H, W), np.float32),
                  depth_rad=np.zeros((H, W), np.float32), grad_rad=[np.zeros_like(g) for g in grads])
    return color, depth, grads, bounds


def _run(color, depth, grads, o_color, o_depth, o_grads, bounds, **kw):
    return PAR.check(color, depth, grads, o_color, o_depth, o_grads, bounds, names=["a", "b"], **kw)


def test_measured_errors_pass():
    color, depth, grads, b = _case()
    rep = _run(color + 1e-6, depth + 1e-6, [g * (1 + 1e-6) for g in grads], color, depth, grads, b)
    assert rep["a"][2] < 0.01


def test_ten_times_regressions_fail():
    color, depth, grads, b = _case()
    with pytest.raises(AssertionError, match="colour"):
        _run(color + 3e-5, depth, grads, color, depth, grads, b)
    # a relative error of 2e-3 on one small element: far below 1e-3 of the tensor's max, above its own bar
    g = [x.copy() for x in grads]
    i = int(np.argmin(np.abs(grads[0][:, 0])))
    g[0][i, 0] = grads[0][i, 0] + 2e-3 * abs(grads[0][i, 0]) + 2e-5 * np.abs(grads[0]).max()
    with pytest.raises(AssertionError, match="bar"):
        _run(color, depth, g, color, depth, grads, b)


def _flagged(b, rows, r):
    b = dict(b, gflag=b["gflag"].copy(), grad_rad=[x.copy() for x in b["grad_rad"]])
    b["gflag"][rows] = 1
    b["grad_rad"][0][rows] = r
    return b


def test_flagged_elements_lie_in_their_flip_interval():
    """An element with a flip bound may move by that bound (plus the per-element bar), not by 10x it; an
    element without one keeps the sharp bars even when its Gaussian is flagged."""
    color, depth, grads, b = _case()
    rad = 0.01 * np.abs(grads[0]).max()
    b = _flagged(b, slice(0, 3), rad)
    g = [x.copy() for x in grads]
    g[0][:3] += rad                               # a whole flip's worth of change: inside the interval
    rep = _run(color, depth, g, color, depth, grads, b)
    assert rep["a"][3] <= 1.0 + 1e-6
    g[0][0, 0] = grads[0][0, 0] + 10 * rad        # 10x the flip bound fails
    with pytest.raises(AssertionError, match="bar|beyond its flip bound"):
        _run(color, depth, g, color, depth, grads, b)
    g = [x.copy() for x in grads]
    g[1][0, 0, 0] += 10 * (1e-3 * abs(grads[1][0, 0, 0]) + 2e-5 * np.abs(grads[1]).max())  # no bound on b
    with pytest.raises(AssertionError, match="bar"):
        _run(color, depth, g, color, depth, grads, b)


def test_flagged_pixels_lie_in_their_flip_interval():
    color, depth, grads, b = _case()
    b = dict(b, pflag=b["pflag"].copy(), pix_rad=b["pix_rad"].copy())
    b["pflag"][3, 4] = 1
    b["pix_rad"][3, 4] = 0.004
    c = color.copy()
    c[:, 3, 4] += 0.004                           # the flipped splat's weight: inside its interval
    _run(c, depth, grads, color, depth, grads, b)
    c[1, 3, 4] += 0.04                            # 10x it fails
    with pytest.raises(AssertionError, match="colour: a flagged pixel"):
        _run(c, depth, grads, color, depth, grads, b)


def test_flagged_shares_are_capped():
    color, depth, grads, b = _case()
    b = _flagged(b, slice(0, 100), 0.0)           # 10 % of the Gaussians flagged: over the cap
    with pytest.raises(AssertionError, match="Gaussians flagged"):
        _run(color, depth, grads, color, depth, grads, b)
