"""Parity bars of the HIP rasterizer against the CPU oracle, shared by tests/ and __graft_entry__.smoke().

TEST INFRASTRUCTURE ONLY (like oracle.py): the product package never imports it.

Tolerances (north_star): RGB within 1e-4, depth within 1e-4 of the depth range, gradients within 1e-3.
The blend has two discrete thresholds, alpha >= 1/255 and T(1 - alpha) >= 1e-4 (forward.cu:346-354,
backward.cu:486-503); two correct float implementations (exp2/FMA on gfx950 against the oracle's
libm/no-FMA arithmetic) can land on either side when the operand lies within rounding of the threshold.
`oracle.flip_bounds` finds every decision whose operand lies within FLIP_BAND_ALPHA / FLIP_BAND_T
(relative) of its threshold -- bands set at twice the largest operand difference measured between the
blend kernels and the oracle (tests/test_gpu_parity.py::test_flip_bands_cover_measured_operands) -- replays
each one the other way, and returns per pixel and per gradient ELEMENT the largest change those flips can
make (the interval the HIP result may lie in around the oracle's).

Bars, as asserted by `check`:
  pixels               colour and depth (relative to max(1, max depth)) within IMG_ATOL and IMG_SHARP
                       (measured maxima over the GPU suite: 1.5e-6 colour, 7.9e-7 depth, so a 10x
                       regression fails) of the oracle, widened by the pixel's flip bound (zero for the
                       pixels without a near-threshold decision)
  gradient elements    every element within GRAD_RTOL |ref| + GRAD_FLOOR max|ref| of its tensor (a relative
                       bar with a floor for elements that are sums of cancelling terms; measured at most 0.41
                       of it), and within GRAD_SHARP of the tensor's max (measured <= 2.1e-5), both widened by
                       the element's flip bound (zero for the Gaussians no flip touches)
  flagged shares       at most `pix_frac` of the pixels and `gauss_frac` of the Gaussians hold a near-threshold
                       decision (a Gaussian counts when its OWN alpha or termination test at some pixel is near
                       the threshold)
"""
import numpy as np

IMG_ATOL = 1e-4
IMG_SHARP = 1e-5
GRAD_RTOL = 1e-3
GRAD_FLOOR = 2e-5
GRAD_SHARP = 1e-4
# twice the largest operand differences measured between the blend kernels and the oracle
# (test_flip_bands_cover_measured_operands, round 5).  Alpha: |255 alpha_gpu - 255 alpha_oracle| reaches 1.4e-4
# where the power's terms cancel (splats elongated along the pixel's offset), so the band is per unit of the
# pair's magnitude factor (oracle near_alpha: 1 + the power's terms' magnitudes): measured at most 2.31e-7 per
# unit (metric; C2 1.98e-7, train-like 2.24e-7, opaque stack 1.27e-7), about two roundings of the terms.
# T(1 - alpha) relative: at most 1.75e-5 (C2; metric 6.4e-6, train-like 2.5e-6).
FLIP_BAND_ALPHA = 5e-7
FLIP_BAND_T = 4e-5
# caps on the shares holding a near-threshold decision, about twice the measured maxima with the bands above
# (round 5): pixels 7.7e-4 (C4), Gaussians 6.7e-3 (a 2304x1296 scene; metric 5.7e-3, C2 1.2e-3, C4 3.4e-3,
# C5 3.6e-4); scenes above these carry their own caps in tests/test_gpu_parity.py
FLIP_PIX_FRAC = 2e-3
FLIP_GAUSS_FRAC = 1.2e-2

GRAD_NAMES = ["dL_dmeans2D", "dL_dcolors", "dL_dopacity", "dL_dmeans3D", "dL_dcov3D", "dL_dsh", "dL_dscales",
              "dL_drotations"]


def _split_max(err, flagged):
    err = np.asarray(err).reshape(-1)
    flagged = np.asarray(flagged).reshape(-1)
    unf, fl = err[~flagged], err[flagged]
    return (float(unf.max()) if unf.size else 0.0), (float(fl.max()) if fl.size else 0.0)


def grad_report(a, b, rad, gflag):
    """For one gradient tensor (rows = Gaussians) against the oracle's b with flip bounds rad:
    (max over unflagged Gaussians of (|a - b| - rad) / max|b|, the same over flagged ones, the largest
    ratio |a - b| / (rad + GRAD_RTOL |b| + GRAD_FLOOR max|b|) over all elements (<= 1 passes), the largest
    share of its flip bound a flagged element uses, |a - b| / rad)."""
    n = len(gflag)
    a = np.asarray(a, np.float64).reshape(n, -1)
    b = np.asarray(b, np.float64).reshape(n, -1)
    rad = np.zeros_like(b) if rad is None else np.asarray(rad, np.float64).reshape(n, -1)
    if a.size == 0:
        return 0.0, 0.0, 0.0, 0.0
    scale = max(float(np.abs(b).max()), 1e-30)
    err = np.abs(a - b)
    ratio = err / (rad + GRAD_RTOL * np.abs(b) + GRAD_FLOOR * scale)
    excess = np.maximum(err - rad, 0.0) / scale
    fl = np.asarray(gflag, bool)
    unf_norm, fl_norm = _split_max(excess.max(1), fl)
    used = np.where(rad > 0, err / np.maximum(rad, 1e-300), 0.0)
    return unf_norm, fl_norm, float(ratio.max()), float(used[fl].max()) if fl.any() else 0.0


def check(color, depth, grads, o_color, o_depth, o_grads, bounds, o_rads=None, pix_frac=FLIP_PIX_FRAC,
          gauss_frac=FLIP_GAUSS_FRAC, names=GRAD_NAMES):
    """Assert the bars above; returns the report (printed by the callers, so every config's measured
    maxima are in the log).  color (3, H, W), depth (1, H, W) or (H, W), grads / o_grads: sequences aligned
    with `names`; bounds: oracle.flip_bounds' dict; o_rads: the flip bounds aligned with o_grads (default
    bounds["grad_rad"], which is aligned with rasterize_backward's outputs)."""
    pflag, gflag = np.asarray(bounds["pflag"]), np.asarray(bounds["gflag"])
    o_rads = bounds["grad_rad"] if o_rads is None else o_rads
    flagged = pflag != 0
    gfl = gflag != 0
    # images in float32 (the difference of two nearby floats is exact; a 2^28-pixel case stays in memory)
    cerr = np.abs(np.asarray(color, np.float32) - np.asarray(o_color, np.float32)).max(0)
    derr = np.abs(np.asarray(depth, np.float32).reshape(flagged.shape) - np.asarray(o_depth, np.float32).reshape(flagged.shape))
    dscale = max(1.0, float(np.abs(o_depth).max()) if np.size(o_depth) else 1.0)
    c_ex = np.maximum(cerr - np.asarray(bounds["pix_rad"], np.float32), 0)
    d_ex = np.maximum(derr - np.asarray(bounds["depth_rad"], np.float32), 0) / dscale
    P = len(gfl)
    rep = {"flagged_pix_frac": float(flagged.mean()) if flagged.size else 0.0,
           "flagged_gauss_frac": float(gfl.mean()) if P else 0.0,
           "color": _split_max(c_ex, flagged), "depth": _split_max(d_ex, flagged),
           "color_flip_max": float(cerr[flagged].max()) if flagged.any() else 0.0}
    for n, a, b, r in zip(names, grads, o_grads, o_rads):
        a = np.asarray(a)
        assert a.shape == b.shape, f"{n} shape {a.shape} != {b.shape}"
        assert r is None or np.asarray(r).size == b.size, f"{n}: flip bounds of another shape"
        if a.size:
            assert np.isfinite(a).all(), f"{n} has non-finite values"
        rep[n] = grad_report(a, b, r, gfl)
    print({k: (tuple(float(f"{x:.3g}") for x in v) if isinstance(v, tuple) else float(f"{v:.3g}"))
           for k, v in rep.items()}, flush=True)
    assert rep["flagged_pix_frac"] <= pix_frac, f"{rep['flagged_pix_frac']:.2e} of the pixels flagged"
    assert rep["flagged_gauss_frac"] <= gauss_frac, f"{rep['flagged_gauss_frac']:.2e} of the Gaussians flagged"
    for what, (u, f) in (("colour", rep["color"]), ("depth", rep["depth"])):
        assert u <= IMG_ATOL and u <= IMG_SHARP, f"{what}: a pixel off by {u:.3e} (no near-threshold decision)"
        assert f <= IMG_SHARP, f"{what}: a flagged pixel off by {f:.3e} beyond its flip bound"
    for n in names[:len(o_grads)]:
        unf, fl, ratio, _ = rep[n]
        assert ratio <= 1.0, f"{n}: an element off by {ratio:.2f}x its bar (flip bound + 1e-3 |ref| + 2e-5 max|ref|)"
        assert unf <= GRAD_SHARP, f"{n}: an unflagged Gaussian off by {unf:.3e} of the tensor's max"
        assert fl <= GRAD_SHARP, f"{n}: a flagged Gaussian off by {fl:.3e} of the tensor's max beyond its flip bound"
    return rep
