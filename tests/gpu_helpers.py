"""Shared helpers for the GPU parity tests: run the HIP `_C` path and the CPU oracle on the same scene."""
import numpy as np
import torch


def to_dev(s, dev):
    t = lambda a: torch.tensor(np.asarray(a), device=dev)
    return dict(bg=t(s["bg"]), means3D=t(s["means3D"]), opacities=t(s["opacities"]), scales=t(s["scales"]),
                rotations=t(s["rotations"]), shs=t(s["shs"]), viewmatrix=t(s["viewmatrix"]),
                projmatrix=t(s["projmatrix"]), campos=t(s["campos"]))


def c_forward(C, s, d, colors=None, cov3D=None, use_sh=True, degree=None, prefiltered=False, debug=False):
    e = torch.empty(0, device=d["means3D"].device)
    return C.rasterize_gaussians(
        d["bg"], d["means3D"], e if colors is None else colors, d["opacities"],
        e if cov3D is not None else d["scales"], e if cov3D is not None else d["rotations"], float(s["scale_modifier"]),
        e if cov3D is None else cov3D, d["viewmatrix"], d["projmatrix"], float(s["tanfovx"]), float(s["tanfovy"]),
        int(s["H"]), int(s["W"]), d["shs"] if use_sh else e, int(s["sh_degree"] if degree is None else degree),
        d["campos"], prefiltered, debug)


def c_backward(C, s, d, fwd, grad, colors=None, cov3D=None, use_sh=True, degree=None, debug=False):
    e = torch.empty(0, device=d["means3D"].device)
    nr, color, depth, radii, gb, bb, ib = fwd
    return C.rasterize_gaussians_backward(
        d["bg"], d["means3D"], radii, e if colors is None else colors, e if cov3D is not None else d["scales"],
        e if cov3D is not None else d["rotations"], float(s["scale_modifier"]), e if cov3D is None else cov3D,
        d["viewmatrix"], d["projmatrix"], float(s["tanfovx"]), float(s["tanfovy"]), grad, d["shs"] if use_sh else e,
        int(s["sh_degree"] if degree is None else degree), d["campos"], gb, nr, bb, ib, debug)


def o_forward(O, s, colors=None, cov3D=None, use_sh=True, degree=None, prefiltered=False):
    return O.rasterize_forward(
        s["bg"], s["means3D"], colors, s["opacities"], None if cov3D is not None else s["scales"],
        None if cov3D is not None else s["rotations"], s["scale_modifier"], cov3D, s["viewmatrix"], s["projmatrix"],
        s["tanfovx"], s["tanfovy"], s["H"], s["W"], s["shs"] if use_sh else None,
        s["sh_degree"] if degree is None else degree, s["campos"], prefiltered)


def o_backward(O, s, st, radii, grad, colors=None, cov3D=None, use_sh=True, degree=None):
    return O.rasterize_backward(
        st, s["bg"], s["means3D"], radii, colors, None if cov3D is not None else s["scales"],
        None if cov3D is not None else s["rotations"], s["scale_modifier"], cov3D, s["viewmatrix"], s["projmatrix"],
        s["tanfovx"], s["tanfovy"], grad, s["shs"] if use_sh else None, s["sh_degree"] if degree is None else degree,
        s["campos"])[0]


def o_bounds(O, s, st, radii, grad, colors=None, cov3D=None, use_sh=True, degree=None):
    """oracle.flip_bounds for the scene (near-threshold flags and the per-pixel / per-element flip bounds the
    parity bars widen by); an all-culled scene (no oracle state) has none."""
    from oracle import parity as PAR
    if st is None:
        P, H, W = len(radii), s["H"], s["W"]
        M = np.asarray(s["shs"]).shape[1] if use_sh else 0
        z = np.zeros
        return dict(pflag=z((H, W), np.uint8), gflag=z(P, np.uint8), pix_rad=z((H, W), np.float32),
                    depth_rad=z((H, W), np.float32),
                    grad_rad=(z((P, 3)), z((P, 3)), z((P, 1)), z((P, 3)), z((P, 6)), z((P, M, 3)), z((P, 3)), z((P, 4))))
    return O.flip_bounds(
        st, PAR.FLIP_BAND_ALPHA, PAR.FLIP_BAND_T, s["bg"], s["means3D"], radii, colors,
        None if cov3D is not None else s["scales"], None if cov3D is not None else s["rotations"], s["scale_modifier"],
        cov3D, s["viewmatrix"], s["projmatrix"], s["tanfovx"], s["tanfovy"], grad, s["shs"] if use_sh else None,
        s["sh_degree"] if degree is None else degree, s["campos"])


def image_parity(a, b, atol=1e-4):
    """(max abs error, fraction of elements above atol)."""
    err = np.abs(np.asarray(a, np.float64) - np.asarray(b, np.float64))
    return float(err.max()) if err.size else 0.0, float((err > atol).mean()) if err.size else 0.0


def grad_errors(a, b):
    """Per-Gaussian max error normalised by the oracle tensor's max magnitude, shape (P,)."""
    a = np.asarray(a, np.float64).reshape(a.shape[0], -1)
    b = np.asarray(b, np.float64).reshape(b.shape[0], -1)
    if a.size == 0:
        return np.zeros(a.shape[0])
    return np.abs(a - b).max(1) / max(np.abs(b).max(), 1e-30)


def split_max(err, flagged):
    """(max of err over unflagged elements, max over flagged ones); 0 for an empty set."""
    err = np.asarray(err).reshape(-1)
    flagged = np.asarray(flagged).reshape(-1)
    unf, fl = err[~flagged], err[flagged]
    return (float(unf.max()) if unf.size else 0.0), (float(fl.max()) if fl.size else 0.0)


def grad_parity(a, b, rtol=1e-3):
    """Per-Gaussian relative error normalised by the tensor's max magnitude.

    Returns (max normalised error, fraction of Gaussians whose normalised error exceeds rtol).  Rare
    discrete threshold flips (alpha vs 1/255, T vs 1e-4 in forward.cu:347,350) move single Gaussians;
    everything else must agree to rtol."""
    a = np.asarray(a, np.float64).reshape(a.shape[0], -1)
    b = np.asarray(b, np.float64).reshape(b.shape[0], -1)
    if a.size == 0:
        return 0.0, 0.0
    scale = max(np.abs(b).max(), 1e-30)
    e = np.abs(a - b).max(1) / scale if a.size else np.zeros(0)
    return (float(e.max()) if e.size else 0.0), (float((e > rtol).mean()) if e.size else 0.0)
