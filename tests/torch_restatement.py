"""Independent float64 autograd restatement of the rasterizer forward (test infrastructure).

Used to cross-check the C oracle's hand-derived backward (backward.cu restated) against automatic
differentiation of the forward math (forward.cu restated in plain matrix form, NOT the glm
column-major transcription), on small scenes chosen so that none of the reference's
non-differentiable quirks (SURVEY §8 a-Q17 alpha clamp, Q22 cov clamp, Q26 scale modifier) is
active.  Per-pixel blending is vectorised over padded per-tile lists taken from the oracle's sort.
"""
import math

import numpy as np
import torch

SH_C0 = 0.28209479177387814
SH_C1 = 0.4886025119029199
SH_C2 = [1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792, 0.5462742152960396]
SH_C3 = [-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154, -0.4570457994644658,
         1.445305721320277, -0.5900435899266435]


def eval_sh_torch(deg, sh, d):
    """sh (P,K,3), d (P,3) unit -> (P,3); same polynomial as forward.cu:20-62."""
    x, y, z = d[:, 0:1], d[:, 1:2], d[:, 2:3]
    r = SH_C0 * sh[:, 0]
    if deg > 0:
        r = r - SH_C1 * y * sh[:, 1] + SH_C1 * z * sh[:, 2] - SH_C1 * x * sh[:, 3]
    if deg > 1:
        xx, yy, zz, xy, yz, xz = x * x, y * y, z * z, x * y, y * z, x * z
        r = (r + SH_C2[0] * xy * sh[:, 4] + SH_C2[1] * yz * sh[:, 5] + SH_C2[2] * (2 * zz - xx - yy) * sh[:, 6]
             + SH_C2[3] * xz * sh[:, 7] + SH_C2[4] * (xx - yy) * sh[:, 8])
    if deg > 2:
        r = (r + SH_C3[0] * y * (3 * xx - yy) * sh[:, 9] + SH_C3[1] * xy * z * sh[:, 10]
             + SH_C3[2] * y * (4 * zz - xx - yy) * sh[:, 11] + SH_C3[3] * z * (2 * zz - 3 * xx - 3 * yy) * sh[:, 12]
             + SH_C3[4] * x * (4 * zz - xx - yy) * sh[:, 13] + SH_C3[5] * z * (xx - yy) * sh[:, 14]
             + SH_C3[6] * x * (xx - 3 * yy) * sh[:, 15])
    return r


def quat_to_rot(q):
    """Standard rotation matrix of an (r,x,y,z) quaternion used as-is (no normalisation, forward.cu:127)."""
    r, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    R = torch.stack([
        1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y),
        2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x),
        2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)], 1).reshape(-1, 3, 3)
    return R


def forward_autograd(scene, point_list, ranges, degree, use_precomp_colors=False, colors=None):
    """Differentiable float64 forward.  Returns dict of outputs and leaf tensors.

    scene: numpy arrays (means3D, scales, rotations, opacities, shs, bg, viewmatrix, projmatrix,
    campos, tanfovx, tanfovy, W, H).  point_list/ranges: the oracle's sorted per-tile lists.
    """
    dt = torch.float64
    means = torch.tensor(scene["means3D"], dtype=dt, requires_grad=True)
    scales = torch.tensor(scene["scales"], dtype=dt, requires_grad=True)
    rots = torch.tensor(scene["rotations"], dtype=dt, requires_grad=True)
    opac = torch.tensor(scene["opacities"], dtype=dt, requires_grad=True)
    shs = torch.tensor(scene["shs"], dtype=dt, requires_grad=True)
    V = torch.tensor(scene["viewmatrix"], dtype=dt).reshape(4, 4)   # flat column-major -> p_h @ V
    Pm = torch.tensor(scene["projmatrix"], dtype=dt).reshape(4, 4)
    campos = torch.tensor(scene["campos"], dtype=dt)
    W, H = scene["W"], scene["H"]
    tfx, tfy = scene["tanfovx"], scene["tanfovy"]
    fx, fy = W / (2 * tfx), H / (2 * tfy)
    P = means.shape[0]

    ph = torch.cat([means, torch.ones(P, 1, dtype=dt)], 1)
    phom = ph @ Pm
    pw = 1.0 / (phom[:, 3:4] + 1e-7)
    ndc_off = torch.zeros(P, 2, dtype=dt, requires_grad=True)          # screenspace_points trick
    ndc = phom[:, :2] * pw + ndc_off
    pix = ((ndc + 1) * torch.tensor([W, H], dtype=dt) - 1) * 0.5
    t = (ph @ V)[:, :3]

    R = quat_to_rot(rots)
    S2 = torch.diag_embed(scales * scales)
    cov3 = R @ S2 @ R.transpose(1, 2)
    cov3.retain_grad()
    Rv = V[:3, :3].T                                                     # rotation part of the view transform
    tz = t[:, 2]
    J = torch.zeros(P, 3, 3, dtype=dt)
    J[:, 0, 0] = fx / tz
    J[:, 0, 2] = -fx * t[:, 0] / tz ** 2
    J[:, 1, 1] = fy / tz
    J[:, 1, 2] = -fy * t[:, 1] / tz ** 2
    Tm = J @ Rv
    cov2 = Tm @ cov3 @ Tm.transpose(1, 2)
    a = cov2[:, 0, 0] + 0.3
    b = cov2[:, 0, 1]
    c = cov2[:, 1, 1] + 0.3
    det = a * c - b * b
    conic = torch.stack([c / det, -b / det, a / det], 1)

    if use_precomp_colors:
        rgb = torch.tensor(colors, dtype=dt, requires_grad=True)
        rgb_leaf = rgb
    else:
        d = means - campos
        d = d / d.norm(dim=1, keepdim=True)
        rgb = torch.clamp_min(eval_sh_torch(degree, shs, d) + 0.5, 0.0)
        rgb_leaf = None
    rgb.retain_grad() if rgb_leaf is None else None

    # per-pixel padded lists
    gx, gy = (W + 15) // 16, (H + 15) // 16
    ys, xs = torch.meshgrid(torch.arange(H), torch.arange(W), indexing="ij")
    tile = (ys // 16) * gx + (xs // 16)
    lens = ranges[:, 1].astype(np.int64) - ranges[:, 0].astype(np.int64)
    K = max(int(lens.max()) if lens.size else 0, 1)
    idx = np.zeros((gx * gy, K), np.int64)
    valid = np.zeros((gx * gy, K), bool)
    for ti in range(gx * gy):
        s, e = int(ranges[ti, 0]), int(ranges[ti, 1])
        idx[ti, :e - s] = point_list[s:e]
        valid[ti, :e - s] = True
    idx_t = torch.from_numpy(idx)[tile.reshape(-1)]          # (Npix, K)
    val_t = torch.from_numpy(valid)[tile.reshape(-1)]
    pxf = xs.reshape(-1, 1).to(dt)
    pyf = ys.reshape(-1, 1).to(dt)
    dx = pix[idx_t, 0] - pxf
    dy = pix[idx_t, 1] - pyf
    co = conic[idx_t]
    power = -0.5 * (co[..., 0] * dx * dx + co[..., 2] * dy * dy) - co[..., 1] * dx * dy
    alpha = opac[idx_t, 0] * torch.exp(power)
    contrib = val_t & (power <= 0) & (alpha >= 1.0 / 255.0) & (alpha <= 0.99)
    a_m = torch.where(contrib, alpha, torch.zeros_like(alpha))
    Tcum = torch.cumprod(torch.cat([torch.ones(a_m.shape[0], 1, dtype=dt), 1 - a_m], 1), 1)
    Tbefore, Tfinal = Tcum[:, :-1], Tcum[:, -1]
    w = a_m * Tbefore
    col = (w.unsqueeze(-1) * rgb[idx_t]).sum(1) + Tfinal.unsqueeze(-1) * torch.tensor(scene["bg"], dtype=dt)
    depth = (w * t[idx_t, 2]).sum(1)
    # discrete checks the caller can compare with the oracle
    alpha_np = alpha.detach().numpy()
    near = val_t.numpy() & (power.detach().numpy() <= 0) & (np.abs(alpha_np - 1.0 / 255.0) < 1e-8)
    pos = np.arange(K)[None, :] + 1
    ncontrib = np.where(contrib.numpy(), pos, 0).max(1)
    return dict(color=col.T.reshape(3, H, W), depth=depth.reshape(1, H, W), Tfinal=Tfinal.reshape(H, W),
                means=means, scales=scales, rots=rots, opac=opac, shs=shs, ndc_off=ndc_off, rgb=rgb, cov3=cov3,
                n_contrib=ncontrib.reshape(H, W), near_threshold=int(near.sum()), clamp099=int(
                    (val_t & (alpha > 0.99)).sum()), min_T=float(Tfinal.detach().min()))
