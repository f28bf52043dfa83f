"""Pins the CPU oracle (oracle/gs4d_oracle.c) before it is trusted as the parity reference.

Evidence, strongest first:
  1. vectors produced by RUNNING the reference's own Python (tests/golden/make_reference_vectors.py):
     utils/sh_utils.eval_sh and utils/graphics_utils camera matrices;
  2. an independent float64 autograd restatement of the forward (tests/torch_restatement.py)
     against the oracle's hand-derived backward (backward.cu restated);
  3. hand-derived known-answer tests for the discrete rules of forward.cu / backward.cu.
The CUDA reference itself cannot be built here, so everything beyond (1) is
"parity unpinned by reference outputs" and is cross-validated instead.
"""
import math
import os

import numpy as np
import pytest
import torch

from gs4d_train.camera import Camera
from gs4d_train.synthetic import make_scene, make_upstream_grad

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _fwd(O, s, colors=None, cov3D=None, sh=True, prefiltered=False, degree=None):
    return O.rasterize_forward(
        s["bg"], s["means3D"], colors, s["opacities"], None if cov3D is not None else s["scales"],
        None if cov3D is not None else s["rotations"], s["scale_modifier"], cov3D, s["viewmatrix"],
        s["projmatrix"], s["tanfovx"], s["tanfovy"], s["H"], s["W"], s["shs"] if sh else None,
        s["sh_degree"] if degree is None else degree, s["campos"], prefiltered)


def _bwd(O, s, st, radii, g, colors=None, cov3D=None, sh=True, degree=None):
    return O.rasterize_backward(
        st, s["bg"], s["means3D"], radii, colors, None if cov3D is not None else s["scales"],
        None if cov3D is not None else s["rotations"], s["scale_modifier"], cov3D, s["viewmatrix"],
        s["projmatrix"], s["tanfovx"], s["tanfovy"], g, s["shs"] if sh else None,
        s["sh_degree"] if degree is None else degree, s["campos"])


# ---------------------------------------------------------------- (1) reference-produced vectors
def test_sh_matches_reference_eval_sh(oracle):
    v = np.load(os.path.join(GOLD, "ref_sh_vectors.npz"))
    for deg in range(4):
        rgb, cl = oracle.sh_forward(deg, v["means"], v["campos"], v["shs"])
        np.testing.assert_allclose(rgb, v[f"deg{deg}"], rtol=0, atol=2e-6)
        raw = v[f"raw{deg}"] + 0.5
        # clamp flags are exactly "result < 0" (forward.cu:67-69); skip values within rounding of 0
        safe = np.abs(raw) > 1e-5
        assert np.array_equal(((cl[:, None] >> np.arange(3)) & 1).astype(bool)[safe], (raw < 0)[safe])


def test_cov3d_matches_reference_build_covariance(oracle):
    """computeCov3D (forward.cu:118-152, the oracle's cov3d_forward) against the reference's own Python
    covariance (scene/gaussian_model.py:30-34 over utils/general_utils.py build_scaling_rotation /
    strip_symmetric, run by tests/golden/make_reference_vectors.py) for unit quaternions, scale_modifier 1
    and 0.7: the same matrix R S S^T R^T, formed in another order (fp32 rounding)."""
    v = np.load(os.path.join(GOLD, "ref_cov3d_vectors.npz"))
    P = v["scales"].shape[0]
    s = make_scene(P, 64, 48, seed=9)
    s["scales"], s["rotations"] = v["scales"], v["rotations"]
    for tag, mod in (("mod1", 1.0), ("mod07", 0.7)):
        s["scale_modifier"] = mod
        *_, st = _fwd(oracle, s)
        cov = st.export()["cov3D"]  # every Gaussian passes the near-plane test (z in [2, 10])
        ref = v[tag]
        scale = np.abs(ref).max(axis=1, keepdims=True)
        assert np.all(np.abs(cov - ref) <= 2e-6 * scale), float((np.abs(cov - ref) / scale).max())


def test_camera_matches_reference_graphics_utils():
    v = np.load(os.path.join(GOLD, "ref_camera_vectors.npz"))
    for i in range(int(v["n"])):
        cam = Camera(v[f"R_{i}"], v[f"T_{i}"], float(v[f"fovx_{i}"]), float(v[f"fovy_{i}"]), int(v[f"W_{i}"]),
                     int(v[f"H_{i}"]))
        np.testing.assert_allclose(cam.world_view_transform.numpy(), v[f"view_{i}"], atol=1e-6)
        np.testing.assert_allclose(cam.full_proj_transform.numpy(), v[f"proj_{i}"], atol=1e-6)
        np.testing.assert_allclose(cam.camera_center.numpy(), v[f"center_{i}"], atol=1e-5)


# ---------------------------------------------------------------- (2) autograd cross-check
def _small_scene(seed, P=60, W=70, H=45, degree=3, opac_max=0.9):
    s = make_scene(P, W, H, seed=seed, sh_degree=degree, log_scale=math.log(0.08), z_range=(2.0, 6.0))
    s["opacities"] = np.minimum(s["opacities"], opac_max).astype(np.float32)
    return s


@pytest.mark.parametrize("seed,degree,mode", [(0, 3, "sh"), (1, 2, "sh"), (2, 1, "sh"), (3, 0, "sh"),
                                              (4, 3, "colors"), (5, 3, "cov3D")])
def test_oracle_backward_matches_autograd(oracle, seed, degree, mode):
    from torch_restatement import forward_autograd
    s = _small_scene(seed, degree=degree)
    colors = None
    cov3D = None
    if mode == "colors":
        colors = np.random.default_rng(seed + 100).uniform(0, 1, (s["means3D"].shape[0], 3)).astype(np.float32)
    if mode == "cov3D":
        from torch_restatement import quat_to_rot
        R = quat_to_rot(torch.tensor(s["rotations"], dtype=torch.float64)).numpy()
        S2 = s["scales"].astype(np.float64) ** 2
        C = np.einsum("pij,pj,pkj->pik", R, S2, R)
        cov3D = np.stack([C[:, 0, 0], C[:, 0, 1], C[:, 0, 2], C[:, 1, 1], C[:, 1, 2], C[:, 2, 2]], 1).astype(np.float32)
    nr, color, depth, radii, st = _fwd(oracle, s, colors=colors, cov3D=cov3D, sh=mode != "colors")
    ex = st.export()
    ref = forward_autograd(s, ex["point_list"], ex["ranges"], degree, use_precomp_colors=mode == "colors",
                           colors=colors)
    assert ref["clamp099"] == 0 and ref["near_threshold"] == 0 and ref["min_T"] > 1e-3
    assert np.array_equal(ref["n_contrib"], ex["n_contrib"])
    np.testing.assert_allclose(color, ref["color"].detach().numpy(), atol=2e-6)
    np.testing.assert_allclose(depth, ref["depth"].detach().numpy(), atol=2e-5)
    np.testing.assert_allclose(ex["final_T"], ref["Tfinal"].detach().numpy(), atol=2e-6)

    g, _ = make_upstream_grad(color, seed=seed + 1)
    g = g * (3 * s["W"] * s["H"])   # O(1) magnitudes for a relative check
    (ref["color"] * torch.tensor(g, dtype=torch.float64)).sum().backward()
    grads, _ = _bwd(oracle, s, st, radii, g, colors=colors, cov3D=cov3D, sh=mode != "colors")
    dm2, dcol, dop, dm3, dcov, dsh, dsc, drot = grads

    def close(a, b, name, rtol=2e-4):
        b = b.detach().numpy() if torch.is_tensor(b) else b
        scale = max(np.abs(b).max(), 1e-12)
        err = np.abs(a - b).max() / scale
        assert err < rtol, f"{name}: rel err {err:.3e} (scale {scale:.3e})"

    vis = radii > 0
    close(dm2[vis, :2], ref["ndc_off"].grad.numpy()[vis], "dL_dmeans2D")
    close(dop[vis], ref["opac"].grad.numpy()[vis], "dL_dopacity")
    close(dm3[vis], ref["means"].grad.numpy()[vis], "dL_dmeans3D")
    if mode == "colors":
        close(dcol[vis], ref["rgb"].grad.numpy()[vis], "dL_dcolors")
    else:
        close(dcol[vis], ref["rgb"].grad.numpy()[vis], "dL_dcolors")
    if mode == "sh":
        close(dsh[vis], ref["shs"].grad.numpy()[vis], "dL_dsh")
    if mode != "cov3D":
        close(dsc[vis], ref["scales"].grad.numpy()[vis], "dL_dscales")
        close(drot[vis], ref["rots"].grad.numpy()[vis], "dL_drotations")
    gc = ref["cov3"].grad.numpy()
    # reference packs the symmetric gradient as [00, 01+10, 02+20, 11, 12+21, 22] (backward.cu:217-227)
    packed = np.stack([gc[:, 0, 0], gc[:, 0, 1] + gc[:, 1, 0], gc[:, 0, 2] + gc[:, 2, 0], gc[:, 1, 1],
                       gc[:, 1, 2] + gc[:, 2, 1], gc[:, 2, 2]], 1)
    close(dcov[vis], packed[vis], "dL_dcov3D")
    # culled Gaussians get exactly zero gradient (backward.cu:156,367)
    for a in (dm3, dsc, drot, dcov):
        assert not np.any(a[~vis])


# ---------------------------------------------------------------- (3) known-answer tests
def _single(opacity, color, W=33, H=21, scale=0.05, depth=3.0, px=None, py=None):
    cam_s = make_scene(1, W, H, seed=0)
    s = dict(cam_s)
    tx, ty = s["tanfovx"], s["tanfovy"]
    x = 0.0 if px is None else px * depth * tx
    y = 0.0 if py is None else py * depth * ty
    s["means3D"] = np.array([[x, y, depth]], np.float32)
    s["scales"] = np.full((1, 3), scale, np.float32)
    s["rotations"] = np.array([[1, 0, 0, 0]], np.float32)
    s["opacities"] = np.array([[opacity]], np.float32)
    return s, np.array([color], np.float32)


def test_kat_single_gaussian_center(oracle):
    """At the Gaussian's own pixel centre power = 0, so C = c*o + (1-o)*bg (forward.cu:338-376)."""
    W, H = 33, 21
    s, col = _single(0.6, [0.2, 0.5, 0.9], W, H)
    nr, color, depth, radii, st = _fwd(oracle, s, colors=col, sh=False)
    ex = st.export()
    mx, my = ex["means2D"][0]
    assert abs(mx - (W - 1) / 2) < 1e-4 and abs(my - (H - 1) / 2) < 1e-4   # ndc 0 -> ((0+1)W-1)/2
    cx, cy = int(round(mx)), int(round(my))
    assert cx == 16 and cy == 10
    np.testing.assert_allclose(color[:, cy, cx], 0.6 * col[0] + 0.4 * 1.0, atol=1e-6)
    assert abs(depth[0, cy, cx] - 0.6 * 3.0) < 1e-5
    assert ex["n_contrib"][cy, cx] == 1 and abs(ex["final_T"][cy, cx] - 0.4) < 1e-7


def test_kat_alpha_clamp_and_termination(oracle):
    """alpha = min(0.99, o*G) (forward.cu:346) and T*(1-a) < 1e-4 stops blending (:349-354)."""
    s, col = _single(1.0, [1, 0, 0])
    P = 3
    s["means3D"] = np.array([[0, 0, 3.0], [0, 0, 3.5], [0, 0, 4.0]], np.float32)
    s["scales"] = np.full((P, 3), 0.05, np.float32)
    s["rotations"] = np.tile(np.array([[1, 0, 0, 0]], np.float32), (P, 1))
    s["opacities"] = np.array([[1.0], [0.5], [1.0]], np.float32)
    cols = np.array([[1, 0, 0], [0, 1, 0], [0, 0, 1]], np.float32)
    nr, color, depth, radii, st = _fwd(oracle, s, colors=cols, sh=False)
    ex = st.export()
    # centre pixel: a1 = min(0.99, 1.0) -> T = 0.01; a2 = 0.5 -> T = 0.005; a3 = 0.99 would leave
    # T = 5e-5 < 1e-4, so blending stops there and the third splat is NOT blended.
    cy, cx = 10, 16
    f = np.float32
    T1 = f(1.0) * f(f(1) - f(0.99))
    T2 = f(T1 * f(f(1) - f(0.5)))
    assert ex["n_contrib"][cy, cx] == 2
    assert ex["final_T"][cy, cx] == T2
    np.testing.assert_allclose(color[:, cy, cx], [0.99, 0.5 * T1, 0] + T2 * 1.0, atol=1e-6)
    # the backward never revisits the terminating splat; its gradients come only from pixels it
    # actually blended into
    g = np.zeros_like(color)
    g[:, cy, cx] = 1.0
    grads, _ = _bwd(oracle, s, st, radii, g, colors=cols, sh=False)
    dcol = grads[1]
    np.testing.assert_allclose(dcol[:, :], [[0.99, 0.99, 0.99], [0.5 * T1] * 3, [0, 0, 0]], atol=1e-6)


def test_near_plane_cull_and_prefiltered(oracle):
    s, col = _single(0.5, [1, 1, 1])
    s["means3D"] = np.array([[0, 0, 0.2]], np.float32)   # z <= 0.2 is culled (auxiliary.h:154)
    nr, color, depth, radii, st = _fwd(oracle, s, colors=col, sh=False)
    assert nr == 0 and radii[0] == 0
    np.testing.assert_allclose(color, 1.0)               # background only
    with pytest.raises(RuntimeError):
        _fwd(oracle, s, colors=col, sh=False, prefiltered=True)
    assert not oracle.mark_visible(s["means3D"], s["viewmatrix"], s["projmatrix"])[0]
    s["means3D"] = np.array([[0, 0, 0.21]], np.float32)
    assert oracle.mark_visible(s["means3D"], s["viewmatrix"], s["projmatrix"])[0]


def test_empty_and_degenerate(oracle):
    s, col = _single(0.5, [1, 1, 1])
    s0 = dict(s, means3D=np.zeros((0, 3), np.float32), scales=np.zeros((0, 3), np.float32),
              rotations=np.zeros((0, 4), np.float32), opacities=np.zeros((0, 1), np.float32))
    nr, color, depth, radii, st = _fwd(oracle, s0, colors=np.zeros((0, 3), np.float32), sh=False)
    assert nr == 0 and radii.shape == (0,) and not color.any()   # P == 0: outputs stay 0, not bg
    # det == 0 culls (forward.cu:220-221): a non-PSD precomputed cov3D that cancels the +0.3
    nr, color, depth, radii, st = _fwd(oracle, s, colors=col, sh=False,
                                       cov3D=np.array([[-0.3 * (3.0 / 27.5) ** 2, 0, 0, 0.1, 0, 0.1]], np.float32))
    assert radii[0] == 0 or nr > 0   # either culled by det==0 or a valid, non-crashing result


def test_odd_sizes_and_offscreen(oracle):
    """W,H not multiples of 16; Gaussians off-screen are kept (no xy frustum cull) but touch no tile."""
    s = make_scene(300, 37, 29, seed=7)
    s["means3D"][:20, 0] += 100.0     # far off-screen in x
    nr, color, depth, radii, st = _fwd(oracle, s)
    ex = st.export()
    assert ex["ranges"].shape == (3 * 2, 2)
    assert np.all(ex["tiles_touched"][:20] == 0)
    assert nr == int(ex["tiles_touched"].sum())
    # sorted list: per tile ascending depth, ties by Gaussian index (stable sort of rasterizer_impl.cu:304)
    for t in range(6):
        a, b = ex["ranges"][t]
        ids = ex["point_list"][a:b]
        d = ex["depths"][ids].view(np.uint32)
        assert np.all((d[1:] > d[:-1]) | ((d[1:] == d[:-1]) & (ids[1:] > ids[:-1])))


def test_threads_deterministic(oracle):
    s = make_scene(3000, 160, 96, seed=3)
    res = []
    for n in (1, 4):
        oracle.set_threads(n)
        nr, color, depth, radii, st = _fwd(oracle, s)
        g, _ = make_upstream_grad(color)
        grads, _ = _bwd(oracle, s, st, radii, g)
        res.append((color, depth, radii) + tuple(grads))
    oracle.set_threads(os.cpu_count())
    for a, b in zip(*res):
        assert np.array_equal(a, b)


def _flip_bounds(O, s, st, radii, g, band):
    return O.flip_bounds(st, band, 0.0, s["bg"], s["means3D"], radii, None, s["scales"], s["rotations"],
                         s["scale_modifier"], None, s["viewmatrix"], s["projmatrix"], s["tanfovx"], s["tanfovy"], g,
                         s["shs"], s["sh_degree"], s["campos"])


def test_flip_bounds_single_splat_near_threshold(oracle):
    """oracle.flip_bounds on one Gaussian whose alpha at one pixel sits just above 1/255, with the upstream
    gradient on that pixel only: flipping that decision removes exactly that pixel's term, so the K7-level
    bounds (dL_dmeans2D, dL_dcolors, dL_dopacity) equal the magnitudes of the oracle's own gradients, the
    bounds carried through K8 + K9 cover the final gradients, and the pixel's colour bound is the splat's
    whole weight there (forward.cu:346-348 taken the other way)."""
    O = oracle
    s = make_scene(1, 64, 48, seed=3, log_scale=math.log(0.1))
    s["means3D"][0] = (0.0123, 0.0071, 4.0)  # off the pixel grid's symmetry: one near pixel
    n, color, depth, radii, st = _fwd(O, s)
    ex = st.export()
    (mx, my), co = ex["means2D"][0], ex["conic_opacity"][0]
    px, py = int(mx) + 4, int(my) + 2  # a few pixels off the centre
    dx, dy = np.float32(mx - px), np.float32(my - py)
    power = -0.5 * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy
    assert power < -0.5
    for delta in (2e-6, 4e-6, 8e-6):
        s["opacities"][0, 0] = np.float32((1.0 / 255.0) * (1 + delta) / math.exp(float(power)))
        n, color, depth, radii, st = _fwd(O, s)
        if st.export()["n_contrib"][py, px] == 1:  # the oracle blends it (alpha >= 1/255 in its arithmetic)
            break
    else:
        pytest.fail("no opacity put the pixel just above 1/255")
    g = np.zeros((3, s["H"], s["W"]), np.float32)
    g[:, py, px] = (0.3, -0.2, 0.5)
    grads = _bwd(O, s, st, radii, g)[0]
    b = _flip_bounds(O, s, st, radii, g, 1e-4)
    assert b["gflag"][0] == 1 and b["pflag"][py, px] == 1 and b["pflag"].sum() == 1
    rad = b["grad_rad"]
    for i in (0, 1, 2):  # dL_dmeans2D, dL_dcolors, dL_dopacity: the pixel's term itself
        np.testing.assert_allclose(rad[i], np.abs(grads[i]), rtol=1e-6, atol=0)
    assert np.abs(grads[0][0, :2]).min() > 0 and rad[3].max() > 0
    for i in (3, 4, 5, 6, 7):  # carried through K8 + K9: they cover the final gradients
        assert np.all(np.abs(grads[i]) <= rad[i] * (1 + 1e-5) + 1e-12), i
    s0 = dict(s, opacities=np.zeros_like(s["opacities"]))
    _, color0, _, _, _ = _fwd(O, s0)
    np.testing.assert_allclose(b["pix_rad"][py, px], np.abs(color[:, py, px] - color0[:, py, px]).max(), rtol=1e-6)
    # outside the band nothing is flagged and every bound is zero
    b = _flip_bounds(O, s, st, radii, g, 1e-7)
    assert not b["pflag"].any() and not b["gflag"].any() and all(not r.any() for r in b["grad_rad"])
