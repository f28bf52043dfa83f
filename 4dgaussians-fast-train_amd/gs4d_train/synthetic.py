"""Seeded synthetic scenes of BASELINE.md §2 / SURVEY.md §8(d).

One generator serves the parity tests, the fixtures, smoke() and bench.py, so every leg sees the
same bytes for a given (P, W, H, seed).  Draw order is fixed: z, x, y, scales, rotations,
opacities, SH DC, SH rest; the upstream image gradient uses its own generator (seed + 1).
"""
import math

import numpy as np

from .camera import Camera

SH_C0 = 0.28209479177387814

# name -> (P, W, H): the BASELINE.json configs that the rasterizer benchmark/parity tests use
CONFIGS = {
    "c1_plumbing": (20_000, 400, 400),
    "c2_800": (100_000, 800, 800),
    "metric": (100_000, 1352, 1014),
    "c4_per_view": (300_000, 1352, 1014),
    "c5_broom": (1_000_000, 960, 536),
}


def make_camera(W, H, fovx_deg=60.0, R=None, T=None, time=0.0):
    fovx = math.radians(fovx_deg)
    fovy = 2.0 * math.atan(math.tan(fovx / 2.0) * H / W)
    R = np.eye(3) if R is None else R
    T = np.zeros(3) if T is None else T
    return Camera(R, T, fovx, fovy, W, H, time=time)


def make_scene(P, W, H, seed=0, sh_degree=3, z_range=(2.0, 10.0), spread=1.1, log_scale=math.log(0.02),
               log_scale_sigma=0.5):
    """Return a dict of float32 numpy arrays + camera settings for one view."""
    cam = make_camera(W, H)
    rng = np.random.default_rng(seed)
    tx, ty = cam.tanfovx, cam.tanfovy
    z = rng.uniform(z_range[0], z_range[1], P)
    x = rng.uniform(-spread, spread, P) * z * tx
    y = rng.uniform(-spread, spread, P) * z * ty
    means3D = np.stack([x, y, z], 1).astype(np.float32)
    scales = np.exp(rng.normal(log_scale, log_scale_sigma, (P, 3))).astype(np.float32)
    q = rng.normal(0, 1, (P, 4))
    rotations = (q / np.linalg.norm(q, axis=1, keepdims=True)).astype(np.float32)
    opacities = (1.0 / (1.0 + np.exp(-rng.normal(0, 1, (P, 1))))).astype(np.float32)
    K = (sh_degree + 1) ** 2
    shs = np.zeros((P, 16 if sh_degree <= 3 else K, 3), np.float32)
    shs[:, 0, :] = (rng.uniform(0, 1, (P, 3)) - 0.5) / SH_C0
    shs[:, 1:, :] = rng.normal(0, 0.1, (P, shs.shape[1] - 1, 3))
    return dict(
        means3D=means3D, scales=scales, rotations=rotations, opacities=opacities, shs=shs.astype(np.float32),
        bg=np.ones(3, np.float32), viewmatrix=cam.world_view_transform.numpy().astype(np.float32),
        projmatrix=cam.full_proj_transform.numpy().astype(np.float32),
        campos=cam.camera_center.numpy().astype(np.float32), tanfovx=cam.tanfovx, tanfovy=cam.tanfovy,
        W=W, H=H, sh_degree=sh_degree, scale_modifier=1.0, camera=cam)


def make_upstream_grad(color, seed=1):
    """L1 gradient of train.py:244 against a uniform-random ground truth: sign(color-gt)/(3HW)."""
    C, H, W = color.shape
    gt = np.random.default_rng(seed).uniform(0, 1, (C, H, W)).astype(np.float32)
    return (np.sign(color - gt) / (C * H * W)).astype(np.float32), gt


def make_training_views(n_views, W, H, seed=0, time_range=(0.0, 1.0), radius=4.0, device="cuda"):
    """Cameras on an arc looking at the origin, one timestamp per view, with uniform-random ground
    truth images (3, H, W) -- synthetic data of the metric's shape (no dataset is available here)."""
    import torch
    rng = np.random.default_rng(seed)
    views = []
    for v in range(n_views):
        a = 2 * math.pi * v / max(1, n_views) * 0.25
        # world->camera rotation looking at the origin from (r sin a, 0, -r cos a)
        c = np.array([radius * math.sin(a), 0.0, -radius * math.cos(a)])
        fwd = -c / np.linalg.norm(c)
        right = np.cross(np.array([0.0, 1.0, 0.0]), fwd)
        right /= np.linalg.norm(right)
        up = np.cross(fwd, right)
        Rw2c = np.stack([right, up, fwd], 0)       # rows: camera axes in world
        R = Rw2c.T                                 # the reference stores R transposed (getWorld2View2)
        T = -Rw2c @ c
        t = time_range[0] + (time_range[1] - time_range[0]) * (v / max(1, n_views - 1) if n_views > 1 else 0.0)
        cam = make_camera(W, H, R=R, T=T, time=t)
        gt = torch.tensor(rng.uniform(0, 1, (3, H, W)).astype(np.float32), device=device)
        views.append((cam, gt))
    return views


def make_train_like_scene(P, W, H, seed=0, extent=1.2, radius=4.0):
    """The rasterizer's input at the start of a training run (a bench workload next to the metric
    scene): `make_point_cloud` initialised as `GaussianModel.create_from_pcd` does
    (scene/gaussian_model.py:134-163) -- scales sqrt(3-NN mean squared distance) on every axis (the
    simple_knn value, here from a k-d tree), identity rotations, opacity 0.1, SH DC from the colours,
    the rest zero -- seen by view 0 of `make_training_views` (radius 4, looking at the origin).
    Its splats are larger than the metric scene's: ~1,200 instances per touched tile."""
    from scipy.spatial import cKDTree
    pts, cols = make_point_cloud(P, seed=seed, extent=extent)
    d, _ = cKDTree(pts.astype(np.float64)).query(pts.astype(np.float64), k=4)
    dist2 = np.maximum((d[:, 1:] ** 2).mean(1), 1e-7)
    scales = np.repeat(np.sqrt(dist2)[:, None], 3, 1).astype(np.float32)
    rotations = np.zeros((P, 4), np.float32)
    rotations[:, 0] = 1.0
    opacities = np.full((P, 1), 0.1, np.float32)
    shs = np.zeros((P, 16, 3), np.float32)
    shs[:, 0, :] = (cols - 0.5) / SH_C0
    c = np.array([0.0, 0.0, -radius])
    Rw2c = np.eye(3)          # view 0 of make_training_views: camera axes = world axes
    cam = make_camera(W, H, R=Rw2c.T, T=-Rw2c @ c)
    return dict(
        means3D=pts, scales=scales, rotations=rotations, opacities=opacities, shs=shs,
        bg=np.ones(3, np.float32), viewmatrix=cam.world_view_transform.numpy().astype(np.float32),
        projmatrix=cam.full_proj_transform.numpy().astype(np.float32),
        campos=cam.camera_center.numpy().astype(np.float32), tanfovx=cam.tanfovx, tanfovy=cam.tanfovy,
        W=W, H=H, sh_degree=3, scale_modifier=1.0, camera=cam)


def make_point_cloud(P, seed=0, extent=1.2):
    """Random initial point cloud inside the deformation field's bounds, with random colours."""
    rng = np.random.default_rng(seed)
    pts = rng.uniform(-extent, extent, (P, 3)).astype(np.float32)
    cols = rng.uniform(0, 1, (P, 3)).astype(np.float32)
    return pts, cols


# ---- a synthetic dynamic scene (the stand-in for D-NeRF bouncingballs in the convergence test) ----------
def look_at_camera(W, H, center, target=(0.0, 0.0, 0.0), time=0.0, fovx_deg=60.0):
    """A Camera at `center` looking at `target` (world y up), in the reference's R/T convention
    (R = world->camera rotation transposed, T = translation; scene/cameras.py, getWorld2View2)."""
    c = np.asarray(center, np.float64)
    fwd = np.asarray(target, np.float64) - c
    fwd /= np.linalg.norm(fwd)
    right = np.cross(np.array([0.0, 1.0, 0.0]), fwd)
    right /= np.linalg.norm(right)
    up = np.cross(fwd, right)
    Rw2c = np.stack([right, up, fwd], 0)
    return make_camera(W, H, fovx_deg=fovx_deg, R=Rw2c.T, T=-Rw2c @ c, time=time)


def bouncing_balls(n_per_ball=1000, seed=0):
    """Three coloured balls of Gaussians (sphere shells, isotropic splats) and their motion: ball k at
    time t in [0, 1] is centred at base_k + (dx_k sin(2 pi t), h_k |sin(pi (t + phase_k))|, 0).
    Returns (canonical dict of float32 arrays, a function t -> means3D at time t)."""
    rng = np.random.default_rng(seed)
    bases = np.array([[-0.6, -0.5, 0.0], [0.5, -0.5, 0.3], [0.0, -0.5, -0.5]])
    amp = np.array([[0.3, 0.8], [0.25, 0.6], [0.35, 0.9]])
    phase = np.array([0.0, 0.33, 0.66])
    colors = np.array([[0.9, 0.15, 0.1], [0.1, 0.7, 0.2], [0.15, 0.3, 0.9]])
    radius = 0.3
    pts, cols, owner = [], [], []
    for k in range(3):
        d = rng.normal(size=(n_per_ball, 3))
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        pts.append(d * radius)
        cols.append(np.clip(colors[k] + rng.normal(0, 0.05, (n_per_ball, 3)), 0, 1))
        owner.append(np.full(n_per_ball, k))
    local, cols, owner = np.concatenate(pts), np.concatenate(cols), np.concatenate(owner)
    P = local.shape[0]
    shs = np.zeros((P, 16, 3), np.float32)
    shs[:, 0, :] = (cols - 0.5) / SH_C0
    rot = np.zeros((P, 4), np.float32)
    rot[:, 0] = 1.0
    canon = dict(scales=np.full((P, 3), 0.045, np.float32), rotations=rot,
                 opacities=np.full((P, 1), 0.95, np.float32), shs=shs)

    def means_at(t):
        off = np.stack([amp[:, 0] * np.sin(2 * np.pi * t), amp[:, 1] * np.abs(np.sin(np.pi * (t + phase))),
                        np.zeros(3)], 1)
        return (local + bases[owner] + off[owner]).astype(np.float32)
    return canon, means_at
