"""Generate golden vectors by RUNNING the reference's own importable Python (this container only).

The reference's CUDA rasterizer cannot be built here (no nvcc/CUB), so the parts of
the path that exist as runnable reference Python pin the oracle:
  * utils/sh_utils.py:57-112  eval_sh          -> SH -> RGB (forward.cu:20-71 restates the same
                                                   polynomial; the rasterizer adds +0.5 and clamps)
  * utils/graphics_utils.py:38-71 getWorld2View2 / getProjectionMatrix, composed as
    scene/cameras.py:61-66 does  -> viewmatrix / projmatrix / campos handed to the rasterizer.
  * utils/general_utils.py:70-116 build_scaling_rotation / strip_symmetric, composed as
    scene/gaussian_model.py:30-34 build_covariance_from_scaling_rotation does -> the 3D covariance the
    rasterizer's computeCov3D (forward.cu:118-152) forms, for unit quaternions.  These helpers allocate
    with a hard-coded device="cuda"; the script runs them with that allocation redirected to the CPU
    (the only change: the arithmetic is the reference's own).
  * scene/hexplane.py (loaded from its file and run as-is: HexPlaneField, init_grid_param,
    grid_sample_wrapper, interpolate_ms_features) -> the deformation field's features and, through
    autograd, the gradients of the planes and of the points;
  * scene/regulation.py:22-28 compute_plane_smoothness -> the planes' smoothness regulariser;
  * utils/general_utils.py:35-68 get_expon_lr_func -> the learning-rate schedules GaussianModel builds
    (scene/gaussian_model.py training_setup) with the DyNeRF / default hyper-parameters.

Usage (from the repo root, in the build container where /root/reference exists):
    python tests/golden/make_reference_vectors.py
Writes tests/golden/ref_{sh,camera,cov3d,hexplane,lr}_vectors.npz (inputs + outputs).
"""
import math
import os
import sys

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def main():
    sys.path.insert(0, REF)
    from utils.sh_utils import eval_sh  # noqa: E402  (reference code, run as-is)
    from utils.graphics_utils import getWorld2View2, getProjectionMatrix  # noqa: E402

    rng = np.random.default_rng(1234)
    # --- SH vectors: means/campos -> dir; sh (P,16,3) in the rasterizer's layout -------------
    P = 512
    means = rng.normal(0, 3, (P, 3)).astype(np.float32)
    campos = rng.normal(0, 1, 3).astype(np.float32)
    shs = rng.normal(0, 0.5, (P, 16, 3)).astype(np.float32)
    rgb = {}
    for deg in range(4):
        d = torch.from_numpy(means) - torch.from_numpy(campos)
        d = d / d.norm(dim=1, keepdim=True)
        # gaussian_renderer/__init__.py:106-110 layout: (P, 3, K)
        sh_view = torch.from_numpy(shs).transpose(1, 2).contiguous()
        val = eval_sh(deg, sh_view, d)
        rgb[f"deg{deg}"] = torch.clamp_min(val + 0.5, 0.0).numpy().astype(np.float32)
        rgb[f"raw{deg}"] = val.numpy().astype(np.float32)
    np.savez_compressed(os.path.join(OUT, "ref_sh_vectors.npz"), means=means, campos=campos, shs=shs, **rgb)

    # --- camera vectors ---------------------------------------------------------------------
    cams = []
    for i in range(6):
        W, H = [(400, 400), (800, 800), (1352, 1014), (960, 536), (97, 61), (1352, 1014)][i]
        fovx = math.radians([60, 50, 60, 70, 45, 30][i])
        fovy = 2 * math.atan(math.tan(fovx / 2) * H / W)
        q = rng.normal(0, 1, 4)
        q /= np.linalg.norm(q)
        r, x, y, z = q
        R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y)],
                      [2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x)],
                      [2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)]])
        if i == 0:
            R = np.eye(3)
        T = rng.normal(0, 2, 3) if i else np.zeros(3)
        # scene/cameras.py:61-66
        wv = torch.tensor(getWorld2View2(R, T, np.array([0.0, 0.0, 0.0]), 1.0)).transpose(0, 1)
        pr = getProjectionMatrix(znear=0.01, zfar=100.0, fovX=fovx, fovY=fovy).transpose(0, 1)
        full = wv.unsqueeze(0).bmm(pr.unsqueeze(0)).squeeze(0)
        center = wv.inverse()[3, :3]
        cams.append(dict(R=R, T=T, fovx=fovx, fovy=fovy, W=W, H=H, view=wv.numpy(), proj=full.numpy(),
                         center=center.numpy()))
    np.savez_compressed(os.path.join(OUT, "ref_camera_vectors.npz"),
                        **{f"{k}_{i}": np.asarray(v) for i, c in enumerate(cams) for k, v in c.items()},
                        n=np.array(len(cams)))
    # --- 3D covariance vectors: scene/gaussian_model.py:30-34 -------------------------------------
    import utils.general_utils as gu  # noqa: E402  (reference code)

    class _CpuTorch:
        """torch with zeros(..., device=...) allocating on the CPU (general_utils hard-codes "cuda")."""

        def __getattr__(self, name):
            return getattr(torch, name)

        @staticmethod
        def zeros(*args, device=None, **kw):
            return torch.zeros(*args, **kw)

    gu.torch = _CpuTorch()
    P = 1024
    scales = np.exp(rng.normal(np.log(0.05), 0.7, (P, 3))).astype(np.float32)
    rots = rng.normal(0, 1, (P, 4))
    rots = (rots / np.linalg.norm(rots, axis=1, keepdims=True)).astype(np.float32)
    cov = {}
    for tag, mod in (("mod1", 1.0), ("mod07", 0.7)):
        L = gu.build_scaling_rotation(mod * torch.from_numpy(scales), torch.from_numpy(rots))
        cov[tag] = gu.strip_symmetric(L @ L.transpose(1, 2)).numpy().astype(np.float32)
    np.savez_compressed(os.path.join(OUT, "ref_cov3d_vectors.npz"), scales=scales, rotations=rots, **cov)
    # --- HexPlane field and smoothness: scene/hexplane.py, scene/regulation.py -------------------------
    import importlib.util

    def load(name, rel):
        spec = importlib.util.spec_from_file_location(name, os.path.join(REF, rel))
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        return mod

    hp = load("ref_hexplane", "scene/hexplane.py")
    rg = load("ref_regulation", "scene/regulation.py")
    torch.manual_seed(5)
    cfg = {"grid_dimensions": 2, "input_coordinate_dim": 4, "output_coordinate_dim": 4, "resolution": [8, 6, 10, 5]}
    field = hp.HexPlaneField(1.6, cfg, [1, 2])
    with torch.no_grad():  # move the planes off their initial values (the time planes start at exactly 1)
        for level in field.grids:
            for pl in level:
                pl.add_(0.2 * torch.randn_like(pl))
    N = 300
    pts = torch.from_numpy(rng.uniform(-1.9, 1.9, (N, 3)).astype(np.float32)).requires_grad_(True)
    tms = torch.from_numpy(rng.uniform(-1.2, 1.2, (N, 1)).astype(np.float32))  # beyond [-1, 1]: border clip
    feat = field(pts, tms)
    G = torch.from_numpy(rng.normal(0, 1, tuple(feat.shape)).astype(np.float32))
    (feat * G).sum().backward()
    hx = dict(pts=pts.detach().numpy(), times=tms.numpy(), G=G.numpy(), feat=feat.detach().numpy(),
              gpts=pts.grad.numpy(), levels=np.array(len(field.grids)))
    for li, level in enumerate(field.grids):
        for pi, pl in enumerate(level):
            hx[f"plane_{li}_{pi}"] = pl.detach().numpy()
            hx[f"gplane_{li}_{pi}"] = pl.grad.numpy()
            hx[f"smooth_{li}_{pi}"] = np.array(float(rg.compute_plane_smoothness(pl.detach())), np.float32)
    np.savez_compressed(os.path.join(OUT, "ref_hexplane_vectors.npz"), **hx)

    # --- learning-rate schedules: utils/general_utils.py:35-68 -------------------------------------------
    steps = np.array([-1, 0, 1, 2, 7, 100, 499, 500, 1000, 3000, 3001, 9999, 14000, 20000, 30000, 10 ** 6])
    lr = dict(steps=steps)
    # (lr_init, lr_final, lr_delay_mult, max_steps): position / deformation / grid of arguments/__init__.py
    # defaults and arguments/dynerf/default.py (spatial_lr_scale folded into the first two as the model does)
    for i, (a0, a1, dm, ms) in enumerate([(0.00016 * 5.0, 0.0000016 * 5.0, 0.01, 20000),
                                          (0.00016 * 5.0, 0.000016 * 5.0, 0.01, 20000),
                                          (0.0016 * 5.0, 0.00016 * 5.0, 0.01, 20000),
                                          (0.0016, 0.000016, 0.01, 14000),
                                          (1e-3, 1e-3, 1.0, 1000)]):
        f = gu.get_expon_lr_func(a0, a1, lr_delay_mult=dm, max_steps=ms)
        lr[f"args_{i}"] = np.array([a0, a1, dm, ms], np.float64)
        lr[f"lr_{i}"] = np.array([f(int(k)) for k in steps], np.float64)
    np.savez_compressed(os.path.join(OUT, "ref_lr_vectors.npz"), **lr)
    print("wrote ref_{sh,camera,cov3d,hexplane,lr}_vectors.npz")


if __name__ == "__main__":
    main()
