"""Which fused piece changes the training trajectory?  The bouncing-balls convergence run of
tests/test_training_quality_gpu.py with the fused model but one piece swapped for its torch formulation
(Adam, densification statistics, L1, deformation tail, HexPlane field, heads), or the reverse."""
import copy
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "4dgaussians-fast-train_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import test_training_quality_gpu as T  # noqa: E402
from gs4d_train import config  # noqa: E402
from gs4d_train.gaussians import GaussianModel  # noqa: E402
from gs4d_train.train import train_step  # noqa: E402


def run(ds, fused, torch_adam=False, torch_stats=False, torch_l1=False, torch_tail=False, torch_field=False,
        torch_heads=False, seed=0, kc=800, kf=2500):
    train_views, test_views = ds
    hyper, opt = config.dnerf()
    opt_c, opt_f = copy.copy(opt), copy.copy(opt)
    opt_c.iterations, opt_f.iterations = kc, kf
    extent = T._extent(train_views)
    torch.manual_seed(seed)
    rng = np.random.default_rng(seed)
    pts = (rng.random((2000, 3)) * 2.6 - 1.3).astype(np.float32)
    cols = ((rng.random((2000, 3)) / 255.0) * 0.28209479177387814 + 0.5).astype(np.float32)
    g = GaussianModel(3, hyper, fused=fused)
    g.create_from_pcd(pts, cols, spatial_lr_scale=extent, device="cuda")
    g.cameras_extent = extent
    g._deformation.deformation_net.grid.fused = fused and not torch_field
    g._deformation.deformation_net.fused_heads = fused and not torch_heads
    if torch_tail:
        g.fused_tail = False
    if torch_stats:
        orig = g.add_densification_stats

        def stats(*a, **k):
            g.fused = False
            try:
                return orig(*a, **k)
            finally:
                g.fused = True
        g.add_densification_stats = stats
    bg = torch.ones(3, device="cuda")
    for stage, o, K in (("coarse", opt_c, kc), ("fine", opt_f, kf)):
        if torch_adam:
            g.fused = False
            g.training_setup(o)
            g.fused = True
        else:
            g.training_setup(o)
        for it in range(1, K + 1):
            v = int(rng.integers(len(train_views)))
            train_step(g, [train_views[v]], o, hyper, it, bg, stage=stage,
                       fused_loss=False if torch_l1 else None)
    torch.cuda.synchronize()
    return T._evaluate(g, test_views, bg), T._evaluate(g, train_views, bg), g.get_xyz.shape[0]


if __name__ == "__main__":
    ds = T.make_dataset()
    variants = [("fused", dict(fused=True)), ("unfused", dict(fused=False)),
                ("fused+torch_adam", dict(fused=True, torch_adam=True)),
                ("fused+torch_stats", dict(fused=True, torch_stats=True)),
                ("fused+torch_l1", dict(fused=True, torch_l1=True)),
                ("fused+torch_tail", dict(fused=True, torch_tail=True)),
                ("fused+torch_field", dict(fused=True, torch_field=True)),
                ("fused+torch_heads", dict(fused=True, torch_heads=True))]
    only = sys.argv[1].split(",") if len(sys.argv) > 1 else None
    for name, kw in variants:
        if only and name not in only:
            continue
        te, tr, n = run(ds, **kw)
        print(f"{name:20s} test {te:.2f} train {tr:.2f} n={n}", flush=True)
