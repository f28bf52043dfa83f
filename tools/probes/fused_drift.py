"""Fused vs unfused training drift (GPU diagnostic): the bouncing-balls setup of
tests/test_training_quality_gpu.py, both models stepped side by side on the same views; after each step the
largest relative parameter difference per group is printed, to tell rounding-level drift from a
systematic difference in one of the fused kernels."""
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


def make(fused, extent, hyper, opt):
    torch.manual_seed(0)
    rng = np.random.default_rng(0)
    pts = (rng.random((2000, 3)) * 2.6 - 1.3).astype(np.float32)
    cols = ((rng.random((2000, 3)) / 255.0) * 0.28209479177387814 + 0.5).astype(np.float32)
    g = GaussianModel(3, hyper, fused=fused)
    g.create_from_pcd(pts, cols, spatial_lr_scale=extent, device="cuda")
    g.cameras_extent = extent
    g._deformation.deformation_net.grid.fused = fused
    g._deformation.deformation_net.fused_heads = fused
    g.training_setup(opt)
    return g


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "dnerf"
    stage = sys.argv[2] if len(sys.argv) > 2 else "fine"
    nsteps = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    train_views, _ = T.make_dataset()
    hyper, opt = getattr(config, cfg)()
    opt = copy.copy(opt)
    opt.iterations = 100000
    opt.densify_from_iter = 10 ** 9  # no densification: same point set in both runs
    extent = T._extent(train_views)
    ga, gb = make(True, extent, hyper, opt), make(False, extent, hyper, opt)
    bg = torch.ones(3, device="cuda")
    rng = np.random.default_rng(0)
    for it in range(1, nsteps + 1):
        v = int(rng.integers(len(train_views)))
        la = float(train_step(ga, [train_views[v]], opt, hyper, it, bg, stage=stage))
        lb = float(train_step(gb, [train_views[v]], opt, hyper, it, bg, stage=stage))
        diffs = {}
        for (na, pa), (nb, pb) in zip(ga._deformation.named_parameters(), gb._deformation.named_parameters()):
            key = "grid" if "grid" in na else "mlp"
            d = ((pa - pb).abs().max() / pb.abs().max().clamp_min(1e-30)).item()
            diffs[key] = max(diffs.get(key, 0.0), d)
        for name in ("_xyz", "_features_dc", "_features_rest", "_opacity", "_scaling", "_rotation"):
            pa, pb = getattr(ga, name), getattr(gb, name)
            diffs[name] = ((pa - pb).abs().max() / pb.abs().max().clamp_min(1e-30)).item()
        print(f"it {it} loss {la:.6f} {lb:.6f} " + " ".join(f"{k}={v:.1e}" for k, v in diffs.items()), flush=True)


if __name__ == "__main__":
    main()
