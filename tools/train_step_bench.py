"""Time the full fine-stage train step (deformation + rasterizer + L1 + backward + densification
stats + Adam) of gs4d_train at a given size, fused (libgs4d kernels) vs the reference's torch tail."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "4dgaussians-fast-train_amd"))
import torch  # noqa: E402

from gs4d_train import config  # noqa: E402
from gs4d_train.gaussians import GaussianModel  # noqa: E402
from gs4d_train.synthetic import make_point_cloud, make_training_views  # noqa: E402
from gs4d_train.train import train_step  # noqa: E402


def run(P, W, H, views_per_step, steps, warmup, fused, hexfused):
    hyper, opt = config.dynerf()
    opt.batch_size = views_per_step
    torch.manual_seed(0)
    g = GaussianModel(3, hyper, fused=fused)
    pts, cols = make_point_cloud(P)
    g.create_from_pcd(pts, cols, spatial_lr_scale=1.0)
    g._deformation.deformation_net.grid.fused = hexfused
    g.training_setup(opt)
    g.active_sh_degree = 3
    views = make_training_views(max(4, views_per_step), W, H)
    bg = torch.ones(3, device="cuda")
    it = 3000  # fine stage, past densify_from_iter but not on a densification iteration
    for i in range(warmup):
        train_step(g, views[:views_per_step], opt, hyper, it + 1 + i, bg)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        train_step(g, views[:views_per_step], opt, hyper, it + 1 + warmup + i, bg)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=100_000)
    ap.add_argument("--W", type=int, default=1352)
    ap.add_argument("--H", type=int, default=1014)
    ap.add_argument("--views", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--modes", default="torch,fused", help="comma list of torch | fused | fused+hex")
    a = ap.parse_args()
    table = {"torch": (False, False), "fused": (True, False), "fused+hex": (True, True)}
    for fused, hexfused in (table[m] for m in a.modes.split(",")):
        ms = run(a.P, a.W, a.H, a.views, a.steps, a.warmup, fused, hexfused)
        print(f"train step P={a.P} {a.W}x{a.H} views={a.views} fused_tail={fused} fused_hexplane={hexfused}: {ms:.3f} ms",
              flush=True)
