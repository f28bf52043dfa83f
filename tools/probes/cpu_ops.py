"""Host-side cost probe (diagnostic, GPU): torch.profiler table of a few train steps sorted by self CPU
time, and the step time with gs4d_train.render's fused deformation tail on and off."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "4dgaussians-fast-train_amd")]
from gs4d_train import config  # noqa: E402
from gs4d_train.gaussians import GaussianModel  # noqa: E402
from gs4d_train.synthetic import CONFIGS, make_point_cloud, make_training_views  # noqa: E402
from gs4d_train.train import train_step  # noqa: E402


def setup():
    P, W, H = CONFIGS["metric"]
    dev = torch.device("cuda:0")
    hyper, opt = config.dynerf()
    torch.manual_seed(0)
    g = GaussianModel(3, hyper, fused=True)
    pts, cols = make_point_cloud(P, seed=0)
    g.create_from_pcd(pts, cols, spatial_lr_scale=1.0, device=dev)
    g._deformation.deformation_net.grid.fused = True
    g._deformation.deformation_net.fused_heads = True
    g.training_setup(opt)
    g.active_sh_degree = 3
    views = make_training_views(1, W, H, seed=1, device=dev)
    return g, views, opt, hyper, torch.ones(3, device=dev)


def timed(g, views, opt, hyper, bg, n=20, it0=3001):
    for i in range(5):
        train_step(g, views, opt, hyper, it0 + i, bg)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(n):
        train_step(g, views, opt, hyper, it0 + 5 + i, bg)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


if __name__ == "__main__":
    from torch.profiler import ProfilerActivity, profile
    g, views, opt, hyper, bg = setup()
    for rep in range(3):
        for tail in (True, False):
            g.fused_tail = tail
            print(f"fused_tail={tail}: step {timed(g, views, opt, hyper, bg, it0=3101):.3f} ms")
    g.fused_tail = True
    with profile(activities=[ProfilerActivity.CPU]) as prof:
        for i in range(3):
            train_step(g, views, opt, hyper, 3201 + i, bg)
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=30, max_name_column_width=50))
