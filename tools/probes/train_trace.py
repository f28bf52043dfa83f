"""Train-step timing probe (diagnostic, GPU): N fine-stage steps of gs4d_train.train.train_step at a
bench config, wall time per step and (under rocprofv3 --kernel-trace) the kernels it launches."""
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


def main(cfg="metric", steps=20, fused=True):
    P, W, H = CONFIGS[cfg]
    dev = torch.device("cuda:0")
    hyper, opt = config.dynerf()
    if "--bf16" in sys.argv:
        hyper.mlp_dtype = "bf16"
    torch.manual_seed(0)
    g = GaussianModel(3, hyper, fused=fused)
    pts, cols = make_point_cloud(P, seed=0)
    g.create_from_pcd(pts, cols, spatial_lr_scale=1.0, device=dev)
    g._deformation.deformation_net.grid.fused = fused
    g._deformation.deformation_net.fused_heads = fused
    g.training_setup(opt)
    g.active_sh_degree = 3
    views = make_training_views(1, W, H, seed=1, device=dev)
    bg = torch.ones(3, device=dev)
    for i in range(5):
        train_step(g, views, opt, hyper, 3001 + i, bg)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        train_step(g, views, opt, hyper, 3006 + i, bg)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / steps * 1e3
    # host-side cost: the same steps with the GPU work queued but not waited on is not separable; report
    # the wall time and let the kernel trace give the device time
    print(f"train_step {cfg} fused={fused} mlp={hyper.mlp_dtype}: {el:.3f} ms/step")


def op_profile(cfg="metric", steps=5):
    """torch.profiler op table (device time) of a few train steps."""
    from torch.profiler import ProfilerActivity, profile
    P, W, H = CONFIGS[cfg]
    dev = torch.device("cuda:0")
    hyper, opt = config.dynerf()
    if "--bf16" in sys.argv:
        hyper.mlp_dtype = "bf16"
    torch.manual_seed(0)
    g = GaussianModel(3, hyper, fused=True)
    pts, cols = make_point_cloud(P, seed=0)
    g.create_from_pcd(pts, cols, spatial_lr_scale=1.0, device=dev)
    g._deformation.deformation_net.grid.fused = True
    g._deformation.deformation_net.fused_heads = True
    g.training_setup(opt)
    g.active_sh_degree = 3
    views = make_training_views(1, W, H, seed=1, device=dev)
    bg = torch.ones(3, device=dev)
    for i in range(5):
        train_step(g, views, opt, hyper, 3001 + i, bg)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes="--shapes" in sys.argv) as prof:
        for i in range(steps):
            train_step(g, views, opt, hyper, 3006 + i, bg)
        torch.cuda.synchronize()
    if "--shapes" in sys.argv:
        print(prof.key_averages(group_by_input_shape=True).table(sort_by="cuda_time_total", row_limit=400,
                                                                 max_name_column_width=40, max_shapes_column_width=70))
    else:
        key = "self_cpu_time_total" if "--cpu" in sys.argv else "cuda_time_total"
        print(prof.key_averages().table(sort_by=key, row_limit=45, max_name_column_width=60))


def py_profile(cfg="metric", steps=30):
    """cProfile of a few train steps (host cost by Python function; the GPU runs asynchronously, so a C
    entry point's time is its launch path, and a wait shows up in whatever call synchronises)."""
    import cProfile
    import pstats
    P, W, H = CONFIGS[cfg]
    dev = torch.device("cuda:0")
    hyper, opt = config.dynerf()
    if "--bf16" in sys.argv:
        hyper.mlp_dtype = "bf16"
    torch.manual_seed(0)
    g = GaussianModel(3, hyper, fused=True)
    pts, cols = make_point_cloud(P, seed=0)
    g.create_from_pcd(pts, cols, spatial_lr_scale=1.0, device=dev)
    g._deformation.deformation_net.grid.fused = True
    g._deformation.deformation_net.fused_heads = True
    g.training_setup(opt)
    g.active_sh_degree = 3
    views = make_training_views(1, W, H, seed=1, device=dev)
    bg = torch.ones(3, device=dev)
    for i in range(5):
        train_step(g, views, opt, hyper, 3001 + i, bg)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    for i in range(steps):
        train_step(g, views, opt, hyper, 3006 + i, bg)
    pr.disable()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"host {1e3 * (t1 - t0) / steps:.3f} ms/step under cProfile, drain {1e3 * (t2 - t1):.3f} ms")
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(45)
    st.sort_stats("cumulative").print_stats(45)


if __name__ == "__main__":
    if "--pyprof" in sys.argv:
        py_profile()
    elif "--ops" in sys.argv:
        op_profile()
    else:
        args = [a for a in sys.argv[1:] if not a.startswith("--")]
        main(args[0] if args else "metric")
