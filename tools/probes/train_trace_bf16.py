"""Train-step kernel trace (GPU, under rocprofv3 --kernel-trace) at the metric config, fp32 or the
opt-in bf16 deformation MLP: python tools/probes/train_trace_bf16.py [fp32|bf16] [steps]."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "4dgaussians-fast-train_amd")]
import torch  # noqa: E402
from gs4d_train import config  # noqa: E402
from gs4d_train.gaussians import GaussianModel  # noqa: E402
from gs4d_train.synthetic import CONFIGS, make_point_cloud, make_training_views  # noqa: E402
from gs4d_train.train import train_step  # noqa: E402

dtype = sys.argv[1] if len(sys.argv) > 1 else "fp32"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
P, W, H = CONFIGS["metric"]
dev = torch.device("cuda:0")
hyper, opt = config.dynerf()
hyper.mlp_dtype = dtype
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
t0 = time.perf_counter()
for i in range(steps):
    train_step(g, views, opt, hyper, 3006 + i, bg)
torch.cuda.synchronize()
print(f"train_step {dtype}: {(time.perf_counter() - t0) / steps * 1e3:.3f} ms/step", flush=True)
