"""Host-side cost of the bf16 deformation MLP step (GPU): torch.profiler CPU-time table of a few train
steps with hyper.mlp_dtype = "bf16"."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "4dgaussians-fast-train_amd")]
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402
from gs4d_train import config  # noqa: E402
from gs4d_train.gaussians import GaussianModel  # noqa: E402
from gs4d_train.synthetic import CONFIGS, make_point_cloud, make_training_views  # noqa: E402
from gs4d_train.train import train_step  # noqa: E402

P, W, H = CONFIGS["metric"]
hyper, opt = config.dynerf()
hyper.mlp_dtype = sys.argv[1] if len(sys.argv) > 1 else "bf16"
torch.manual_seed(0)
g = GaussianModel(3, hyper, fused=True)
pts, cols = make_point_cloud(P, seed=0)
g.create_from_pcd(pts, cols, spatial_lr_scale=1.0, device="cuda")
g._deformation.deformation_net.grid.fused = True
g._deformation.deformation_net.fused_heads = True
g.training_setup(opt)
g.active_sh_degree = 3
views = make_training_views(1, W, H, seed=1, device="cuda")
bg = torch.ones(3, device="cuda")
for i in range(5):
    train_step(g, views, opt, hyper, 3001 + i, bg)
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU]) as prof:
    for i in range(3):
        train_step(g, views, opt, hyper, 3006 + i, bg)
    torch.cuda.synchronize()
print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=25, max_name_column_width=50))
