"""Diagnostic (GPU): one fused train step with the heads' second layers through gs4d_heads_forward vs
through torch.addmm (everything else identical): per-gradient max and 99.9th-percentile relative
differences, to tell summation-order noise (+ rare blend threshold flips) from a defect."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "4dgaussians-fast-train_amd")]
from gs4d_train import config, deformation  # noqa: E402
from gs4d_train.gaussians import GaussianModel  # noqa: E402
from gs4d_train.synthetic import make_point_cloud, make_training_views  # noqa: E402
from gs4d_train.train import train_step  # noqa: E402


def run(use_kernel, fused=True):
    hyper, opt = config.dynerf()
    opt.iterations = 0
    pts, cols = make_point_cloud(20000, seed=5)
    views = make_training_views(2, 320, 240, seed=6)
    bg = torch.ones(3, device="cuda")
    torch.manual_seed(7)
    g = GaussianModel(3, hyper, fused=fused)
    g.create_from_pcd(pts, cols, 1.0)
    g._deformation.deformation_net.grid.fused = fused
    g._deformation.deformation_net.fused_heads = fused
    g.training_setup(opt)
    g.active_sh_degree = 3
    from gs4d_train import _C
    orig = _C.heads_forward
    if not use_kernel:
        def addmm_heads(a, w2, b2):
            W = a.shape[1] // len(w2)
            return [torch.addmm(b, a[:, i * W:(i + 1) * W], w.t()) for i, (w, b) in enumerate(zip(w2, b2))]
        _C.heads_forward = addmm_heads
    try:
        loss = float(train_step(g, views, opt, hyper, 3001, bg))
    finally:
        _C.heads_forward = orig
    grads = {n: p.grad.detach().clone() for n, p in g._deformation.named_parameters() if p.grad is not None}
    for name in ("_xyz", "_features_dc", "_features_rest", "_opacity", "_scaling", "_rotation"):
        grads[name] = getattr(g, name).grad.detach().clone()
    return loss, grads


la, ga = run(True)
lb, gb = run(False)
lc, gc = run(False, fused=False)
print("loss", la, lb, lc)
for k in ga:
    for tag, ref in (("vs addmm", gb), ("vs unfused", gc)):
        a, b = ga[k], ref[k]
        s = max(b.abs().max().item(), 1e-30)
        d = ((a - b).abs() / s).flatten()
        print(f"{k:40s} {tag:10s} max {d.max().item():.2e}  p99.9 {d.kthvalue(max(1, int(0.999 * d.numel()))).values.item():.2e}")
    d = ((gb[k] - gc[k]).abs() / max(gc[k].abs().max().item(), 1e-30)).flatten()
    print(f"{k:40s} addmm-vs-unfused max {d.max().item():.2e}")
