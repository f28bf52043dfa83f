"""One fine-stage step, fused vs unfused (bouncing-balls setup, D-NeRF config): per HexPlane plane,
how the parameter gradients differ -- zero patterns, and the elementwise relative error of small
gradients, which Adam's first steps turn into full-size updates."""
import copy
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "4dgaussians-fast-train_amd"), os.path.join(ROOT, "tests"),
                os.path.join(ROOT, "tools", "probes")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import fused_drift as F  # noqa: E402
import test_training_quality_gpu as T  # noqa: E402
from gs4d_train import config  # noqa: E402
from gs4d_train.train import train_step  # noqa: E402

train_views, _ = T.make_dataset()
hyper, opt = config.dnerf()
opt = copy.copy(opt)
opt.iterations = 0  # no optimizer step: compare the gradients themselves
extent = T._extent(train_views)
ga, gb = F.make(True, extent, hyper, opt), F.make(False, extent, hyper, opt)
bg = torch.ones(3, device="cuda")
v = 3
for g in (ga, gb):
    train_step(g, [train_views[v]], opt, hyper, 1, bg, stage=sys.argv[1] if len(sys.argv) > 1 else "fine")
for (na, pa), (nb, pb) in zip(ga._deformation.named_parameters(), gb._deformation.named_parameters()):
    a, b = pa.grad, pb.grad
    if a is None or b is None:
        print(na, "grad None", a is None, b is None)
        continue
    za, zb = a == 0, b == 0
    scale = b.abs().max().clamp_min(1e-30)
    big = b.abs() > 1e-3 * scale
    rel = ((a - b).abs() / b.abs().clamp_min(1e-30))
    print(f"{na:60s} n={a.numel():8d} zero a/b {int(za.sum()):8d}/{int(zb.sum()):8d} mismatch {int((za != zb).sum()):7d} "
          f"max|d|/max {float((a - b).abs().max() / scale):.1e} rel(big) {float(rel[big].max()) if big.any() else 0:.1e} "
          f"rel(small) median {float(rel[~big & ~zb].median()) if (~big & ~zb).any() else 0:.1e}")
