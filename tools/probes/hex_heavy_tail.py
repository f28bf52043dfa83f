"""Per-cell accuracy of the fused HexPlane backward's fixed-point sums with heavy-tailed dfeat (1 % of the points'
gradients scaled by 1e4), against float64 grid_sample, beside the float32 grid_sample graph's own error.
Prints, per plane, the max / median relative error over cells in magnitude bands of the plane's largest cell."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "4dgaussians-fast-train_amd"))
from gs4d_train import _C  # noqa: E402
from gs4d_train.deformation import HexPlaneField, interpolate_ms_features  # noqa: E402

torch.manual_seed(3)
F, N = 16, 50_000
f = HexPlaneField(1.6, {"grid_dimensions": 2, "input_coordinate_dim": 4, "output_coordinate_dim": F,
                        "resolution": [64, 64, 64, 150]}, [1, 2]).cuda()
with torch.no_grad():
    for level in f.grids:
        for p in level:
            p.uniform_(0.1, 1.2)
planes = [p.detach() for l in f.grids for p in l]
g = torch.Generator(device="cuda").manual_seed(21)
pts = torch.rand(N, 4, device="cuda", generator=g) * 2 - 1
feat, packed, order = _C.hexplane_forward(pts, planes)
for heavy in (False, True):
    dfeat = torch.randn(feat.shape, device="cuda", generator=g)
    if heavy:
        rows = torch.randperm(N, device="cuda", generator=g)[: N // 100]
        dfeat[rows] *= 1e4
    _, gf = _C.hexplane_backward(pts, planes, packed, dfeat, order)
    p64 = [p.double().requires_grad_(True) for p in planes]
    g64 = torch.autograd.grad(interpolate_ms_features(pts.double(), [p64[:6], p64[6:]]), p64, dfeat.double())
    g32 = torch.autograd.grad(interpolate_ms_features(pts, [list(f.grids[0]), list(f.grids[1])]),
                              [p for l in f.grids for p in l], dfeat)
    print(f"heavy={heavy}")
    for i, (a, b, r) in enumerate(zip(gf, g32, g64)):
        m = r.abs().max().item()
        out = []
        for lo, hi in ((1e-3, 1.01), (1e-5, 1e-3), (1e-7, 1e-5), (1e-9, 1e-7)):
            sel = (r.abs() >= lo * m) & (r.abs() < hi * m)
            if int(sel.sum()) == 0:
                out.append(f"[{lo:.0e}: none]")
                continue
            ea = ((a.double() - r).abs() / r.abs())[sel]
            eb = ((b.double() - r).abs() / r.abs())[sel]
            out.append(f"[{lo:.0e}: n={int(sel.sum())} fused max {ea.max().item():.1e} med {ea.median().item():.1e} | "
                       f"torch32 max {eb.max().item():.1e} med {eb.median().item():.1e}]")
        print(f"  plane {i}: " + " ".join(out), flush=True)
