"""Diagnostic (GPU): error of gs4d_heads_forward and of torch.addmm on the same column slices against
fp64, on random ReLU'd inputs (RMS and max of |err| / |terms| sum)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "4dgaussians-fast-train_amd")]
from gs4d_train import _C  # noqa: E402

torch.manual_seed(0)
P, W, ns = 100_000, 128, [3, 3, 4, 1, 48]
a = torch.relu(torch.randn(P, len(ns) * W, device="cuda"))
w2 = [torch.randn(n, W, device="cuda") * 0.05 for n in ns]
b2 = [torch.randn(n, device="cuda") * 0.01 for n in ns]
out = _C.heads_forward(a, w2, b2)
for i, (w, b) in enumerate(zip(w2, b2)):
    x = a[:, i * W:(i + 1) * W]
    ref = x.double() @ w.double().t() + b.double()
    scale = x.double().abs() @ w.double().abs().t() + b.double().abs()
    mm = torch.addmm(b, x, w.t())
    ek = ((out[i].double() - ref).abs() / scale)
    em = ((mm.double() - ref).abs() / scale)
    print(f"head {i} n={ns[i]}: kernel rms {ek.pow(2).mean().sqrt().item():.2e} max {ek.max().item():.2e} | "
          f"addmm rms {em.pow(2).mean().sqrt().item():.2e} max {em.max().item():.2e} | "
          f"kernel-addmm max |d|/|ref| {((out[i] - mm).abs() / ref.abs().float().clamp_min(1e-30)).median().item():.2e}")
