"""Host-side timing of one training step's calls (GPU box): how long the host spends inside each call
versus the GPU time, to tell launch-bound from GPU-bound phases."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "4dgaussians-fast-train_amd"))
from gs4d_train.synthetic import CONFIGS, make_scene  # noqa: E402
import diff_gaussian_rasterization as dgr  # noqa: E402


def main():
    P, W, H = CONFIGS["metric"]
    s = make_scene(P, W, H, seed=0)
    dev = torch.device("cuda", 0)
    t = lambda a: torch.tensor(np.asarray(a), device=dev)
    bg, vm, pm, cp = t(s["bg"]), t(s["viewmatrix"]), t(s["projmatrix"]), t(s["campos"])
    means3D, opac, scales, rots, shs = (t(s[k]) for k in ("means3D", "opacities", "scales", "rotations", "shs"))
    e = torch.empty(0, device=dev)
    gt = torch.rand(3, H, W, device=dev)
    C = dgr._C
    rec = {"fwd_call": [], "loss_ops": [], "bwd_call": [], "step_wall": []}
    for it in range(60):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = C.rasterize_gaussians(bg, means3D, e, opac, scales, rots, 1.0, e, vm, pm, s["tanfovx"], s["tanfovy"],
                                    H, W, shs, 3, cp, False, False)
        t1 = time.perf_counter()
        nr, color, depth, radii, gb, bb, ib = out
        diff = color - gt
        loss = diff.abs().mean()
        grad = torch.sign(diff) / diff.numel()
        t2 = time.perf_counter()
        C.rasterize_gaussians_backward(bg, means3D, radii, e, scales, rots, 1.0, e, vm, pm, s["tanfovx"],
                                       s["tanfovy"], grad, shs, 3, cp, gb, nr, bb, ib, False)
        t3 = time.perf_counter()
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        if it >= 10:
            rec["fwd_call"].append(t1 - t0)
            rec["loss_ops"].append(t2 - t1)
            rec["bwd_call"].append(t3 - t2)
            rec["step_wall"].append(t4 - t0)
    for k, v in rec.items():
        print(f"{k:10s} median {np.median(v) * 1e6:8.1f} us")


if __name__ == "__main__":
    main()
