"""Per-tile work distribution of the blend kernels at a bench config (diagnostic, GPU).

Reads the image scratch the forward returns (ImageState layout, csrc/capi.hip): final_T | n_contrib |
ranges, each 256-byte aligned.  Prints the tile list lengths and the backward walk lengths (max
n_contrib over the tile's pixels) as percentiles, and how the work concentrates in the longest tiles.
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "4dgaussians-fast-train_amd")]
from gs4d_train.synthetic import CONFIGS, make_scene  # noqa: E402
import diff_gaussian_rasterization as dgr  # noqa: E402


def a256(x):
    return (x + 255) // 256 * 256


def main(cfg="metric"):
    P, W, H = CONFIGS[cfg]
    dev = torch.device("cuda:0")
    s = make_scene(P, W, H, seed=0)
    t = lambda a: torch.tensor(np.asarray(a), device=dev)
    e = torch.empty(0, device=dev)
    nr, color, depth, radii, gb, bb, ib = dgr._C.rasterize_gaussians(
        t(s["bg"]), t(s["means3D"]), e, t(s["opacities"]), t(s["scales"]), t(s["rotations"]), 1.0, e,
        t(s["viewmatrix"]), t(s["projmatrix"]), s["tanfovx"], s["tanfovy"], H, W, t(s["shs"]), 3, t(s["campos"]),
        False, False)
    torch.cuda.synchronize()
    assert ib.data_ptr() % 256 == 0
    N = W * H
    gx, gy = (W + 15) // 16, (H + 15) // 16
    raw = ib.cpu().numpy()
    o_nc = a256(4 * N)
    o_rg = o_nc + a256(4 * N)
    n_contrib = raw[o_nc:o_nc + 4 * N].view(np.uint32).reshape(H, W)
    ranges = raw[o_rg:o_rg + 8 * gx * gy].view(np.uint32).reshape(gx * gy, 2)
    lens = (ranges[:, 1] - ranges[:, 0]).astype(np.int64)
    pad = np.zeros((gy * 16, gx * 16), np.uint32)
    pad[:H, :W] = n_contrib
    walk = pad.reshape(gy, 16, gx, 16).max(axis=(1, 3)).reshape(-1).astype(np.int64)
    print(f"config {cfg}: P={P} {W}x{H} tiles={gx * gy} L={nr} L'={lens.sum()}")
    for name, v in (("list length", lens), ("bwd walk", walk)):
        q = np.percentile(v, [0, 25, 50, 75, 90, 99, 100])
        srt = np.sort(v)[::-1]
        top = [srt[:k].sum() / max(v.sum(), 1) for k in (54, 272, 544)]
        print(f"{name}: mean {v.mean():.1f} pct[0,25,50,75,90,99,100] {q.astype(int).tolist()} "
              f"share of top 1%/5%/10% tiles {top[0]:.3f}/{top[1]:.3f}/{top[2]:.3f}")
    for S in (128, 256, 512):
        segs = np.maximum(1, (walk + S - 1) // S)
        print(f"segments of {S}: {segs.sum()} work items, max per item {min(S, walk.max())}")
    # tile-row profile: mean walk per tile row (where the heavy tiles are)
    rows = walk.reshape(gy, gx).mean(axis=1)
    print("mean walk by tile row:", np.round(rows[::4]).astype(int).tolist())


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "metric")
