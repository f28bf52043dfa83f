"""Per-tile workload statistics of the metric scene (GPU): instances per tile after culling and
per-pixel contributor counts -- the inputs for render-kernel scheduling decisions."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "4dgaussians-fast-train_amd"))
from gs4d_train.synthetic import CONFIGS, make_scene, make_train_like_scene  # noqa: E402
import diff_gaussian_rasterization as dgr  # noqa: E402


def main():
    P, W, H = CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "metric"]
    s = (make_train_like_scene if "--train-like" in sys.argv else make_scene)(P, W, H, seed=0)
    dev = torch.device("cuda", 0)
    t = lambda a: torch.tensor(np.asarray(a), device=dev)
    e = torch.empty(0, device=dev)
    out = dgr._C.rasterize_gaussians(t(s["bg"]), t(s["means3D"]), e, t(s["opacities"]), t(s["scales"]),
                                     t(s["rotations"]), 1.0, e, t(s["viewmatrix"]), t(s["projmatrix"]),
                                     s["tanfovx"], s["tanfovy"], H, W, t(s["shs"]), 3, t(s["campos"]), False, False)
    torch.cuda.synchronize()
    nr, color, depth, radii, gb, bb, ib = out
    N = W * H
    T = ((W + 15) // 16) * ((H + 15) // 16)
    al = lambda x: (x + 255) // 256 * 256
    raw = ib.cpu().numpy().view(np.uint8)
    base = (-ib.data_ptr()) % 256
    ncontrib = raw[base + al(4 * N): base + al(4 * N) + 4 * N].view(np.uint32)
    rng = raw[base + 2 * al(4 * N): base + 2 * al(4 * N) + 8 * T].view(np.uint32).reshape(T, 2)
    cnt = (rng[:, 1] - rng[:, 0]).astype(np.int64)
    q = lambda a: {p: int(np.percentile(a, p)) for p in (50, 90, 99, 100)}
    print("num_rendered", nr, "emitted", int(cnt.sum()), "tiles", T)
    print("instances/tile", q(cnt), "mean", float(cnt.mean()))
    hist = {f"{lo}-{hi}": int(((cnt >= lo) & (cnt <= hi)).sum()) for lo, hi in
            ((0, 128), (129, 256), (257, 512), (513, 1024), (1025, 2048), (2049, 1 << 30))}
    print("tiles by run length", hist)
    order = np.sort(cnt)[::-1]
    print("top tiles", order[:16].tolist())
    print("n_contrib/pixel", q(ncontrib), "mean", float(ncontrib.mean()))
    # per tile: max over the tile's pixels of n_contrib (how far the wave must walk)
    gx = (W + 15) // 16
    nc = np.zeros((((H + 15) // 16) * 16, gx * 16), np.uint32)
    nc[:H, :W] = ncontrib.reshape(H, W)
    tmax = nc.reshape(-1, 16, gx, 16).max(axis=(1, 3)).reshape(-1)
    print("walk length/tile (max n_contrib)", q(tmax), "mean", float(tmax.mean()), "sum", int(tmax.sum()))
    print("sum over tiles of instances", int(cnt.sum()), "frac walked", float(tmax.sum() / max(1, cnt.sum())))
    os.makedirs("gpurun_out", exist_ok=True)
    np.savez_compressed("gpurun_out/tile_stats.npz", cnt=cnt, tmax=tmax, gx=gx)


if __name__ == "__main__":
    main()
