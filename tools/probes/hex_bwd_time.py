"""Time _C.hexplane_backward alone (100k points, DyNeRF planes F=16 [64,64,64,150] x multires [1,2]),
points spread in xyz, one timestamp (a training step's single view) or random times."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "4dgaussians-fast-train_amd")]
from gs4d_train import _C  # noqa: E402
from gs4d_train.deformation import HexPlaneField  # noqa: E402


def main():
    torch.manual_seed(3)
    f = HexPlaneField(1.6, {"grid_dimensions": 2, "input_coordinate_dim": 4, "output_coordinate_dim": 16,
                            "resolution": [64, 64, 64, 150]}, [1, 2]).cuda()
    with torch.no_grad():
        for level in f.grids:
            for p in level:
                p.uniform_(0.1, 1.2)
    planes = [p.detach() for l in f.grids for p in l]
    g = torch.Generator(device="cuda").manual_seed(7)
    for one_time in (True, False):
        pts = torch.rand(100_000, 4, device="cuda", generator=g) * 2 - 1
        if one_time:
            pts[:, 3] = 0.3137
        feat, packed, order = _C.hexplane_forward(pts, planes)
        dfeat = torch.randn_like(feat) * 1e-3
        for _ in range(3):
            _C.hexplane_backward(pts, planes, packed, dfeat, order)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            _C.hexplane_backward(pts, planes, packed, dfeat, order)
        e1.record()
        torch.cuda.synchronize()
        print(f"hexplane_backward one_time={one_time}: {e0.elapsed_time(e1) / 20 * 1e3:.1f} us per call", flush=True)


if __name__ == "__main__":
    main()
