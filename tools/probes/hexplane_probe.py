"""HexPlane field kernel timing probe (diagnostic, GPU): forward / order / backward at the DyNeRF
layout (F = 16, resolution [64, 64, 64, 150], multires [1, 2]) for P points uniform in the field,
backward with the Morton order and with the identity order."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "4dgaussians-fast-train_amd")]
from gs4d_train import _C  # noqa: E402


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main(P=100_000):
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    F = 16
    planes = []
    for res in (1, 2):
        reso = [64 * res, 64 * res, 64 * res, 150]
        for c0, c1 in [(0, 1), (0, 2), (0, 3), (1, 2), (1, 3), (2, 3)]:
            planes.append(torch.rand(1, F, reso[c1], reso[c0], device=dev))
    pts = torch.rand(P, 4, device=dev) * 1.5 - 0.75
    pts[:, 3] = 0.3
    feat, packed, order = _C.hexplane_forward(pts, planes)
    dfeat = torch.randn_like(feat)
    ident = torch.arange(P, device=dev, dtype=torch.int32)
    print(f"P={P}")
    print(f"forward (pack + order + field): {timed(lambda: _C.hexplane_forward(pts, planes)):.1f} us")
    print(f"backward, Morton order:   {timed(lambda: _C.hexplane_backward(pts, planes, packed, dfeat, order)):.1f} us")
    print(f"backward, identity order: {timed(lambda: _C.hexplane_backward(pts, planes, packed, dfeat, ident)):.1f} us")
    d1, g1 = _C.hexplane_backward(pts, planes, packed, dfeat, order)
    d2, g2 = _C.hexplane_backward(pts, planes, packed, dfeat, ident)
    err = max(float((a - b).abs().max() / b.abs().max()) for a, b in zip(g1, g2))
    print(f"plane gradients, Morton vs identity order: max rel diff {err:.2e}; dpts {float((d1 - d2).abs().max()):.2e}")


if __name__ == "__main__":
    main()
