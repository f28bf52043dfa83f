"""Device time of the train step's smaller HIP passes at its shapes (diagnostic, GPU): the first deformation
layer's backward (P = 100k, 32 -> 128), the deformation tail both ways, HIP events over R calls.  For A/B of
libgs4d variants (LD_LIBRARY_PATH=4dgaussians-fast-train_amd/build/variant_<name>)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "4dgaussians-fast-train_amd")]
from gs4d_train import _C  # noqa: E402


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    P, Fin, Fout = 100_000, 32, 128
    torch.manual_seed(0)
    x = torch.randn(P, Fin, device="cuda")
    w = torch.randn(Fout, Fin, device="cuda") / Fin ** 0.5
    b = torch.randn(Fout, device="cuda") * 0.1
    h = _C.feature_relu_forward(x, w, b)[0]
    g = torch.randn(P, Fout, device="cuda")
    rows = [("feature_relu_forward", lambda: _C.feature_relu_forward(x, w, b)),
            ("feature_relu_forward (+hb)", lambda: _C.feature_relu_forward(x, w, b, with_hb=True)),
            ("feature_relu_backward", lambda: _C.feature_relu_backward(g, h, x, w))]
    # the HexPlane regulariser's gradient (+ value) at DyNeRF's planes (F = 16, [64, 64, 64, 150] x multires [1, 2])
    from gs4d_train.kernels import hexplane_regulation_accumulate_grad
    grids = []
    for reso in ([64, 64, 64, 150], [128, 128, 128, 150]):
        pairs = [(0, 1), (0, 2), (0, 3), (1, 2), (1, 3), (2, 3)]
        grids.append([torch.rand(1, 16, reso[c1], reso[c0], device="cuda").requires_grad_(True) for c0, c1 in pairs])
    for lvl in grids:
        for q in lvl:
            q.grad = torch.zeros_like(q)
    rows.append(("reg accumulate + value", lambda: hexplane_regulation_accumulate_grad(grids, 1.0, 1e-4, 2e-4, 1.0, True)))
    rows.append(("reg accumulate", lambda: hexplane_regulation_accumulate_grad(grids, 1.0, 1e-4, 2e-4, 1.0, False)))
    # the L1 value + gradient at the bench image (3 x 1014 x 1352)
    img, gt = torch.rand(3, 1014, 1352, device="cuda"), torch.rand(3, 1014, 1352, device="cuda")
    rows.append(("l1_loss_grad", lambda: _C.l1_loss_grad(img, gt, 1.0)))
    for name, fn in rows:
        print(f"{name:28s} {timed(fn):8.1f} us", flush=True)


if __name__ == "__main__":
    main()
