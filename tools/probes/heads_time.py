"""Device time of the deformation heads' kernels at the train step's shapes (diagnostic, GPU): P = 100k,
W = 128, heads n = [3, 3, 4, 1, 48] (arguments/dynerf), fp32 and bf16 forms, HIP events over R calls."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "4dgaussians-fast-train_amd")]
from gs4d_train import _C, deformation as D  # noqa: E402


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
    P, W, ns = 100_000, 128, [3, 3, 4, 1, 48]
    k = len(ns)
    torch.manual_seed(0)
    dev = "cuda"
    h = torch.relu(torch.randn(P, W, device=dev))
    w1 = torch.randn(k * W, W, device=dev) / W ** 0.5
    b1 = torch.randn(k * W, device=dev) * 0.1
    w2 = [torch.randn(n, W, device=dev) / W ** 0.5 for n in ns]
    b2 = [torch.randn(n, device=dev) for n in ns]
    gs = [torch.randn(P, n, device=dev) for n in ns]
    a32, _, *_ = _C.heads_block_forward(h, w1, b1, w2, b2)
    abf, hb, w1t, *_ = _C.heads_block_forward_bf16(h, w1, b1, w2, b2)
    da32 = _C.heads_backward(a32.contiguous(), gs, w2)[0]
    dabf = _C.heads_backward(abf.contiguous(), gs, w2)[0]
    w1b = w1.to(torch.bfloat16)
    rows = [
        ("block forward fp32", lambda: _C.heads_block_forward(h, w1, b1, w2, b2)),
        ("block forward bf16", lambda: _C.heads_block_forward_bf16(h, w1, b1, w2, b2)),
        ("heads backward fp32", lambda: _C.heads_backward(a32.contiguous(), gs, w2)),
        ("heads backward bf16", lambda: _C.heads_backward(abf.contiguous(), gs, w2)),
        ("dW1 split-K fp32", lambda: D._splitk_dw(da32, h)),
        ("dW1 split-K bf16 (rocBLAS)", lambda: D._splitk_dw(dabf, hb)),
        ("dW1 bf16 (mlp_dw_bf16)", lambda: _C.mlp_dw_bf16(dabf, hb)),
        ("dh fp32", lambda: D._mm_dx(da32, w1)),
        ("dh bf16 (rocBLAS)", lambda: D._mm_dx(dabf, w1b)),
        ("dh bf16 (mlp_dx_bf16)", lambda: _C.mlp_dx_bf16(dabf, w1t)),
    ]
    if "--fwd32" in sys.argv:  # only the fp32 block forward (PMC passes: tools/hfpmc.sh)
        rows = rows[:1]
    for name, fn in rows:
        print(f"{name:24s} {timed(fn):8.1f} us", flush=True)


if __name__ == "__main__":
    main()
