"""Host-side cost per call of the deformation MLP's GPU entry points (diagnostic, GPU): each call is issued
N times on small operands without synchronising, so the wall time per call is the host path (argument
checks, allocator, library heuristics), not the kernel."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "4dgaussians-fast-train_amd")]
from gs4d_train import _C, deformation as D  # noqa: E402


def per_call(fn, n=200):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    return (t1 - t0) / n * 1e6


def main():
    dev = "cuda"
    P, kW, W = 4096, 640, 128
    bf = torch.bfloat16
    da32 = torch.randn(P, kW, device=dev)
    h32 = torch.relu(torch.randn(P, W, device=dev))
    w1 = torch.randn(kW, W, device=dev)
    da, hb, w1b = da32.to(bf), h32.to(bf), w1.to(bf)
    rows = {
        "splitk_dw f32 (tuned)": lambda: D._splitk_dw(da32, h32),
        "splitk_dw bf16 (rocBLAS default)": lambda: D._splitk_dw(da, hb),
        "mm_dx f32 (tuned)": lambda: D._mm_dx(da32, w1),
        "mm_dx bf16 (rocBLAS default)": lambda: D._mm_dx(da, w1b),
        "torch bf16 mm": lambda: da @ w1b,
        "w1.to(bf16)": lambda: w1.to(bf),
        "heads_block_forward": lambda: _C.heads_block_forward(h32, w1, torch.zeros(kW, device=dev),
                                                              [torch.randn(3, W, device=dev)] * 5,
                                                              [torch.zeros(3, device=dev)] * 5),
        "heads_block_forward_bf16": lambda: _C.heads_block_forward_bf16(h32, w1, torch.zeros(kW, device=dev),
                                                                        [torch.randn(3, W, device=dev)] * 5,
                                                                        [torch.zeros(3, device=dev)] * 5),
    }
    for name, fn in rows.items():
        print(f"{name:36s} {per_call(fn):8.1f} us/call (host)", flush=True)


if __name__ == "__main__":
    main()
