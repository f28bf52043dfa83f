"""dW = dy^T x split-K chunk size sweep (diagnostic, GPU): _splitk_dw at the heads' first-layer shape (P = 100k,
N = 640, K = 128, fp32) for several _LinearSplitK.kChunk values (argv, or a default list), HIP events over R calls."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "4dgaussians-fast-train_amd")]
from gs4d_train import deformation as D  # noqa: E402


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
    P, N, K = 100_000, 640, 128
    torch.manual_seed(0)
    dy = torch.randn(P, N, device="cuda")
    x = torch.relu(torch.randn(P, K, device="cuda"))
    ref = (dy.double().t() @ x.double())
    for c in [int(a) for a in sys.argv[1:]] or (1024, 2048, 4096, 8192, 16384):
        D._LinearSplitK.kChunk = c
        out = D._splitk_dw(dy, x)
        err = float((out.double() - ref).abs().max() / ref.abs().max())
        print(f"kChunk {c:6d}: {timed(lambda: D._splitk_dw(dy, x)):8.1f} us  rel err {err:.2e}", flush=True)
        torch.cuda.synchronize()
        torch.full((7,), 1.0, device="cuda")  # a marker launch: a trace's kernels after it are 10 steady calls
        for _ in range(10):
            D._splitk_dw(dy, x)
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
