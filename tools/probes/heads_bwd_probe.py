"""gs4d_heads_backward timing probe (diagnostic, GPU): the DyNeRF heads block (P = 100k, W = 128) with
all five heads, the four narrow ones only (a 4W wide) and the 48-wide one only, against the bytes it
must move (read a, write da)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "4dgaussians-fast-train_amd")]
from gs4d_train import _C  # noqa: E402
from heads_probe import timed  # noqa: E402


def main(P=100_000, W=128):
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    for ns in ([3, 3, 4, 1, 48], [3, 3, 4, 1], [48], [3]):
        k = len(ns)
        a = torch.relu(torch.randn(P, k * W, device=dev))
        gs = [torch.randn(P, n, device=dev) for n in ns]
        w2 = [torch.randn(n, W, device=dev) for n in ns]
        t = timed(lambda: _C.heads_backward(a, gs, w2), reps=30)
        gb = 2 * a.numel() * 4 / 1e9
        print(f"heads {ns}: {t:.1f} us  ({gb / (t * 1e-6) / 1e3:.2f} TB/s on read a + write da)")


if __name__ == "__main__":
    main()
