"""Split-K weight-gradient timing probe (diagnostic, GPU): dW = dy^T x over P = 100k rows as
gs4d_train.deformation._splitk_dw does it, for several chunk sizes and output widths."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "4dgaussians-fast-train_amd")]
from gs4d_train.deformation import _LinearSplitK, _splitk_dw  # noqa: E402
from heads_probe import timed  # noqa: E402


def main(P=100_000):
    dev = torch.device("cuda:0")
    x = torch.randn(P, 128, device=dev)
    xw = torch.randn(P, 640, device=dev)
    for n in (1, 3, 48, 128, 640):
        dy = torch.randn(P, n, device=dev)
        row = []
        for c in (512, 1024, 2048, 4096, 8192):
            _LinearSplitK.kChunk = c
            row.append(f"{c}: {timed(lambda: _splitk_dw(dy, x)):.1f}")
        print(f"n={n:4d} (x: P x 128)  " + "  ".join(row) + " us")
    _LinearSplitK.kChunk = 1024


if __name__ == "__main__":
    main()
