"""Linear weight-gradient probe (diagnostic, GPU): gs4d_linear_dw (dw = dy^T x and db = dy.sum(0) in one
pass over the rows) against the split-K GEMM + sum the heads block uses, at P = 100k, for the head widths
n = 1, 3, 4, 48 (x a 128-column slice of a 640-wide matrix) and the feature layer (n = 64, x P x 32)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "4dgaussians-fast-train_amd")]
from gs4d_train import _C  # noqa: E402
from gs4d_train.deformation import _splitk_dw  # noqa: E402
from heads_probe import timed  # noqa: E402


def main(P=100_000):
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    a = torch.relu(torch.randn(P, 640, device=dev))
    feat = torch.randn(P, 32, device=dev)
    cases = [(1, a[:, 128:256]), (3, a[:, :128]), (4, a[:, 256:384]), (48, a[:, 512:]), (16, a[:, :128])]
    for n, x in cases:
        dy = torch.randn(P, n, device=dev)
        dw, db = _C.linear_dw([dy], [x])
        rw, rb = (dy.double().t() @ x.double()), dy.double().sum(0)
        ew = float((dw.double() - rw).abs().max() / rw.abs().max())
        eb = float((db.double() - rb).abs().max() / rb.abs().max())
        t_new = timed(lambda: _C.linear_dw([dy], [x]))
        t_old = timed(lambda: (_splitk_dw(dy, x), dy.sum(0)))
        print(f"n={n:3d} W={x.shape[1]:3d}: linear_dw {t_new:6.1f} us  splitk+sum {t_old:6.1f} us  "
              f"rel err dw {ew:.1e} db {eb:.1e}")
    ns = [3, 3, 4, 1, 48]
    dys = [torch.randn(P, n, device=dev) for n in ns]
    xs = [a[:, i * 128:(i + 1) * 128] for i in range(5)]
    outs = _C.linear_dw(dys, xs)
    err = 0.0
    for i in range(5):
        rw, rb = dys[i].double().t() @ xs[i].double(), dys[i].double().sum(0)
        err = max(err, float((outs[2 * i].double() - rw).abs().max() / rw.abs().max()),
                  float((outs[2 * i + 1].double() - rb).abs().max() / rb.abs().max()))
    t_new = timed(lambda: _C.linear_dw(dys, xs))
    t_small = timed(lambda: _C.linear_dw(dys[:4], xs[:4]))
    t_old = timed(lambda: [(_splitk_dw(d, x), d.sum(0)) for d, x in zip(dys, xs)])
    print(f"5 heads in one launch: {t_new:.1f} us (4 small heads {t_small:.1f} us); split-K + sums: {t_old:.1f} us; "
          f"max rel err {err:.1e}")


if __name__ == "__main__":
    main()
