"""Deformation-heads timing probe (diagnostic, GPU): the _DeformHeads block at P = 100k, W = 128,
heads n = (3, 3, 4, 1, 48), forward and forward+backward, and the second layers' share of it."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "4dgaussians-fast-train_amd")]
from gs4d_train.deformation import _DeformHeads, _splitk_dw  # noqa: E402


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


def main(P=100_000, W=128):
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    ns = [3, 3, 4, 1, 48]
    hid = torch.randn(P, W, device=dev, requires_grad=True)
    w1 = torch.randn(5 * W, W, device=dev, requires_grad=True)
    b1 = torch.randn(5 * W, device=dev, requires_grad=True)
    second = []
    for n in ns:
        second += [torch.randn(n, W, device=dev, requires_grad=True), torch.randn(n, device=dev, requires_grad=True)]
    ups = [torch.randn(P, n, device=dev) for n in ns]

    def fwd():
        with torch.no_grad():
            return _DeformHeads.apply(False, hid, w1, b1, *second)

    def fwdbwd():
        outs = _DeformHeads.apply(False, hid, w1, b1, *second)
        torch.autograd.backward(outs, ups)

    a = torch.relu(torch.randn(P, 5 * W, device=dev))

    @torch.no_grad()
    def second_fwd():
        return [torch.addmm(second[2 * i + 1], a[:, i * W:(i + 1) * W], second[2 * i].t()) for i in range(5)]

    da = torch.empty_like(a)

    @torch.no_grad()
    def second_bwd():
        for i in range(5):
            torch.mm(ups[i], second[2 * i], out=da[:, i * W:(i + 1) * W])
            _splitk_dw(ups[i], a[:, i * W:(i + 1) * W])
            ups[i].sum(0)

    w2 = [second[2 * i].detach() for i in range(5)]
    dy = torch.cat(ups, 1)
    bd = torch.block_diag(*w2)

    @torch.no_grad()
    def part(which):
        for i in range(5):
            sl = a[:, i * W:(i + 1) * W]
            if which == "mm_slices":
                torch.mm(ups[i], w2[i], out=da[:, i * W:(i + 1) * W])
            elif which == "mm_contig":
                ups[i] @ w2[i]
            elif which == "splitk":
                _splitk_dw(ups[i], sl)
            elif which == "plain_dw":
                ups[i].t() @ sl
            elif which == "sum":
                ups[i].sum(0)

    for w in ("mm_slices", "mm_contig", "splitk", "plain_dw", "sum"):
        print(f"  second-layer backward part {w}: {timed(lambda: part(w)):.1f} us")
    print(f"  block-diagonal da: {timed(lambda: dy @ bd):.1f} us; dw: {timed(lambda: _splitk_dw(dy, a)):.1f} us")
    print(f"heads forward: {timed(fwd):.1f} us; forward+backward: {timed(fwdbwd):.1f} us")
    print(f"second layers: forward {timed(second_fwd):.1f} us, backward {timed(second_bwd):.1f} us")


if __name__ == "__main__":
    main()
