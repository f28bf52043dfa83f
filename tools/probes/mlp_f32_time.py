"""Timing + fp64 check of the fp32 heads-block GEMMs: gs4d_mlp_dx_f32 / gs4d_mlp_dw_f32 against rocBLAS's own pick
and the tuned rocBLAS kernel (the round-5 path), at the train step's shapes.  Usage: python tools/probes/mlp_f32_time.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "4dgaussians-fast-train_amd"))
from gs4d_train import _C, deformation as D  # noqa: E402


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return 1e3 * e0.elapsed_time(e1) / reps


for P, KW, W in [(100_000, 640, 128), (100_003, 640, 128), (2000, 192, 64), (300_000, 640, 128)]:
    torch.manual_seed(0)
    da = torch.randn(P, KW, device="cuda")
    h = torch.relu(torch.randn(P, W, device="cuda"))
    w1 = torch.randn(KW, W, device="cuda") / KW ** 0.5
    w1t = w1.t().contiguous()
    dh = _C.mlp_dx_f32(da, w1t)
    dw = _C.mlp_dw_f32(da, h)
    ref_x = da.double() @ w1.double()
    sc_x = da.double().abs() @ w1.double().abs()
    ref_w = da.double().t() @ h.double()
    sc_w = da.double().abs().t() @ h.double().abs()
    ex = float(((dh.double() - ref_x).abs() / sc_x.clamp_min(1e-30)).max())
    ew = float(((dw.double() - ref_w).abs() / sc_w.clamp_min(1e-30)).max())
    flops = 2.0 * P * KW * W
    tx = timeit(lambda: _C.mlp_dx_f32(da, w1t))
    tw = timeit(lambda: _C.mlp_dw_f32(da, h))
    D._TUNE = False
    rx = timeit(lambda: D._mm_dx(da, w1))
    rw = timeit(lambda: D._splitk_dw(da, h))
    D._TUNE = True
    qx = timeit(lambda: D._mm_dx(da, w1))
    qw = timeit(lambda: D._splitk_dw(da, h))
    D._TUNE = False
    same = torch.equal(_C.mlp_dx_f32(da, w1t), dh) and torch.equal(_C.mlp_dw_f32(da, h), dw)
    print(f"P={P} KW={KW} W={W}: dx_f32 {tx:.1f} us ({flops / tx / 1e6:.1f} TF/s, rel err {ex:.2e}) | "
          f"dw_f32 {tw:.1f} us ({flops / tw / 1e6:.1f} TF/s, rel err {ew:.2e}) | rocBLAS own pick dx {rx:.1f} dw {rw:.1f} | "
          f"tuned dx {qx:.1f} dw {qw:.1f} | repeat bitwise {same}", flush=True)
