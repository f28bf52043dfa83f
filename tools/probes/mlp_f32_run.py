"""A short run of the fp32 heads-block GEMM kernels (gs4d_mlp_dx_f32 / gs4d_mlp_dw_f32) at the train step's
shape, for rocprofv3 kernel traces and PMC passes.  Usage: python tools/probes/mlp_f32_run.py [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "4dgaussians-fast-train_amd"))
from gs4d_train import _C  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
torch.manual_seed(0)
P, KW, W = 100_000, 640, 128
da = torch.randn(P, KW, device="cuda")
h = torch.relu(torch.randn(P, W, device="cuda"))
w1 = torch.randn(KW, W, device="cuda") / KW ** 0.5
w1t = w1.t().contiguous()
for _ in range(reps):
    _C.mlp_dx_f32(da, w1t)
    _C.mlp_dw_f32(da, h)
torch.cuda.synchronize()
print("done")
