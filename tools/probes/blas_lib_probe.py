"""Diagnostic (GPU): the train step's three W x 5W f32 GEMMs at P = 100k, W = 128 under each BLAS backend
torch offers on ROCm (hipBLASLt vs rocBLAS), and the split-K chunk of the weight gradient."""
import time

import torch

P, W, K5 = 100_000, 128, 640
dev = "cuda"


def tm(f, n=20):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e6


h = torch.randn(P, W, device=dev)
w1 = torch.randn(K5, W, device=dev)
b1 = torch.randn(K5, device=dev)
da = torch.randn(P, K5, device=dev)
fl = 2 * P * W * K5
for lib in ("cublaslt", "cublas"):
    try:
        torch.backends.cuda.preferred_blas_library(lib)
    except Exception as e:  # noqa: BLE001
        print(lib, "unavailable", e)
        continue
    r = {"fwd addmm_act": tm(lambda: torch._addmm_activation(b1, h, w1.t())),
         "dh da@w1": tm(lambda: da @ w1)}
    for c in (512, 1024, 2048, 4096):
        S = P // c

        def dw(c=c, S=S):
            return torch.bmm(da[:S * c].unflatten(0, (S, c)).transpose(1, 2), h[:S * c].unflatten(0, (S, c))).sum(0)
        r[f"dW splitK c={c}"] = tm(dw)
    r["dW da.T@h"] = tm(lambda: da.t() @ h)
    print(lib, {k: f"{v:.0f}us {fl / v / 1e6:.0f}TF" for k, v in r.items()}, flush=True)
