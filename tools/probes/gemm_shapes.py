"""hipBLASLt timing of the heads-block GEMM shapes (P = 100k rows, W = 128, kW = 640) in the layouts
torch can express, to pick the fastest formulation (GPU diagnostic)."""
import torch

P, W, KW = 100_000, 128, 640
dev = torch.device("cuda:0")
torch.manual_seed(0)
h = torch.randn(P, W, device=dev)
w1 = torch.randn(KW, W, device=dev) * 0.05
b1 = torch.randn(KW, device=dev)
da = torch.randn(P, KW, device=dev)
hT = h.t().contiguous()
daT = da.t().contiguous()


def bench(name, fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / n
    print(f"{name:48s} {ms * 1e3:8.1f} us  {2 * P * W * KW / ms / 1e9:6.1f} TFLOP/s", flush=True)


bench("fwd addmm_act(b1, h, w1.t())", lambda: torch._addmm_activation(b1, h, w1.t()))
bench("fwd addmm(b1, h, w1.t())", lambda: torch.addmm(b1, h, w1.t()))
bench("fwd mm(h, w1.t())", lambda: torch.mm(h, w1.t()))
bench("fwd (w1 @ hT) -> (kW, P)", lambda: torch.mm(w1, hT))
bench("fwd addmm(b1[:,None], w1, hT)", lambda: torch.addmm(b1[:, None], w1, hT))
bench("bwd dh = da @ w1", lambda: torch.mm(da, w1))
bench("bwd dh^T = w1.t() @ da.t()", lambda: torch.mm(w1.t(), da.t()))
bench("bwd dh^T = w1.t() @ daT", lambda: torch.mm(w1.t(), daT))
bench("bwd dw1 = da.t() @ h", lambda: torch.mm(da.t(), h))
bench("bwd dw1 = daT @ h", lambda: torch.mm(daT, h))
c = 4096
S = P // c
bench("bwd dw1 splitK bmm(c=4096)", lambda: torch.bmm(da[:S * c].view(S, c, -1).transpose(1, 2), h[:S * c].view(S, c, -1)).sum(0))
c2 = 8192
S2 = P // c2
bench("bwd dw1 splitK bmm(c=8192)", lambda: torch.bmm(da[:S2 * c2].view(S2, c2, -1).transpose(1, 2), h[:S2 * c2].view(S2, c2, -1)).sum(0))
bench("bwd dw1 splitK bmm(c=2048)", lambda: torch.bmm(da[:48 * 2048].view(48, 2048, -1).transpose(1, 2), h[:48 * 2048].view(48, 2048, -1)).sum(0))
