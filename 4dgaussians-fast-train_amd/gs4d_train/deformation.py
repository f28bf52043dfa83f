"""The HexPlane deformation field that runs before the rasterizer in the fine stage.

Restates scene/hexplane.py and scene/deformation.py of the reference in
PyTorch, module for module, so that a trained reference `deformation.pth` state dict loads into it
unchanged (same parameter names and shapes: `deformation_net.grid.grids.{level}.{plane}`,
`deformation_net.feature_out.*`, `deformation_net.{pos,scales,rotations,opacity,shs}_deform.*`,
`timenet.*`).  The grid interpolation (the field's cost centre) can run either through
`F.grid_sample` exactly as the reference does, or through the fused HIP kernel of libgs4d
(`gs4d_train.kernels.hexplane`), selected by `HexPlaneField.fused`.
"""
import itertools
import os
import warnings
from typing import Sequence

import torch
import torch.nn as nn
import torch.nn.functional as F


def normalize_aabb(pts, aabb):
    """scene/hexplane.py:20-21.  aabb[0] is the MAX corner, aabb[1] the min (set_aabb order)."""
    return (pts - aabb[0]) * (2.0 / (aabb[1] - aabb[0])) - 1.0


def grid_sample_wrapper(grid, coords, align_corners=True):
    """scene/hexplane.py:22-48: bilinear, border padding, (1, F, H, W) grid at (n, 2) coords -> (n, F)."""
    grid_dim = coords.shape[-1]
    if grid.dim() == grid_dim + 1:
        grid = grid.unsqueeze(0)
    if coords.dim() == 2:
        coords = coords.unsqueeze(0)
    coords = coords.view([coords.shape[0]] + [1] * (grid_dim - 1) + list(coords.shape[1:]))
    B, feature_dim = grid.shape[:2]
    n = coords.shape[-2]
    interp = F.grid_sample(grid, coords, align_corners=align_corners, mode="bilinear", padding_mode="border")
    interp = interp.view(B, feature_dim, n).transpose(-1, -2)
    return interp.squeeze()


def init_grid_param(grid_nd, in_dim, out_dim, reso: Sequence[int], a=0.1, b=0.5):
    """scene/hexplane.py:50-72: one (1, out_dim, reso[c1], reso[c0]) plane per coordinate pair;
    planes that involve time (coordinate 3) start at 1, the others uniform in [a, b]."""
    assert in_dim == len(reso)
    has_time_planes = in_dim == 4
    grid_coefs = nn.ParameterList()
    for coo_comb in itertools.combinations(range(in_dim), grid_nd):
        p = nn.Parameter(torch.empty([1, out_dim] + [reso[cc] for cc in coo_comb[::-1]]))
        if has_time_planes and 3 in coo_comb:
            nn.init.ones_(p)
        else:
            nn.init.uniform_(p, a=a, b=b)
        grid_coefs.append(p)
    return grid_coefs


class HexPlaneField(nn.Module):
    """scene/hexplane.py:113-190 (concat_features=True)."""

    def __init__(self, bounds, planeconfig, multires):
        super().__init__()
        aabb = torch.tensor([[bounds, bounds, bounds], [-bounds, -bounds, -bounds]])
        self.aabb = nn.Parameter(aabb, requires_grad=False)
        self.grid_config = [planeconfig]
        self.multiscale_res_multipliers = multires
        self.concat_features = True
        self.grids = nn.ModuleList()
        self.feat_dim = 0
        for res in multires:
            config = dict(self.grid_config[0])
            config["resolution"] = [r * res for r in config["resolution"][:3]] + config["resolution"][3:]
            gp = init_grid_param(config["grid_dimensions"], config["input_coordinate_dim"],
                                 config["output_coordinate_dim"], config["resolution"])
            self.feat_dim += gp[-1].shape[1]
            self.grids.append(gp)
        self.fused = False  # True: the HIP kernel (kernels.hexplane) instead of F.grid_sample

    @property
    def get_aabb(self):
        return self.aabb[0], self.aabb[1]

    def set_aabb(self, xyz_max, xyz_min):
        self.aabb = nn.Parameter(torch.tensor([xyz_max, xyz_min], dtype=torch.float32, device=self.aabb.device),
                                 requires_grad=False)

    def forward(self, pts, timestamps=None, alias=None):
        """get_density (scene/hexplane.py:160-177): normalised (x, y, z, t) -> per-level plane products.
        alias (a list, fused path only): receives a pass-through view of pts for their other use, whose
        gradient the points' backward then sums in (kernels.hexplane_points)."""
        # the fused field differentiates w.r.t. the points only: timestamps that need a gradient take
        # the grid_sample graph
        if (self.fused and pts.is_cuda and pts.dim() == 2 and timestamps is not None and timestamps.dim() == 2
                and not timestamps.requires_grad):
            from .kernels import hexplane, hexplane_points
            return hexplane(hexplane_points(pts, timestamps, self.aabb, alias), [list(g) for g in self.grids])
        pts = normalize_aabb(pts, self.aabb)
        pts = torch.cat((pts, timestamps), dim=-1).reshape(-1, 4)
        if self.fused:
            from .kernels import hexplane
            return hexplane(pts, [list(g) for g in self.grids])
        return interpolate_ms_features(pts, self.grids)


def interpolate_ms_features(pts, ms_grids):
    """scene/hexplane.py:75-110 with concat_features=True, grid_dimensions=2."""
    coo_combs = list(itertools.combinations(range(pts.shape[-1]), 2))
    out = []
    for grid in ms_grids:
        interp_space = 1.0
        for ci, coo_comb in enumerate(coo_combs):
            feature_dim = grid[ci].shape[1]
            interp_space = interp_space * grid_sample_wrapper(grid[ci], pts[..., coo_comb]).view(-1, feature_dim)
        out.append(interp_space)
    return torch.cat(out, dim=-1)


class _LinearSplitK(torch.autograd.Function):
    """F.linear whose weight gradient dW = dY^T X (a (out x in) result reduced over P ~ 1e5 rows) is
    computed as a split-K batched GEMM: the library's default kernel for that tall-skinny reduction
    tiles only the tiny output and runs at ~4-12 TF/s on MI355X (tools/gemm_probe.py); splitting the P
    rows into chunks of kChunk restores ~25-50 TF/s.  Forward, dX and db are unchanged."""

    kChunk = 1024

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        ctx.has_bias = b is not None
        return F.linear(x, w, b)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy = dy.contiguous()
        dx = dy @ w if ctx.needs_input_grad[0] else None
        dw = db = None
        if ctx.needs_input_grad[1]:
            P, c = x.shape[0], _LinearSplitK.kChunk
            S = P // c
            if S >= 2:
                dw = torch.bmm(dy[:S * c].view(S, c, -1).transpose(1, 2), x[:S * c].view(S, c, -1)).sum(0)
                if P > S * c:
                    dw = dw + dy[S * c:].t() @ x[S * c:]
            else:
                dw = dy.t() @ x
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = dy.sum(0)
        return dx, dw, db


class Linear(nn.Linear):
    """nn.Linear (same parameters and state-dict entries) with the split-K weight gradient on GPU."""

    def forward(self, x):
        if x.is_cuda and x.dim() == 2 and torch.is_grad_enabled():
            return _LinearSplitK.apply(x.contiguous(), self.weight, self.bias)
        return F.linear(x, self.weight, self.bias)


# The heads block's two large GEMMs (W in {64, 128}) run on this library's f32-MFMA passes (gs4d_mlp_dw_f32,
# gs4d_mlp_dx_f32): one fixed summation order, so a train step gives the same bits in every process.  The
# shapes those do not serve (W = 256, the bf16 path's W = 64 weight gradient) go to rocBLAS through gemm_f32:
# by default rocBLAS's own pick, which depends only on the shape (the same kernel in every process).
# GS4D_GEMM_TUNE=1 opts into the run-time tuner instead (gemm_f32(..., tune=True) times every solution rocBLAS
# has for a shape class on its first call and keeps the fastest, train_glue.cpp): faster on some shapes, but
# the choice depends on timings, so two processes may run different kernels and round differently.
# _C.gemm_tuned() lists the tuner's choices.


_USE_ROCBLAS = os.environ.get("GS4D_MLP_ROCBLAS", "1") != "0"  # 0: torch's GEMMs (A/B runs)
_TUNE = os.environ.get("GS4D_GEMM_TUNE", "0") == "1"


def _rocblas_ok(*ts):
    """rocBLAS through gemm_f32: device matrices with unit column stride, all f32 or all bf16 (C is f32)."""
    return _USE_ROCBLAS and len({t.dtype for t in ts}) == 1 and ts[0].dtype in (torch.float32, torch.bfloat16) and \
        all(t.is_cuda and t.dim() == 2 and t.stride(1) == 1 for t in ts)


def _chunk_rows(P):
    """The split-K chunk for P rows on rocBLAS: the largest multiple of 8 in [3/4, 2] x kChunk that divides P (no
    remainder GEMM: at P = 100k, 50 chunks of 2000 rows took 162 us per dW where 97 of 1024 plus the 672-row
    remainder took 172, tools/sk_probe.sh), else kChunk and a remainder."""
    c0 = _LinearSplitK.kChunk
    for c in range(2 * c0 - (2 * c0) % 8, (3 * c0) // 4 - 1, -8):
        if P % c == 0:
            return c
    return c0


def _splitk_dw(dy, x):
    """dW = dy^T x reduced over the P rows as a split-K batched GEMM (see _LinearSplitK); x may be a
    column slice of a wider row-major tensor (its rows are then strided).  On the GPU: the chunks' partials
    and the remainder's on rocBLAS (gemm_f32, the tuned kernels above) into one (S + 1, N, K) buffer,
    summed in chunk order by one pass (gs4d_sum_slices) -- the bmm, its .sum(0), the remainder GEMM and
    the add of the torch form in three launches."""
    P, c = x.shape[0], _LinearSplitK.kChunk
    if _rocblas_ok(dy, x):
        c = _chunk_rows(P)
    S = P // c
    if S < 2 and not (_rocblas_ok(dy, x) and P > 0):
        return (dy.t() @ x).float()
    if _rocblas_ok(dy, x):
        from . import _C
        N, K = dy.shape[1], x.shape[1]
        if S < 2:  # one GEMM, f32 out (a bf16 torch GEMM would round the result to bf16)
            out = torch.empty(N, K, device=dy.device)
            _C.gemm_f32(x, dy, out, False, True, K, N, P, x.stride(0), dy.stride(0), K, 1, 0, 0, 0, _TUNE)
            return out
        rem = P - S * c
        parts = torch.empty(S + (1 if rem else 0), N, K, device=dy.device)
        # column-major: part_s^T (K x N) = x_s^T (K x c) . dy_s (c x N)
        _C.gemm_f32(x, dy, parts, False, True, K, N, c, x.stride(0), dy.stride(0), K, S, c * x.stride(0),
                    c * dy.stride(0), N * K, _TUNE)
        if rem:
            _C.gemm_f32(x[S * c:], dy[S * c:], parts[S], False, True, K, N, rem, x.stride(0), dy.stride(0), K, 1,
                        0, 0, 0, _TUNE)
        return _C.sum_slices(parts)
    xs = x[:S * c].unflatten(0, (S, c))
    dw = torch.bmm(dy[:S * c].unflatten(0, (S, c)).transpose(1, 2), xs).sum(0)
    if P > S * c:
        dw = dw + dy[S * c:].t() @ x[S * c:]
    return dw


def _mm_dx(dy, w):
    """dy @ w (P x N)(N x K): the MLP's input gradient; on the GPU rocBLAS with the tuned kernel."""
    if _rocblas_ok(dy, w) and w.is_contiguous() and dy.shape[0] > 0:
        from . import _C
        P, N, K = dy.shape[0], dy.shape[1], w.shape[1]
        out = torch.empty(P, K, device=dy.device)
        # column-major: out^T (K x P) = w^T (K x N) . dy^T (N x P)
        _C.gemm_f32(w, dy, out, False, False, K, P, N, K, dy.stride(0), K, 1, 0, 0, 0, _TUNE)
        return out
    return (dy @ w).float()


_NO_BLOCK_FORWARD = set()  # devices whose LDS cannot hold the heads block forward's weights


def _block_forward_ok(dev):
    return dev.index not in _NO_BLOCK_FORWARD


def _block_forward_unavailable(dev, err):
    """gs4d_heads_block_forward[_bf16] returned GS4D_TRAIN_ERR_LDS (the device cannot give the kernel the
    LDS its weights need): this device uses the GEMM formulation from now on."""
    _NO_BLOCK_FORWARD.add(dev.index)
    warnings.warn(f"heads block forward unavailable on {dev} ({err}); using the GEMM formulation")


class _Stacked(torch.autograd.Function):
    """torch.cat of tensors that already lie back to back in one storage, without the copy: the forward
    returns one view over all of them, the backward hands each its slice of the gradient (views: no
    kernel).  Deformation._pack_heads keeps the heads' first-layer weights and biases so (the parameters
    stay the reference's separate tensors, for state dicts and optimizers)."""

    @staticmethod
    def forward(ctx, *ts):
        ctx.rows = [t.shape[0] for t in ts]
        n = sum(ctx.rows)
        shape = (n,) + tuple(ts[0].shape[1:])
        stride = ts[0].stride()
        return ts[0].as_strided(shape, stride)

    @staticmethod
    def backward(ctx, g):
        return tuple(g.split(ctx.rows, 0))


_STACKED_OK = {}  # (ids of the tensors) -> (their data pointers and row counts) when last found stacked


def _stacked(ts):
    """cat(ts, 0) as a view when the tensors are contiguous and consecutive in one storage, else None.
    The full check runs once per layout: the same tensor objects at the same addresses with the same row counts
    (a moved or replaced .data changes the address) take the cached verdict -- host time every train step."""
    key = tuple(map(id, ts))
    sig = tuple((t.data_ptr(), t.shape[0]) for t in ts)
    if _STACKED_OK.get(key) == sig:
        return _Stacked.apply(*ts)
    t0 = ts[0]
    if not t0.is_contiguous():
        return None
    off = t0.storage_offset()
    for t in ts:
        if not t.is_contiguous() or t.dtype != t0.dtype or t.device != t0.device or t.shape[1:] != t0.shape[1:] \
                or t.untyped_storage().data_ptr() != t0.untyped_storage().data_ptr() or t.storage_offset() != off:
            return None
        off += t.numel()
    if len(_STACKED_OK) > 64:
        _STACKED_OK.clear()
    _STACKED_OK[key] = sig
    return _Stacked.apply(*ts)


class _DeformHeads(torch.autograd.Function):
    """The deformation heads (scene/deformation.py:73-78, each nn.Sequential(ReLU, Linear(W, W), ReLU,
    Linear(W, n)) applied to the same hidden features) evaluated together: one ReLU of the shared
    input, ONE (P x W) @ (W x kW) GEMM for the k first layers (weights concatenated), one ReLU, then
    the k small second layers on column slices.  On the GPU (W in {64, 128}) both layers are one HIP
    pass (gs4d_heads_block_forward) that writes the first layers' output a for the backward and never
    reads it back.  The backward mirrors it: the k (P x n) @ (n x W)
    products land in column slices of one (P x kW) gradient, then one ReLU mask, one GEMM with K = kW
    for the input gradient and one split-K GEMM for the concatenated first-layer weight gradient.  On
    the GPU the second layers' backward, the ReLU mask and the first-layer bias gradient are one HIP
    pass over the first layers' output (gs4d_heads_backward); the PyTorch formulation below it is the
    CPU path (and the narrow heads' dW/db there come from gs4d_linear_dw when on the GPU).
    Same function as the k separate heads (and the same parameters, concatenated per call); the
    GEMMs sum in a different order, so results agree to fp32 rounding."""

    @staticmethod
    def forward(ctx, relu_done, hidden, w1, b1, *second):
        """relu_done: `hidden` is already relu(hidden) (_FeatureReLU); the returned input gradient is
        then the gradient of that ReLU's output."""
        k = len(second) // 2
        W = hidden.shape[1]
        h = hidden if relu_done else torch.relu(hidden)
        if h.is_cuda and W in (64, 128) and k <= 8 and all(t.shape[0] <= 64 for t in second[0::2]) and \
                _block_forward_ok(h.device):
            # both layers in one MFMA pass (gs4d_heads_block_forward): a is written once, for the backward
            from . import _C
            try:
                a, w1t, *outs = _C.heads_block_forward(h.contiguous(), w1.contiguous(), b1.contiguous(),
                                                       [t.contiguous() for t in second[0::2]], list(second[1::2]))
            except RuntimeError as e:
                if "status 4" not in str(e):
                    raise
                _block_forward_unavailable(h.device, e)
            else:
                ctx.save_for_backward(h, a, w1, *second[0::2])
                ctx.w1t = w1t  # W1^T (W, kW), written by the same pass, for the input gradient
                ctx.W = W
                ctx.relu_done = relu_done
                return tuple(outs)
        ctx.w1t = None
        a = torch._addmm_activation(b1, h, w1.t())  # bias + ReLU in the GEMM epilogue where supported
        if a.is_cuda and W in (64, 128, 256) and k <= 8 and all(t.shape[0] <= 64 for t in second[0::2]) and \
                sum(t.shape[0] for t in second[0::2]) * (W + 4) * 4 <= 64 * 1024:
            # the k second layers in one MFMA pass over a (gs4d_heads_forward)
            from . import _C
            outs = _C.heads_forward(a, list(second[0::2]), list(second[1::2]))
        else:
            outs = [torch.addmm(second[2 * i + 1], a[:, i * W:(i + 1) * W], second[2 * i].t()) for i in range(k)]
        ctx.save_for_backward(h, a, w1, *second[0::2])
        ctx.W = W
        ctx.relu_done = relu_done
        return tuple(outs)

    @staticmethod
    def backward(ctx, *douts):
        return (None,) + _DeformHeads._backward(ctx, *douts)

    @staticmethod
    def _backward(ctx, *douts):
        h, a, w1, *w2 = ctx.saved_tensors
        W, k = ctx.W, len(w2)
        relu_in = (lambda d: d) if ctx.relu_done else (lambda d: torch.ops.aten.threshold_backward(d, h, 0))
        douts = [d if d is not None else torch.zeros(a.shape[0], w2[i].shape[0], device=a.device)
                 for i, d in enumerate(douts)]
        if a.is_cuda and W in (64, 128, 256) and k * W <= 768 and all(x.shape[0] <= 16 or (x.shape[0] == 48 and W <= 128)
                                                                        for x in w2):
            # second layers' backward + ReLU mask + first-layer bias gradient in one HIP pass over a
            from . import _C
            out = _C.heads_backward(a, list(douts), [x.contiguous() for x in w2])
            da, db1 = out[0], out[1]
            if W in (64, 128) and da.shape[1] % 64 == 0:
                # the two large GEMMs on hand-written f32-MFMA passes: fixed summation order, the same bits in
                # every process (gs4d_mlp_dw_f32 / gs4d_mlp_dx_f32)
                dw1 = _C.mlp_dw_f32(da, h.contiguous())
                w1t = ctx.w1t if ctx.w1t is not None else w1.t().contiguous()
                dh = relu_in(_C.mlp_dx_f32(da, w1t))
            else:
                dw1 = _splitk_dw(da, h)
                dh = relu_in(_mm_dx(da, w1))
            return tuple([dh, dw1, db1] + out[2:])
        da = torch.empty_like(a)
        dw2, db2 = [None] * k, [None] * k
        small = []  # heads whose (dw, db) one gs4d_linear_dw launch forms (n <= 8)
        for i in range(k):
            do = douts[i].contiguous()
            sl = a[:, i * W:(i + 1) * W]
            torch.mm(do, w2[i], out=da[:, i * W:(i + 1) * W])
            if do.shape[1] <= 8 and W in (64, 128, 256):
                small.append((i, do, sl))
            else:
                dw2[i], db2[i] = _splitk_dw(do, sl), do.sum(0)
        if small:
            from . import _C
            out = _C.linear_dw([d for _, d, _ in small], [x for _, _, x in small])
            for j, (i, _, _) in enumerate(small):
                dw2[i], db2[i] = out[2 * j], out[2 * j + 1]
        da = torch.ops.aten.threshold_backward(da, a, 0)  # ReLU backward (a = relu(z): a > 0 <=> z > 0)
        dw1 = _splitk_dw(da, h)
        db1 = da.sum(0)
        dh = relu_in(da @ w1)  # the heads' first ReLU
        grads = [dh, dw1, db1]
        for i in range(k):
            grads += [dw2[i], db2[i]]
        return tuple(grads)


def _sum0_f32(parts):
    """parts (S, ...) -> their sum over S in fp32, as a (1 x S) @ (S x N) GEMM (torch's reduction over
    a leading dimension of a few dozen rows is far slower here)."""
    S = parts.shape[0]
    flat = parts.reshape(S, -1).float()
    return (torch.ones(1, S, device=parts.device) @ flat).view(parts.shape[1:])


def _splitk_dw_bf16(dy, x):
    """dy^T x over the P rows on bf16 operands (fp32 accumulate inside each chunk): split-K batched
    GEMM (see _LinearSplitK for why), the chunk partials summed in fp32."""
    P, c = x.shape[0], _LinearSplitK.kChunk
    S = P // c
    if S < 2:
        return (dy.t() @ x).float()
    dw = _sum0_f32(torch.bmm(dy[:S * c].unflatten(0, (S, c)).transpose(1, 2), x[:S * c].unflatten(0, (S, c))))
    if P > S * c:
        dw = dw + (dy[S * c:].t() @ x[S * c:]).float()
    return dw


def _colsum(x):
    """x (P, n) -> its column sums (n,) in fp32: chunks of kChunk rows reduced over their middle dimension
    (a contiguous-inner reduction), then the chunk partials (no N = 1 GEMM: hipBLASLt's host-side
    heuristics for that shape cost milliseconds per call)."""
    P, c = x.shape[0], _LinearSplitK.kChunk
    S = P // c
    out = x[:S * c].unflatten(0, (S, c)).sum(1, dtype=torch.float32).sum(0) if S else 0
    if P > S * c:
        out = out + x[S * c:].sum(0, dtype=torch.float32)
    return out


class _DeformHeadsBF16(torch.autograd.Function):
    """The opt-in bf16 form of _DeformHeads (hyper.mlp_dtype = "bf16", BASELINE C3's bf16 leg): the same
    block on bf16 operands with fp32 accumulation; parameters, their gradients and the heads' outputs stay
    fp32.  On the GPU (W in {64, 128}, n_i <= 16 or 48) every piece is a HIP bf16-MFMA kernel:
      forward   gs4d_heads_block_forward_bf16: both layers on v_mfma_f32_16x16x32_bf16 in one pass, a =
                relu(h W1^T + b1) written once in bf16 (half the fp32 block's bytes) with h and W1^T in bf16
                for the backward;
      backward  gs4d_heads_backward_bf16: the second layers' backward, the ReLU mask and db1 in one pass
                over a (da in bf16, sums fp32); dW1 = da^T h by gs4d_mlp_dw_bf16 and dh = da W1 by
                gs4d_mlp_dx_bf16 (f32 out; rocBLAS bf16 GEMMs for widths those do not serve).
    Rounding: h, W1, W2, a and da are rounded to bf16 once each (tests/test_train_gpu.py bounds the effect
    on a train step against the fp32 path).  Elsewhere (CPU, other widths) the same function in torch bf16
    ops: _torch_forward / _torch_backward."""

    @staticmethod
    def _fast(h, second):
        W, w2 = h.shape[1], second[0::2]
        return h.is_cuda and W in (64, 128) and len(w2) <= 8 and _block_forward_ok(h.device) and \
            all(t.shape[0] <= 16 or t.shape[0] == 48 for t in w2)

    @staticmethod
    def forward(ctx, h, hb_in, w1, b1, *second):
        """h: relu already applied (every head starts with ReLU; _FeatureReLU).  hb_in: h rounded to bf16 by
        _FeatureReLUHB, or None (the kernel then rounds h itself)."""
        ctx.W = h.shape[1]
        if _DeformHeadsBF16._fast(h, second):
            from . import _C
            try:
                a, hb, w1t, *outs = _C.heads_block_forward_bf16(h.contiguous(), w1.contiguous(), b1.contiguous(),
                                                           [t.contiguous() for t in second[0::2]],
                                                           [t.contiguous() for t in second[1::2]], hb=hb_in)
            except RuntimeError as e:
                if "status 4" not in str(e):
                    raise
                _block_forward_unavailable(h.device, e)
            else:
                ctx.fast = True
                ctx.save_for_backward(hb, a, w1t, *second[0::2])
                return tuple(outs)
        ctx.fast = False
        return _DeformHeadsBF16._torch_forward(ctx, h, w1, b1, *second)

    @staticmethod
    def backward(ctx, *douts):
        if not ctx.fast:
            return _DeformHeadsBF16._torch_backward(ctx, *douts)
        from . import _C
        hb, a, w1t, *w2 = ctx.saved_tensors
        douts = [d if d is not None else torch.zeros(a.shape[0], w2[i].shape[0], device=a.device)
                 for i, d in enumerate(douts)]
        out = _C.heads_backward(a, list(douts), [x.contiguous() for x in w2])
        da, db1 = out[0], out[1]                       # da (P, kW) bf16, masked by the first ReLU
        # (kW, W) fp32: gs4d_mlp_dw_bf16 (bf16 MFMA, LDS transpose reads) for W = 128, else rocBLAS split-K
        dw1 = _C.mlp_dw_bf16(da, hb) if hb.shape[1] == 128 and da.shape[1] % 128 == 0 else _splitk_dw(da, hb)
        # (P, W) fp32: gs4d_mlp_dx_bf16 (bf16 MFMA) when KW is a multiple of its 64-wide k chunk
        dh = _C.mlp_dx_bf16(da, w1t) if da.shape[1] % 64 == 0 else _mm_dx(da, w1t.t().contiguous())
        return tuple([dh, None, dw1, db1] + out[2:])

    @staticmethod
    def _torch_forward(ctx, h, w1, b1, *second):
        bf = torch.bfloat16
        k = len(second) // 2
        W = h.shape[1]
        hb = h.to(bf)
        w1b = w1.to(bf)
        a = torch._addmm_activation(b1.to(bf), hb, w1b.t())  # (P, kW) bf16, relu(h w1^T + b1)
        w2b = [second[2 * i].to(bf) for i in range(k)]
        outs = [torch.addmm(second[2 * i + 1].to(bf), a[:, i * W:(i + 1) * W], w2b[i].t()).float() for i in range(k)]
        ctx.save_for_backward(hb, a, w1b, *w2b)
        return tuple(outs)

    @staticmethod
    def _torch_backward(ctx, *douts):
        bf = torch.bfloat16
        hb, a, w1b, *w2b = ctx.saved_tensors
        W, k = ctx.W, len(w2b)
        P = a.shape[0]
        ns = [x.shape[0] for x in w2b]
        do32 = torch.cat([d if d is not None else torch.zeros(P, n, device=a.device) for d, n in zip(douts, ns)], 1)
        do = do32.to(bf)
        da = torch.ops.aten.threshold_backward(do @ torch.block_diag(*w2b), a, 0)  # (P, kW) bf16
        dw2full = _splitk_dw_bf16(do, a)                                            # keep the diagonal blocks
        db2full = _colsum(do32)
        grads2, o = [], 0
        for i in range(k):
            grads2 += [dw2full[o:o + ns[i], i * W:(i + 1) * W].contiguous(), db2full[o:o + ns[i]]]
            o += ns[i]
        dw1 = _splitk_dw_bf16(da, hb)
        db1 = _colsum(da)
        dh = (da @ w1b).float()
        return tuple([dh, None, dw1, db1] + grads2)  # None: hb_in


class _FeatureReLU(torch.autograd.Function):
    """feature_out with defor_depth <= 1 (scene/deformation.py:51-55: ONE Linear(feat_dim, W)) followed by
    the ReLU every head starts with (:73-78): h = relu(x W^T + b) in one f32-MFMA pass (gs4d_feature_relu_forward).
    Backward in one HIP pass on the f32 MFMA (gs4d_feature_relu_backward): the ReLU mask, dx = dz W,
    dW = dz^T x and db.  Same function as Linear + ReLU (the sums run in another order: fp32 rounding)."""

    shapes = ((32, 128), (64, 64), (32, 64))  # (feat_dim, W) the HIP backward is built for

    @staticmethod
    def forward(ctx, x, w, b):
        from . import _C
        h = _C.feature_relu_forward(x, w.contiguous(), b.contiguous())[0]  # one f32-MFMA pass, bias + ReLU fused
        ctx.save_for_backward(x, w, h)
        return h

    @staticmethod
    def backward(ctx, g):
        x, w, h = ctx.saved_tensors
        from . import _C
        dx, dw, db = _C.feature_relu_backward(g, h, x, w)
        return dx, dw, db


class _FeatureReLUHB(_FeatureReLU):
    """_FeatureReLU that also returns h rounded to bf16 (gs4d_feature_relu_forward_hb, the same pass): the bf16
    heads block reads it instead of converting h once per head.  The bf16 copy carries no gradient."""

    @staticmethod
    def forward(ctx, x, w, b):
        from . import _C
        h, hb = _C.feature_relu_forward(x, w.contiguous(), b.contiguous(), with_hb=True)
        ctx.save_for_backward(x, w, h)
        ctx.mark_non_differentiable(hb)
        ctx.set_materialize_grads(False)  # no zero-filled (P, W) bf16 gradient for hb in the backward
        return h, hb

    @staticmethod
    def backward(ctx, g, ghb):
        if g is None:
            return None, None, None
        return _FeatureReLU.backward(ctx, g)


class Deformation(nn.Module):
    """scene/deformation.py:16-172 (no_grid=False, grid_pe=0, empty_voxel=False, static_mlp=False)."""

    def __init__(self, D=8, W=256, args=None):
        super().__init__()
        self.D, self.W, self.args = D, W, args
        self.grid = HexPlaneField(args.bounds, args.kplanes_config, args.multires)
        self.feature_out = [Linear(self.grid.feat_dim, W)]
        for _ in range(D - 1):
            self.feature_out += [nn.ReLU(), Linear(W, W)]
        self.feature_out = nn.Sequential(*self.feature_out)
        head = lambda n: nn.Sequential(nn.ReLU(), Linear(W, W), nn.ReLU(), Linear(W, n))
        self.pos_deform, self.scales_deform, self.rotations_deform = head(3), head(3), head(4)
        self.opacity_deform, self.shs_deform = head(1), head(16 * 3)
        self.fused_heads = False  # True: the heads as one _DeformHeads block (GPU training)
        # "bf16" (opt-in, GPU): the heads block (the MLP's FLOPs) runs on bf16 operands with fp32
        # accumulation (_DeformHeadsBF16); feature_out (K = feat_dim, a few % of the FLOPs) stays fp32, as do
        # parameters, their gradients and the heads' outputs (BASELINE C3's "bf16/fp32" train loop).
        # "fp32" (default) is the reference's precision.
        self.mlp_dtype = getattr(args, "mlp_dtype", "fp32")

    def deltas(self, xyz, time, alias=None):
        """The active heads' outputs {name: (P, n)} of forward_dynamic (scene/deformation.py:97-139),
        before the residual adds (which gs4d_train.kernels.deform_tail fuses with the activations).
        alias (a list): may receive a pass-through view of xyz to use in those adds (HexPlaneField.forward)."""
        a = self.args
        if a.apply_rotation and not a.no_dr:
            raise NotImplementedError("apply_rotation (documented as unused in arguments/__init__.py:104)")
        xyz = xyz if xyz.shape[1] == 3 else xyz[:, :3]
        time = time if time.shape[1] == 1 else time[:, :1]
        active = [name for name, flag in (("pos_deform", a.no_dx), ("scales_deform", a.no_ds),
                                          ("rotations_deform", a.no_dr), ("opacity_deform", a.no_do),
                                          ("shs_deform", a.no_dshs)) if not flag]
        return self._heads(self.grid(xyz, time, alias) if alias is not None else self.grid(xyz, time), active)

    def _heads_bf16(self, feat, active):
        """The bf16 form of _heads: feature_out and its ReLU as on the fp32 path (a K = feat_dim layer,
        cheap), then the heads block on bf16 operands (_DeformHeadsBF16).  The heads' outputs (the
        deltas) are fp32, as are all parameters and gradients."""
        lin = self.feature_out[0]
        hb = None
        if len(self.feature_out) == 1 and (feat.shape[1], self.W) in _FeatureReLU.shapes and torch.is_grad_enabled():
            # h and its bf16 copy in one pass; the heads block reads the copy (half the bytes per head)
            h, hb = _FeatureReLUHB.apply(feat.contiguous(), lin.weight, lin.bias)
        else:
            h = torch.relu(self.feature_out(feat))  # every head starts with ReLU (scene/deformation.py:73-78)
        heads = [getattr(self, name) for name in active]
        w1, b1 = self._first_layers(heads)
        second = [t for hd in heads for t in (hd[3].weight, hd[3].bias)]
        return dict(zip(active, _DeformHeadsBF16.apply(h.contiguous(), hb, w1, b1, *second)))

    def _pack_heads(self, heads):
        """Lay the given (active) heads' first-layer weights (and biases) back to back in one storage, in that
        order, each parameter a view of its slice (same Parameter objects, so optimizers and state dicts are
        untouched): the heads block then takes them as one (kW x W) operand with no per-step cat (_stacked).
        Re-done whenever a move, load or surgery has given a parameter its own storage again."""
        for attr in ("weight", "bias"):
            ps = [hd[1].__getattr__(attr) for hd in heads]
            with torch.no_grad():
                big = torch.cat([p.data for p in ps], 0)
                o = 0
                for p in ps:
                    n = p.shape[0]
                    p.data = big[o:o + n]
                    o += n

    def _first_layers(self, heads):
        """(cat of the heads' first-layer weights, of their biases): views when the storage is packed."""
        ws = [hd[1].weight for hd in heads]
        bs = [hd[1].bias for hd in heads]
        w1, b1 = _stacked(ws), _stacked(bs)
        if (w1 is None or b1 is None) and ws[0].is_cuda:
            # only the active heads, in their order: any subset then stacks (packing all five left a
            # non-contiguous subset, e.g. no_do without no_dshs, re-packing and falling back to cat every step)
            self._pack_heads(heads)
            w1, b1 = _stacked(ws), _stacked(bs)
        if w1 is None or b1 is None:
            return torch.cat(ws, 0), torch.cat(bs, 0)
        return w1, b1

    def _heads(self, feat, active):
        """{name: head output} of the active heads on the field features (feature_out, then the heads)."""
        if self.mlp_dtype == "bf16" and feat.is_cuda and active:
            return self._heads_bf16(feat, active)
        if self.fused_heads and feat.is_cuda and torch.is_grad_enabled() and active:
            heads = [getattr(self, name) for name in active]
            w1, b1 = self._first_layers(heads)
            second = [t for hd in heads for t in (hd[3].weight, hd[3].bias)]
            lin = self.feature_out[0]
            if len(self.feature_out) == 1 and (feat.shape[1], self.W) in _FeatureReLU.shapes:
                h = _FeatureReLU.apply(feat.contiguous(), lin.weight, lin.bias)
                return dict(zip(active, _DeformHeads.apply(True, h, w1, b1, *second)))
            return dict(zip(active, _DeformHeads.apply(False, self.feature_out(feat), w1, b1, *second)))
        hidden = self.feature_out(feat)
        return {name: getattr(self, name)(hidden) for name in active}

    def forward(self, xyz, scales, rotations, opacity, shs, time):
        """forward_dynamic (scene/deformation.py:97-146); mask = 1 (no static_mlp / empty_voxel)."""
        a = self.args
        if a.apply_rotation and not a.no_dr:
            raise NotImplementedError("apply_rotation (documented as unused in arguments/__init__.py:104)")
        # the inputs' leading columns (xyz[:, :3], ...) are the whole tensors here: no slicing, so
        # autograd records no slice nodes
        xyz, scales, rotations, opacity = (t if t.shape[1] == n else t[:, :n] for t, n in
                                           ((xyz, 3), (scales, 3), (rotations, 4), (opacity, 1)))
        time = time if time.shape[1] == 1 else time[:, :1]
        active = [name for name, flag in (("pos_deform", a.no_dx), ("scales_deform", a.no_ds),
                                          ("rotations_deform", a.no_dr), ("opacity_deform", a.no_do),
                                          ("shs_deform", a.no_dshs)) if not flag]
        outs = self._heads(self.grid(xyz, time), active)
        pts = xyz if a.no_dx else xyz + outs["pos_deform"]
        sc = scales if a.no_ds else scales + outs["scales_deform"]
        rot = rotations if a.no_dr else rotations + outs["rotations_deform"]
        op = opacity if a.no_do else opacity + outs["opacity_deform"]
        sh = shs if a.no_dshs else shs + outs["shs_deform"].reshape([shs.shape[0], 16, 3])
        return pts, sc, rot, op, sh

    def get_mlp_parameters(self):
        return [p for n, p in self.named_parameters() if "grid" not in n]

    def get_grid_parameters(self):
        return [p for n, p in self.named_parameters() if "grid" in n]


class DeformNetwork(nn.Module):
    """deform_network (scene/deformation.py:173-234).  The reference computes positional encodings of
    the inputs (poc_fre) but its Deformation only reads their raw leading columns, so they are not
    materialised here; the (unused) timenet is kept so state dicts match."""

    def __init__(self, args):
        super().__init__()
        times_ch = 2 * args.timebase_pe + 1
        self.timenet = nn.Sequential(nn.Linear(times_ch, args.timenet_width), nn.ReLU(),
                                     nn.Linear(args.timenet_width, args.timenet_output))
        self.deformation_net = Deformation(W=args.net_width, D=args.defor_depth, args=args)
        self.register_buffer("time_poc", torch.FloatTensor([(2 ** i) for i in range(args.timebase_pe)]))
        self.register_buffer("pos_poc", torch.FloatTensor([(2 ** i) for i in range(args.posebase_pe)]))
        self.register_buffer("rotation_scaling_poc", torch.FloatTensor([(2 ** i) for i in range(args.scale_rotation_pe)]))
        self.register_buffer("opacity_poc", torch.FloatTensor([(2 ** i) for i in range(args.opacity_pe)]))
        self.apply(initialize_weights)

    @property
    def get_aabb(self):
        return self.deformation_net.grid.get_aabb

    def forward(self, point, scales=None, rotations=None, opacity=None, shs=None, times_sel=None):
        return self.deformation_net(point, scales, rotations, opacity, shs, times_sel)

    def deltas(self, point, times_sel, alias=None):
        return self.deformation_net.deltas(point, times_sel, alias)

    def get_mlp_parameters(self):
        return self.deformation_net.get_mlp_parameters() + list(self.timenet.parameters())

    def get_grid_parameters(self):
        return self.deformation_net.get_grid_parameters()


def initialize_weights(m):
    """scene/deformation.py:236-242: xavier-uniform weights (the bias keeps nn.Linear's default)."""
    if isinstance(m, nn.Linear):
        nn.init.xavier_uniform_(m.weight, gain=1)
