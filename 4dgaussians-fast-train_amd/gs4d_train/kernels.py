"""Torch-facing wrappers of libgs4d's train-step kernels (include/gs4d_train.h, csrc/train_tail.hip).

Importing this module loads the in-tree `gs4d_train._C` extension and fails loudly when it is not
built: there is no silent torch fallback here.  (The reference's torch formulations live in the
callers -- GaussianModel(fused=False), losses.l1_loss_torch -- and serve the parity tests.)
"""
import math

import torch
import torch.optim.optimizer as _optim_mod

from . import _C

__all__ = ["deform_tail", "l1_loss", "densify_stats", "FusedAdam", "hexplane", "hexplane_points", "set_deterministic", "hexplane_regulation", "hexplane_regulation_value",
           "hexplane_regulation_accumulate_grad"]


class _L1Loss(torch.autograd.Function):
    """utils/loss_utils.py:20-21 |x - y|.mean() in one pass; backward = sign(x - y) / N * dL/dloss."""

    @staticmethod
    def forward(ctx, x, y):
        loss, sign = _C.l1_forward(x, y)
        ctx.save_for_backward(sign)
        ctx.x_dtype = x.dtype
        return loss

    @staticmethod
    def backward(ctx, grad_out):
        (sign,) = ctx.saved_tensors
        return _C.l1_backward(sign, grad_out.reshape(1)).to(ctx.x_dtype), None


def l1_loss(network_output, gt):
    """Drop-in for utils/loss_utils.l1_loss; the ground truth receives no gradient (as in training)."""
    return _L1Loss.apply(network_output, gt.detach())


def l1_loss_and_grad(network_output, gt, dloss=1.0):
    """(detached L1 value, its gradient w.r.t. network_output for the upstream gradient `dloss`) in one pass
    (gs4d_l1_loss_grad): bitwise what l1_loss(...).backward(dloss) deposits, without the sign buffer and
    the autograd node.  Falls back to the two-pass form when numel % 4 != 0."""
    x, y = network_output.detach(), gt.detach()
    if x.numel() % 4 == 0:
        return _C.l1_loss_grad(x, y, float(dloss))
    loss, sign = _C.l1_forward(x, y)
    return loss, _C.l1_backward(sign, torch.full((1,), float(dloss), device=x.device)).to(x.dtype)


@torch.no_grad()
def densify_stats(viewspace_grad, visibility, radii, grad_accum, denom, max_radii2D):
    """train.py:346-349 + gaussian_model.py:521-523 in one launch, in place.  visibility None: the mask is
    radii > 0 (train.py's definition of it), evaluated inside the launch."""
    e = torch.empty(0, dtype=torch.int32, device=viewspace_grad.device)
    r = radii if radii is not None else e
    v = visibility if visibility is not None else e.bool()
    _C.densify_stats(viewspace_grad.contiguous(), v, r, grad_accum, denom, max_radii2D)


class FusedAdam(torch.optim.Optimizer):
    """torch.optim.Adam (no weight decay / amsgrad / maximize) with the whole update in ONE launch.

    Keeps torch.optim.Adam's param_groups and per-parameter state layout ({"step", "exp_avg",
    "exp_avg_sq"}), so scene/gaussian_model.py's optimizer-state surgery (replace / prune / cat of
    exp_avg and exp_avg_sq, :316-388) works on it unchanged.  The per-tensor scalars are formed in
    double precision exactly as torch's multi-tensor path does (torch/optim/adam.py
    _multi_tensor_adam): step_size = -lr / (1 - beta1^step), sqrt(1 - beta2^step).
    """

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps))
        # Host-side step counts keyed by the identity of each state's "step" tensor (which the reference's
        # optimizer-state surgery, gaussian_model.py:316-388, carries from a replaced parameter to its
        # successor).  A torch add on each of ~50 CPU step tensors plus a .item() read cost ~0.45 ms of host
        # time per step (the GPU idled behind it); the count is kept here and written through a numpy view
        # of the tensor (the tensor stays current for any reader).  A step tensor the cache has not seen (a
        # fresh state, load_state_dict) is read once.
        self._step_cache = {}
        # torch.optim.Optimizer wraps step() in a profiler range plus the step-hook loops (~25 us of host time
        # per call).  The class's step (set once per class, after Optimizer.__init__ has wrapped it) skips that
        # wrapper while no hook is registered and no profiler runs, and takes the wrapped method otherwise (hooks
        # and profiler ranges behave as with torch's optimizers).  It lives on the class, not the instance, so
        # an optimizer holds no reference to itself and is freed with its last reference.
        cls = type(self)
        if not getattr(cls.step, "_gs4d_fast", False):
            wrapped = cls.step

            def step(self, closure=None):
                if (_optim_mod._global_optimizer_pre_hooks or _optim_mod._global_optimizer_post_hooks
                        or self._optimizer_step_pre_hooks or self._optimizer_step_post_hooks
                        or torch.autograd.profiler._is_profiler_enabled):
                    return wrapped(self, closure)
                return self._step(closure)

            step.hooked = True  # Optimizer._patch_step_function: already wrapped
            step._gs4d_fast = True
            step.__doc__ = wrapped.__doc__
            cls.step = step

    def step(self, closure=None):
        return self._step(closure)

    def zero_grad(self, set_to_none: bool = True):
        """torch's zero_grad.  set_to_none (the train step's call) while no profiler runs: the same loop without
        torch's profiler range around it (host time every step, with the GPU idle behind it at a step's start)."""
        if not set_to_none or torch.autograd.profiler._is_profiler_enabled:
            return super().zero_grad(set_to_none)
        for group in self.param_groups:
            for p in group["params"]:
                p.grad = None

    @torch.no_grad()
    def _step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        # One pass over the parameters with the per-parameter work kept to a few attribute and dict reads:
        # this loop is host time every train step (~50 parameters), and the GPU waits behind it.  The rare
        # cases (a fresh state, a step tensor the cache has not seen or that was edited, a sparse gradient)
        # take the slow branch.  Non-contiguous gradients are made contiguous by the extension.
        state, cache = self.state, self._step_cache
        by_hyper = {}
        pending = []
        live = 0
        for group in self.param_groups:
            lists = None
            lr = group["lr"]
            beta1, beta2 = group["betas"]
            for p in group["params"]:
                g = p.grad
                if g is None:
                    continue
                st = state[p]
                if not st:
                    st["step"] = torch.tensor(0.0, dtype=torch.float32)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                t = st["step"]
                e = cache.get(id(t))
                # the cached count holds while the tensor is the one cached and was not edited in place since
                # the last step (zero_(), copy_(), a manual reset): a host read through the numpy view, no sync
                if e is None or e[0] is not t or e[1][()] != e[2]:
                    if g.is_sparse:
                        raise RuntimeError("FusedAdam does not support sparse gradients")
                    if t.device.type != "cpu":  # a step tensor moved off the host (not torch's default)
                        step = t.item() + 1.0
                        e = None
                    else:  # CPU float32 0-d tensor, as torch's Adam keeps it
                        e = cache[id(t)] = [t, t.numpy(), t.item()]
                if e is not None:
                    step = e[2] + 1.0
                # the counts advance only once every update below has been accepted (a rejected tensor
                # leaves every step count as it was)
                pending.append((e, t, step))
                if lists is None:
                    key = (beta1, beta2, group["eps"])
                    lists = by_hyper.get(key)
                    if lists is None:
                        lists = by_hyper[key] = ([], [], [], [], [], [])
                    ps, gs, ms, vs, ss, bs = lists
                ps.append(p)
                gs.append(g)
                ms.append(st["exp_avg"])
                vs.append(st["exp_avg_sq"])
                ss.append((lr / (1 - beta1 ** step)) * -1)
                bs.append((1 - beta2 ** step) ** 0.5)
                live += 1
        if not live:
            return loss
        if len(cache) > 4 * live + 64:  # states of parameters no longer optimised
            keep = {id(state[p]["step"]) for ps in (l[0] for l in by_hyper.values()) for p in ps}
            for k in [k for k in cache if k not in keep]:
                del cache[k]
        for (beta1, beta2, eps), (ps, gs, ms, vs, ss, bs) in by_hyper.items():
            _C.adam_step(ps, gs, ms, vs, ss, bs, beta1, beta2, eps)
        for e, t, step in pending:
            if e is None:
                t.fill_(step)
            else:
                e[2] = step
                e[1][()] = step
        return loss


class _DeformTail(torch.autograd.Function):
    """The deformation's residual adds (scene/deformation.py:140-146, on features = cat(f_dc, f_rest),
    scene/gaussian_model.py:116-118) and render()'s activations exp / normalize / sigmoid
    (gaussian_renderer/__init__.py:97-99) in one HIP pass each way (gs4d_deform_tail_*).  A delta that
    is None is a head switched off.  The gradient of each residual input is the gradient of its base.
    Forward values match the torch graph bitwise; the backward follows torch's operation order for exp
    and sigmoid (grad * (1 - y) * y) but restates normalize's backward in closed form, so it agrees
    with autograd to fp32 rounding rather than bitwise (test_deform_tail_matches_torch: 1e-5)."""

    @staticmethod
    def forward(ctx, xyz, s, r, o, f_dc, f_rest, dx, ds, dr, d_o, dshs):
        c = lambda t: None if t is None else t.contiguous()
        dshs_flat = None if dshs is None else dshs.reshape(dshs.shape[0], -1)
        means, scales, rot, opac, shs = _C.deform_tail_forward(xyz.contiguous(), s.contiguous(), r.contiguous(),
                                                               o.contiguous(), f_dc.contiguous(), f_rest.contiguous(),
                                                               c(dx), c(ds), c(dr), c(d_o), c(dshs_flat))
        ctx.save_for_backward(scales, r, dr, opac)
        ctx.K = f_rest.shape[1] + 1
        ctx.has = tuple(t is not None for t in (dx, ds, dr, d_o, dshs))
        ctx.dshs_shape = None if dshs is None else dshs.shape
        ctx.set_materialize_grads(False)
        return means, scales, rot, opac, shs

    @staticmethod
    def backward(ctx, g_means, g_scales, g_rot, g_opac, g_shs):
        scales, r, dr, opac = ctx.saved_tensors
        c = lambda t: None if t is None else t.contiguous()
        g_shs_flat = None if g_shs is None else g_shs.contiguous().reshape(g_shs.shape[0], -1)
        has = ctx.has
        d_xyz, d_s, d_r, d_o, d_fdc, d_frest, g_dx, g_ds, g_dr, g_do = _C.deform_tail_backward(
            scales, r.contiguous(), c(dr), opac, c(g_means), c(g_scales), c(g_rot), c(g_opac), g_shs_flat, ctx.K,
            list(has[:4]))
        d_dshs = None
        if has[4]:
            d_dshs = (g_shs_flat if g_shs_flat is not None else torch.zeros(scales.shape[0], 3 * ctx.K,
                                                                          device=scales.device)).reshape(ctx.dshs_shape)
        return (d_xyz, d_s, d_r, d_o, d_fdc, d_frest, g_dx if has[0] else None, g_ds if has[1] else None,
                g_dr if has[2] else None, g_do if has[3] else None, d_dshs)


def deform_tail(xyz, scales, rotations, opacity, f_dc, f_rest, dx=None, ds=None, dr=None, d_o=None, dshs=None):
    """(means3D, exp(scales + ds), normalize(rotations + dr), sigmoid(opacity + do), cat(f_dc, f_rest) + dshs)."""
    return _DeformTail.apply(xyz, scales, rotations, opacity, f_dc, f_rest, dx, ds, dr, d_o, dshs)


class _HexPlane(torch.autograd.Function):
    """scene/hexplane.py:75-110 interpolate_ms_features over all levels in one launch each way.

    The points are visited in a Morton order of their coordinates; the field is evaluated at the
    Gaussians' canonical means, which the optimizer moves little per step, so the order (any
    permutation gives the same field -- it only buys locality) is kept across calls while the point
    count is unchanged and refreshed every `order_refresh` calls."""

    order_refresh = 100
    _order = None
    _calls = 0

    @staticmethod
    def forward(ctx, pts, *planes):
        cls = _HexPlane
        cached = cls._order
        if (cached is None or cached.numel() != pts.shape[0] or cached.device != pts.device
                or cls._calls % cls.order_refresh == 0):
            cached = None
        cls._calls += 1
        feat, packed, order = _C.hexplane_forward(pts, list(planes), cached)
        cls._order = order
        ctx.save_for_backward(pts, packed, order, *planes)
        return feat

    @staticmethod
    def backward(ctx, dfeat):
        pts, packed, order, *planes = ctx.saved_tensors
        dpts, dplanes = _C.hexplane_backward(pts, planes, packed, dfeat, order)
        return (dpts, *dplanes)


class _HexPoints(torch.autograd.Function):
    """scene/hexplane.py:20-21 normalize_aabb + :166 torch.cat((pts, timestamps), -1) in one HIP pass each
    way (gs4d_hexplane_points): the reference's float operations, so the result is bitwise its graph's.
    The time column takes no gradient (as the reference's timestamps, which never require one here)."""

    @staticmethod
    def forward(ctx, xyz, t, aabb):
        ctx.save_for_backward(aabb)
        return _C.hexplane_points(xyz, t, aabb)

    @staticmethod
    def backward(ctx, dpts):
        (aabb,) = ctx.saved_tensors
        return _C.hexplane_points_backward(dpts, aabb), None, None


class _HexPointsAlias(torch.autograd.Function):
    """_HexPoints that also passes xyz through (a view of it) for xyz's other use, the deformation tail's
    xyz + dx: the backward then forms xyz's whole gradient -- the tail's plus the field's -- in its one pass
    (gs4d_hexplane_points_backward_add), where autograd would sum the two with a separate add launch.  Same
    sum (one fp32 add per element, which is commutative), one launch fewer."""

    @staticmethod
    def forward(ctx, xyz, t, aabb):
        ctx.save_for_backward(aabb)
        ctx.set_materialize_grads(False)  # a use without a gradient arrives as None, not as a zero fill
        return _C.hexplane_points(xyz, t, aabb), xyz.view_as(xyz)

    @staticmethod
    def backward(ctx, dpts, dxyz):
        (aabb,) = ctx.saved_tensors
        if dpts is None:
            return dxyz, None, None
        return _C.hexplane_points_backward(dpts, aabb, add=dxyz), None, None


def set_deterministic(flag=True):
    """The round-4 API for a bitwise-reproducible train step.  Every kernel of the fused step is deterministic by
    default (the HexPlane field's backward sums exact 64-bit fixed-point terms, the rasterizer and the MLP's
    f32-MFMA GEMMs reduce in a fixed order), and the GEMMs rocBLAS serves use its own shape-determined pick, so
    two processes given the same inputs compute the same bits.  flag=True additionally switches off the opt-in
    timing-based GEMM tuner (GS4D_GEMM_TUNE=1), whose choice can differ between processes; flag=False changes
    nothing."""
    if flag:
        from . import deformation
        deformation._TUNE = False


def hexplane_points(xyz, t, aabb, alias=None):
    """(N, 4) = (normalize_aabb(xyz, aabb), t) for the field (gradient to xyz only).  alias (a list): also
    append a pass-through view of xyz for its other differentiable use (_HexPointsAlias)."""
    if alias is not None and torch.is_grad_enabled() and xyz.requires_grad:
        pts, xa = _HexPointsAlias.apply(xyz, t.detach(), aabb.detach())
        alias.append(xa)
        return pts
    return _HexPoints.apply(xyz, t.detach(), aabb.detach())


def hexplane(pts, ms_grids):
    """pts (N, 4) normalised (x, y, z, t); ms_grids: per level the 6 (1, F, H, W) planes."""
    planes = [p for level in ms_grids for p in level]
    return _HexPlane.apply(pts.contiguous(), *planes)


class _HexPlaneReg(torch.autograd.Function):
    """scene/gaussian_model.py:538-577 compute_regulation over the planes in one launch each way."""

    @staticmethod
    def forward(ctx, w_smooth, w_l1, *planes):
        ctx.w = (w_smooth, w_l1)
        ctx.save_for_backward(*planes)
        return _C.hexplane_reg_forward(list(planes), w_smooth, w_l1)

    @staticmethod
    def backward(ctx, dloss):
        planes = ctx.saved_tensors
        grads = _C.hexplane_reg_backward(list(planes), ctx.w[0], ctx.w[1], dloss.reshape(1))
        return (None, None, *grads)


def _reg_batch(ms_grids, time_smoothness_weight, l1_time_planes_weight, plane_tv_weight):
    planes, ws, wl = [], [], []
    for g in ms_grids:
        if len(g) == 3:
            continue
        for i in range(6):
            planes.append(g[i])
            time = i in (2, 4, 5)
            ws.append(float(time_smoothness_weight if time else plane_tv_weight))
            wl.append(float(l1_time_planes_weight if time else 0.0))
    return planes, ws, wl


@torch.no_grad()
def hexplane_regulation_value(ms_grids, time_smoothness_weight, l1_time_planes_weight, plane_tv_weight):
    """hexplane_regulation's value, outside autograd (its gradient comes from
    hexplane_regulation_accumulate_grad after the step's backward)."""
    planes, ws, wl = _reg_batch(ms_grids, time_smoothness_weight, l1_time_planes_weight, plane_tv_weight)
    if not planes:
        return torch.zeros((), device=ms_grids[0][0].device)
    return _C.hexplane_reg_forward([p.detach().contiguous() for p in planes], ws, wl)


@torch.no_grad()
def hexplane_regulation_accumulate_grad(ms_grids, time_smoothness_weight, l1_time_planes_weight, plane_tv_weight,
                                        scale=1.0, with_value=False, base=None):
    """Adds scale * d(regulariser)/d(plane) to every plane's .grad in one launch: the gradient autograd
    would add to the field's plane gradients when the regulariser is part of the loss (train.py:251-254),
    without autograd's separate add per plane.  A plane without a gradient yet gets one.  with_value: also
    returns the regulariser's (unscaled) value from the same pass over the planes, bitwise
    hexplane_regulation_value's.  base (a one-value fp32 device tensor, with_value only): returns base + value
    instead, the add done by the same launch (bitwise torch's fp32 add of the two)."""
    planes, ws, wl = _reg_batch(ms_grids, time_smoothness_weight, l1_time_planes_weight, plane_tv_weight)
    if not planes:
        if not with_value:
            return None
        z = torch.zeros((), device=ms_grids[0][0].device)
        return z if base is None else base.reshape(()) + z
    for p in planes:
        if p.grad is None:
            p.grad = torch.zeros_like(p)
    # the upstream scale as a device scalar, made once per (device, value): no fill launch per step
    key = (planes[0].device, float(scale))
    dloss = _DLOSS.get(key)
    if dloss is None:
        dloss = _DLOSS[key] = torch.full((1,), float(scale), device=planes[0].device)
    if base is not None and not (base.is_cuda and base.dtype == torch.float32 and base.numel() == 1
                                 and base.device == planes[0].device):
        v = hexplane_regulation_accumulate_grad(ms_grids, time_smoothness_weight, l1_time_planes_weight,
                                                plane_tv_weight, scale, with_value)
        return base.detach().reshape(()) + v if with_value else v
    # the planes go to the extension as they are (it only reads their storage: no detach per plane per step)
    v = _C.hexplane_reg_accumulate(planes, [p.grad for p in planes], ws, wl, dloss,
                                   with_value=with_value,
                                   base=base.detach().contiguous() if (with_value and base is not None) else None)
    return v if with_value else None


_DLOSS = {}


def hexplane_regulation(ms_grids, time_smoothness_weight, l1_time_planes_weight, plane_tv_weight):
    """plane_tv_weight * sum smoothness(spatial planes 0, 1, 3) + time_smoothness_weight * sum
    smoothness(time planes 2, 4, 5) + l1_time_planes_weight * sum mean|1 - time plane| over the levels
    (levels with 3 planes contribute nothing, as in the reference)."""
    planes, ws, wl = [], [], []
    for g in ms_grids:
        if len(g) == 3:
            continue
        for i in range(6):
            planes.append(g[i].contiguous())
            time = i in (2, 4, 5)
            ws.append(float(time_smoothness_weight if time else plane_tv_weight))
            wl.append(float(l1_time_planes_weight if time else 0.0))
    if not planes:
        return torch.zeros((), device=ms_grids[0][0].device)
    return _HexPlaneReg.apply(ws, wl, *planes)
