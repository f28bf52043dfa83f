"""render() of gaussian_renderer/__init__.py:17-140, the rasterizer's caller, restated.

Same argument mapping and return dict as the reference: screen-space points are a zero tensor with
retain_grad (:24-29); the fine stage deforms (xyz, scales, rotations, opacity, SHs) at the camera's
time (:79-89); activations exp / normalize / sigmoid (:94-96); SH -> RGB happens in the rasterizer;
returns {render, viewspace_points, visibility_filter = radii > 0, radii, depth} (:134-139).
"""
import math

import numpy as np

import torch

import diff_gaussian_rasterization as dgr


_TIMES = {}


def _time_value(t, dev):
    """a (1, 1) float32 device tensor holding t, cached per (device, t)"""
    key = (str(dev), t)
    v = _TIMES.get(key)
    if v is None:
        if len(_TIMES) > 4096:
            _TIMES.clear()
        v = _TIMES[key] = torch.full((1, 1), t, dtype=torch.float32, device=dev)
    return v


def _time_float(t):
    """float(torch.tensor(t)): a Python float becomes float32 on the way (torch's default dtype), without building a
    CPU tensor per call; anything else takes torch.tensor as the reference does"""
    if type(t) is float:
        return float(np.float32(t))
    return float(torch.tensor(t))


_ZERO_POINTS = {}


def _zero_points(xyz):
    """the means2D gradient sink: a fresh leaf (requires_grad, its own .grad) over a zero (P, 3) buffer kept per
    (device, shape, dtype) -- its values are never written, so one fill serves every call (no fill per step)"""
    key = (xyz.device, tuple(xyz.shape), xyz.dtype)
    z = _ZERO_POINTS.get(key)
    if z is None:
        if len(_ZERO_POINTS) >= 4:
            _ZERO_POINTS.clear()
        z = _ZERO_POINTS[key] = torch.zeros_like(xyz, dtype=xyz.dtype, device=xyz.device)
    return z.detach().requires_grad_(True)


class RenderPackage(dict):
    """render()'s dict (gaussian_renderer/__init__.py:130-138) with "visibility_filter" = radii > 0 formed on
    first use: the fused train step filters the densification statistics by radii > 0 inside their kernel,
    so a step that never reads the mask launches no compare for it.  Every key the reference returns is
    there for any reader (in, keys(), items() and indexing all see it)."""

    def __init__(self, **kw):
        super().__init__(**kw)
        self._lazy_vis = True

    def _vis(self):
        if self._lazy_vis:
            self._lazy_vis = False
            dict.__setitem__(self, "visibility_filter", dict.__getitem__(self, "radii") > 0)

    def __getitem__(self, k):
        if k == "visibility_filter":
            self._vis()
        return dict.__getitem__(self, k)

    def get(self, k, default=None):
        if k == "visibility_filter":
            self._vis()
        return dict.get(self, k, default)

    def __contains__(self, k):
        return k == "visibility_filter" or dict.__contains__(self, k)

    def keys(self):
        self._vis()
        return dict.keys(self)

    def items(self):
        self._vis()
        return dict.items(self)

    def values(self):
        self._vis()
        return dict.values(self)

    def __iter__(self):
        self._vis()
        return dict.__iter__(self)

    def __len__(self):
        self._vis()
        return dict.__len__(self)


def render(viewpoint_camera, pc, pipe_debug, bg_color, scaling_modifier=1.0, stage="fine"):
    xyz = pc.get_xyz
    # the rasterizer's means2D gradient sink (:24-29 builds zeros + 0 and retains its grad; a zero leaf
    # holds the same values and receives the same .grad)
    screenspace_points = _zero_points(xyz)
    dev = xyz.device
    if hasattr(viewpoint_camera, "on_device"):
        view_m, proj_m, cam_c = viewpoint_camera.on_device(dev)
    else:
        view_m, proj_m, cam_c = (viewpoint_camera.world_view_transform.to(dev),
                                 viewpoint_camera.full_proj_transform.to(dev), viewpoint_camera.camera_center.to(dev))
    settings = dgr.GaussianRasterizationSettings(
        image_height=int(viewpoint_camera.image_height), image_width=int(viewpoint_camera.image_width),
        tanfovx=math.tan(viewpoint_camera.FoVx * 0.5), tanfovy=math.tan(viewpoint_camera.FoVy * 0.5),
        bg=bg_color, scale_modifier=scaling_modifier, viewmatrix=view_m, projmatrix=proj_m,
        sh_degree=pc.active_sh_degree, campos=cam_c, prefiltered=False, debug=pipe_debug)
    # torch.tensor(time).to(dev).repeat(P, 1) (:52): the same float32 column, as one device value broadcast
    # over the P rows (made once per (device, time); no fill per call)
    time = _time_value(_time_float(viewpoint_camera.time), dev).expand(xyz.shape[0], 1)
    rasterizer = dgr.GaussianRasterizer(raster_settings=settings)
    if "coarse" not in stage and "fine" not in stage:
        raise NotImplementedError(stage)
    if getattr(pc, "fused", False) and getattr(pc, "fused_tail", True) and xyz.is_cuda:
        # the heads' residual adds, cat(f_dc, f_rest) and the activations as one HIP pass each way
        from .kernels import deform_tail
        alias = []  # xyz passed through the field's points op, which then sums in the tail's xyz gradient
        d = pc._deformation.deltas(xyz, time, alias) if "fine" in stage else {}
        m3, sc, rot, op, sh = deform_tail(alias[0] if alias else xyz, pc._scaling, pc._rotation, pc._opacity, pc._features_dc,
                                          pc._features_rest, d.get("pos_deform"), d.get("scales_deform"),
                                          d.get("rotations_deform"), d.get("opacity_deform"), d.get("shs_deform"))
    else:
        opacity, shs, scales, rotations = pc._opacity, pc.get_features, pc._scaling, pc._rotation
        if "coarse" in stage:
            m3, sc, rot, op, sh = xyz, scales, rotations, opacity, shs
        else:
            m3, sc, rot, op, sh = pc._deformation(xyz, scales, rotations, opacity, shs, time)
        sc = pc.scaling_activation(sc)
        rot = pc.rotation_activation(rot)
        op = pc.opacity_activation(op)
    image, radii, depth = rasterizer(means3D=m3, means2D=screenspace_points, shs=sh, colors_precomp=None,
                                     opacities=op, scales=sc, rotations=rot, cov3D_precomp=None)
    return RenderPackage(render=image, viewspace_points=screenspace_points, radii=radii, depth=depth)
