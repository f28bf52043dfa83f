"""MI355X drop-in for the `diff_gaussian_rasterization` extension API.

Public surface identical to the reference package
(submodules/depth-diff-gaussian-rasterization/diff_gaussian_rasterization/__init__.py:12-220):

  GaussianRasterizationSettings  NamedTuple, same field order (:157-169)
  GaussianRasterizer             nn.Module with forward(...) and markVisible(...) (:171-220)
  rasterize_gaussians            functional entry (:21-42)
  _RasterizeGaussians            torch.autograd.Function (:44-155)

so gaussian_renderer/__init__.py and train.py run unchanged.  The compute runs in libgs4d (HIP
kernels for gfx950) through the `_C` binding built in-tree by build_ext.py; importing this package
without the built extension raises ImportError -- there is no CPU fallback.
"""
from typing import NamedTuple

import torch
import torch.nn as nn

from . import _C  # noqa: F401  (fails loudly when the HIP extension is missing)

__all__ = ["GaussianRasterizationSettings", "GaussianRasterizer", "rasterize_gaussians", "_RasterizeGaussians"]


class GaussianRasterizationSettings(NamedTuple):
    image_height: int
    image_width: int
    tanfovx: float
    tanfovy: float
    bg: torch.Tensor
    scale_modifier: float
    viewmatrix: torch.Tensor
    projmatrix: torch.Tensor
    sh_degree: int
    campos: torch.Tensor
    prefiltered: bool
    debug: bool


def _snapshot(args):
    """Host copies of the call arguments, taken before the call in debug mode (reference :17-19)."""
    return tuple(a.detach().cpu().clone() if isinstance(a, torch.Tensor) else a for a in args)


def _invoke(fn, args, debug, dump_name, stage):
    """Run a `_C` entry point; in debug mode dump the arguments if it raises (reference :83-90,132-139)."""
    if not debug:
        return fn(*args)
    saved = _snapshot(args)
    try:
        return fn(*args)
    except Exception:
        torch.save(saved, dump_name)
        print(f"\nAn error occured in {stage}. Please forward {dump_name} for debugging.")
        raise


def rasterize_gaussians(means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                        raster_settings):
    return _RasterizeGaussians.apply(means3D, means2D, sh, colors_precomp, opacities, scales, rotations,
                                     cov3Ds_precomp, raster_settings)


class _RasterizeGaussians(torch.autograd.Function):
    @staticmethod
    def forward(ctx, means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                raster_settings):
        s = raster_settings
        # positional order of _C.rasterize_gaussians (rasterize_points.h:18-38)
        args = (s.bg, means3D, colors_precomp, opacities, scales, rotations, s.scale_modifier, cov3Ds_precomp,
                s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, s.image_height, s.image_width, sh, s.sh_degree,
                s.campos, s.prefiltered, s.debug)
        num_rendered, color, depth, radii, geom_buf, binning_buf, img_buf = _invoke(
            _C.rasterize_gaussians, args, s.debug, "snapshot_fw.dump", "forward")
        ctx.raster_settings = s
        ctx.num_rendered = num_rendered
        # radii are integers and the depth image gets no gradient (below): autograd need not build
        # zero gradients for them before calling backward
        ctx.mark_non_differentiable(radii)
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(colors_precomp, means3D, scales, rotations, cov3Ds_precomp, radii, sh, geom_buf,
                              binning_buf, img_buf)
        return color, radii, depth

    @staticmethod
    def backward(ctx, grad_out_color, grad_radii, grad_depth):
        # grad_radii and grad_depth are ignored, exactly like the reference (:100-101): no gradient
        # flows from the depth image.
        s = ctx.raster_settings
        if grad_out_color is None:  # only the depth image was used: nothing flows back (as the reference)
            return (None,) * 9
        (colors_precomp, means3D, scales, rotations, cov3Ds_precomp, radii, sh, geom_buf, binning_buf,
         img_buf) = ctx.saved_tensors
        # positional order of _C.rasterize_gaussians_backward (rasterize_points.h:40-62)
        args = (s.bg, means3D, radii, colors_precomp, scales, rotations, s.scale_modifier, cov3Ds_precomp,
                s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, grad_out_color, sh, s.sh_degree, s.campos,
                geom_buf, ctx.num_rendered, binning_buf, img_buf, s.debug)
        (g_means2D, g_colors, g_opacities, g_means3D, g_cov3D, g_sh, g_scales, g_rotations) = _invoke(
            _C.rasterize_gaussians_backward, args, s.debug, "snapshot_bw.dump", "backward")
        return g_means3D, g_means2D, g_sh, g_colors, g_opacities, g_scales, g_rotations, g_cov3D, None


def _empty_if_none(t):
    # "not provided" travels as an empty tensor (reference :197-207)
    return torch.Tensor([]) if t is None else t


class GaussianRasterizer(nn.Module):
    def __init__(self, raster_settings):
        super().__init__()
        self.raster_settings = raster_settings

    def markVisible(self, positions):
        """Near-plane visibility mask of `positions` for this camera (reference :176-185)."""
        with torch.no_grad():
            s = self.raster_settings
            return _C.mark_visible(positions, s.viewmatrix, s.projmatrix)

    def forward(self, means3D, means2D, opacities, shs=None, colors_precomp=None, scales=None, rotations=None,
                cov3D_precomp=None):
        # argument exclusivity rules and messages of the reference (:191-195)
        if (shs is None) == (colors_precomp is None):
            raise Exception('Please provide excatly one of either SHs or precomputed colors!')
        have_sr = scales is not None or rotations is not None
        if (cov3D_precomp is None and (scales is None or rotations is None)) or (have_sr and cov3D_precomp is not None):
            raise Exception('Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!')
        return rasterize_gaussians(means3D, means2D, _empty_if_none(shs), _empty_if_none(colors_precomp), opacities,
                                   _empty_if_none(scales), _empty_if_none(rotations), _empty_if_none(cov3D_precomp),
                                   self.raster_settings)
