"""render() of gaussian_renderer/__init__.py:17-140, the rasterizer's caller, restated.

Same argument mapping and return dict as the reference: screen-space points are a zero tensor with
retain_grad (:24-29); the fine stage deforms (xyz, scales, rotations, opacity, SHs) at the camera's
time (:79-89); activations exp / normalize / sigmoid (:94-96); SH -> RGB happens in the rasterizer;
returns {render, viewspace_points, visibility_filter = radii > 0, radii, depth} (:134-139).
"""
import math

import torch

import diff_gaussian_rasterization as dgr


def render(viewpoint_camera, pc, pipe_debug, bg_color, scaling_modifier=1.0, stage="fine"):
    xyz = pc.get_xyz
    screenspace_points = torch.zeros_like(xyz, dtype=xyz.dtype, requires_grad=True, device=xyz.device) + 0
    try:
        screenspace_points.retain_grad()
    except Exception:
        pass
    dev = xyz.device
    settings = dgr.GaussianRasterizationSettings(
        image_height=int(viewpoint_camera.image_height), image_width=int(viewpoint_camera.image_width),
        tanfovx=math.tan(viewpoint_camera.FoVx * 0.5), tanfovy=math.tan(viewpoint_camera.FoVy * 0.5),
        bg=bg_color, scale_modifier=scaling_modifier,
        viewmatrix=viewpoint_camera.world_view_transform.to(dev),
        projmatrix=viewpoint_camera.full_proj_transform.to(dev), sh_degree=pc.active_sh_degree,
        campos=viewpoint_camera.camera_center.to(dev), prefiltered=False, debug=pipe_debug)
    time = torch.tensor(viewpoint_camera.time).to(dev).repeat(xyz.shape[0], 1)
    rasterizer = dgr.GaussianRasterizer(raster_settings=settings)
    opacity, shs, scales, rotations = pc._opacity, pc.get_features, pc._scaling, pc._rotation
    if "coarse" in stage:
        m3, sc, rot, op, sh = xyz, scales, rotations, opacity, shs
    elif "fine" in stage:
        m3, sc, rot, op, sh = pc._deformation(xyz, scales, rotations, opacity, shs, time)
    else:
        raise NotImplementedError(stage)
    sc = pc.scaling_activation(sc)
    rot = pc.rotation_activation(rot)
    op = pc.opacity_activation(op)
    image, radii, depth = rasterizer(means3D=m3, means2D=screenspace_points, shs=sh, colors_precomp=None,
                                     opacities=op, scales=sc, rotations=rot, cov3D_precomp=None)
    return {"render": image, "viewspace_points": screenspace_points, "visibility_filter": radii > 0,
            "radii": radii, "depth": depth}
