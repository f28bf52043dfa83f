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
    # the rasterizer's means2D gradient sink (:24-29 builds zeros + 0 and retains its grad; a zero leaf
    # holds the same values and receives the same .grad)
    screenspace_points = torch.zeros_like(xyz, dtype=xyz.dtype, requires_grad=True, device=xyz.device)
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
    # torch.tensor(time).to(dev).repeat(P, 1) (:52): the same float32 column, filled on the device
    time = torch.full((xyz.shape[0], 1), float(torch.tensor(viewpoint_camera.time)), device=dev)
    rasterizer = dgr.GaussianRasterizer(raster_settings=settings)
    if "coarse" not in stage and "fine" not in stage:
        raise NotImplementedError(stage)
    if getattr(pc, "fused", False) and getattr(pc, "fused_tail", True) and xyz.is_cuda:
        # the heads' residual adds, cat(f_dc, f_rest) and the activations as one HIP pass each way
        from .kernels import deform_tail
        d = pc._deformation.deltas(xyz, time) if "fine" in stage else {}
        m3, sc, rot, op, sh = deform_tail(xyz, pc._scaling, pc._rotation, pc._opacity, pc._features_dc,
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
    return {"render": image, "viewspace_points": screenspace_points, "visibility_filter": radii > 0,
            "radii": radii, "depth": depth}
