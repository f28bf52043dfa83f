"""One training iteration of the reference's train.py (scene_reconstruction, :144-387), restated.

train_step() renders a batch of views through the deformation field and the rasterizer, takes the
L1 loss (+ HexPlane regularisers in the fine stage, + D-SSIM when lambda_dssim != 0), back-propagates,
sums the viewspace gradients over the views, updates the densification statistics, densifies /
prunes / resets opacity on the reference's schedule, and steps the optimizer.  What it leaves out
is logging and I/O: the reference's per-step host syncs for the progress bar (loss.item(), psnr)
and the NaN check that re-execs the program (:255-257) are not part of a training step's work.

With `data_parallel=True` the views of the batch are sharded over the torch.distributed ranks
(gs4d_train.dp): each rank renders its share, and the parameter gradients, viewspace gradients,
radii and visibility are reduced so every replica takes the single-process step.
"""
import torch

from . import dp
from .losses import l1_loss_torch


def train_step(gaussians, views, opt, hyper, iteration, background, stage="fine", fused_loss=None,
               data_parallel=False, render_fn=None):
    """views: list of (camera, gt_image (3, H, W)).  Returns the (detached) batch loss tensor.

    render_fn(camera, gaussians, debug, bg, stage=...) -> render()'s dict; defaults to
    gs4d_train.render.render (the HIP rasterizer).  The multi-process CPU tests pass a torch stand-in."""
    if render_fn is None:
        from .render import render as render_fn
    fused = gaussians.fused if fused_loss is None else fused_loss
    gaussians.update_learning_rate(iteration)
    if iteration % 1000 == 0:
        gaussians.oneupSHdegree()
    mine = dp.shard_views(len(views)) if data_parallel else list(range(len(views)))
    images, gts, radii_list, vis_list, vs_list = [], [], [], [], []
    for v in mine:
        cam, gt = views[v]
        pkg = render_fn(cam, gaussians, False, background, stage=stage)
        images.append(pkg["render"].unsqueeze(0))
        gts.append(gt.unsqueeze(0))
        radii_list.append(pkg["radii"].unsqueeze(0))
        vis_list.append(pkg)  # its visibility_filter (radii > 0) is read only where needed below
        vs_list.append(pkg["viewspace_points"])
    P = gaussians.get_xyz.shape[0]
    dev = gaussians.get_xyz.device
    # train.py:221-228 batches the views with torch.cat and reduces radii / visibility over them; with one view
    # per rank those are the view's own tensors (no copies, no reductions)
    one = len(mine) == 1
    if one:
        # the fused statistics filter by radii > 0 inside their kernel (visibility_filter's definition)
        radii = radii_list[0][0]
        visibility_filter = None if (gaussians.fused and not data_parallel) else vis_list[0]["visibility_filter"]
    else:
        vis_list = [pk["visibility_filter"].unsqueeze(0) for pk in vis_list]
        radii = torch.cat(radii_list, 0).max(dim=0).values if radii_list else torch.zeros(P, dtype=torch.int32,
                                                                                       device=dev)
        visibility_filter = torch.cat(vis_list).any(dim=0) if vis_list else torch.zeros(P, dtype=torch.bool,
                                                                                      device=dev)
    image_grad = None  # fused path, no D-SSIM: the L1's image gradient, formed with its value in one pass
    if images:
        image_tensor = images[0] if one else torch.cat(images, 0)
        gt_image_tensor = gts[0] if one else torch.cat(gts, 0)
        # the batch mean over all views: each rank holds len(mine) of len(views)
        share = len(mine) / len(views) if data_parallel else 1.0
        if fused and opt.lambda_dssim == 0:
            # loss = L1 * share (+ the regulariser, deferred below) is linear in the L1, so
            # loss.backward() deposits exactly image.backward(sign / N * share): value and gradient in one
            # pass (gs4d_l1_loss_grad), no L1 autograd node
            from .kernels import l1_loss_and_grad
            Ll1, image_grad = l1_loss_and_grad(image_tensor, gt_image_tensor[:, :3, :, :], share)
            loss = Ll1 * share if data_parallel else Ll1
        elif fused:
            from .kernels import l1_loss
            Ll1 = l1_loss(image_tensor, gt_image_tensor[:, :3, :, :])
            loss = Ll1 * share if data_parallel else Ll1
        else:
            Ll1 = l1_loss_torch(image_tensor, gt_image_tensor[:, :3, :, :])
            loss = Ll1 * share if data_parallel else Ll1
    else:
        loss = torch.zeros((), device=dev)
    reg_w = (hyper.time_smoothness_weight, hyper.l1_time_planes, hyper.plane_tv_weight)
    reg_scale = 1.0 / dp.world() if data_parallel else 1.0
    reg_deferred = False
    if stage == "fine" and hyper.time_smoothness_weight != 0:
        if fused:
            # the regulariser depends only on the planes: after the backward one pass over them adds its
            # gradient to the planes' gradients and gives its value, which joins the reported loss
            reg_deferred = True
        else:
            reg = gaussians.compute_regulation(*reg_w)
            loss = loss + reg * reg_scale
    if opt.lambda_dssim != 0 and images:
        from .losses import ssim
        loss = loss + opt.lambda_dssim * (1.0 - ssim(image_tensor, gt_image_tensor)) * (
            len(mine) / len(views) if data_parallel else 1.0)
    # a data-parallel rank with no view of the batch (len(views) < world) and no regulariser has a
    # constant loss: nothing to back-propagate, its gradients are the zeros filled in below
    if image_grad is not None:
        if image_tensor.requires_grad:
            image_tensor.backward(image_grad)
    elif loss.requires_grad:
        loss.backward()
    if reg_deferred:
        if reg_scale == 1.0:
            # loss.detach() + value, the add inside the regulariser's own launch
            loss = gaussians.add_regulation_grad(*reg_w, scale=reg_scale, with_value=True, base=loss.detach())
        else:
            loss = loss.detach() + gaussians.add_regulation_grad(*reg_w, scale=reg_scale, with_value=True) * reg_scale
    if len(vs_list) == 1 and vs_list[0].grad is not None:
        viewspace_grad = vs_list[0].grad
    else:
        viewspace_grad = torch.zeros_like(gaussians.get_xyz)
        for t in vs_list:
            if t.grad is not None:
                viewspace_grad = viewspace_grad + t.grad
    # the returned loss: a view when nothing writes it later (the data-parallel all-reduce sums in place)
    loss_out = loss.detach().reshape(1)
    if data_parallel:
        loss_out = loss_out.clone()
    if data_parallel and dp.world() > 1:
        # a parameter gets a gradient on every replica iff some rank produced one (a rank without views
        # produces none); parameters no rank touched keep grad None, so the optimizer skips them as the
        # single-process step does (their Adam step counts stay in step)
        params = [p for g in gaussians.optimizer.param_groups for p in g["params"]]
        has = torch.tensor([p.grad is not None for p in params], dtype=torch.int32, device=dev)
        torch.distributed.all_reduce(has, op=torch.distributed.ReduceOp.MAX)
        params = [p for p, h in zip(params, has.tolist()) if h]
        for p in params:
            if p.grad is None:
                p.grad = torch.zeros_like(p)
        vis_i = visibility_filter.to(torch.int32)
        dp.allreduce_sum_([p.grad for p in params] + [viewspace_grad, loss_out])
        torch.distributed.all_reduce(radii, op=torch.distributed.ReduceOp.MAX)
        torch.distributed.all_reduce(vis_i, op=torch.distributed.ReduceOp.MAX)
        visibility_filter = vis_i.bool()
    with torch.no_grad():
        if iteration < opt.densify_until_iter:
            gaussians.add_densification_stats(viewspace_grad, visibility_filter, radii)
            if stage == "coarse":
                opacity_threshold = opt.opacity_threshold_coarse
                densify_threshold = opt.densify_grad_threshold_coarse
            else:
                opacity_threshold = opt.opacity_threshold_fine_init - iteration * (
                    opt.opacity_threshold_fine_init - opt.opacity_threshold_fine_after) / opt.densify_until_iter
                densify_threshold = opt.densify_grad_threshold_fine_init - iteration * (
                    opt.densify_grad_threshold_fine_init - opt.densify_grad_threshold_after) / opt.densify_until_iter
            extent = getattr(gaussians, "cameras_extent", 1.0)
            if iteration > opt.densify_from_iter and iteration % opt.densification_interval == 0 and P < 360000:
                size_threshold = 20 if iteration > opt.opacity_reset_interval else None
                # the split's random offsets are rank 0's on every replica only in a data-parallel step
                gaussians.data_parallel_step = bool(data_parallel)
                try:
                    gaussians.densify(densify_threshold, opacity_threshold, extent, size_threshold)
                finally:
                    gaussians.data_parallel_step = False
            if iteration > opt.pruning_from_iter and iteration % opt.pruning_interval == 0 and \
                    gaussians.get_xyz.shape[0] > 200000:
                size_threshold = 20 if iteration > opt.opacity_reset_interval else None
                gaussians.prune(densify_threshold, opacity_threshold, extent, size_threshold)
            if iteration % opt.opacity_reset_interval == 0:
                gaussians.reset_opacity()
        if iteration < opt.iterations:
            gaussians.optimizer.step()
            gaussians.optimizer.zero_grad(set_to_none=True)
    return loss_out[0]
