"""The Gaussian model around the rasterizer: parameters, activations, optimizer, densification.

Restates scene/gaussian_model.py of the reference (the train-step tail) for the
fine-stage training path: the same parameter tensors and activations (:29-45), the Adam parameter
groups and learning-rate schedules (:165-212), the densification statistics (:521-523), the
clone / split / prune events (:316-506, as row plans: gs4d_train/surgery.py), opacity reset (:269-272),
the HexPlane regularisers (:538-566) and the PLY layout (:214-226, 250-314; see gs4d_train/ply.py).

Four places run libgs4d HIP kernels when `fused=True` (the default on a GPU): the optimizer step
(one multi-tensor Adam launch, kernels.FusedAdam), the densification statistics
(kernels.densify_stats), the HexPlane regularisers (kernels.hexplane_regulation) and the densify / prune
row surgery (one gs4d_rows_assemble launch per event).  `fused=False` runs the torch formulations, which the
parity tests compare against.
"""
import math

import numpy as np
import torch
import torch.nn as nn

from . import surgery
from .deformation import DeformNetwork


def inverse_sigmoid(x):
    """utils/general_utils.py:18-19"""
    return torch.log(x / (1 - x))


def get_expon_lr_func(lr_init, lr_final, lr_delay_steps=0, lr_delay_mult=1.0, max_steps=1000000):
    """utils/general_utils.py:35-68 (log-linear decay with an optional cosine warm-up)."""
    def helper(step):
        if step < 0 or (lr_init == 0.0 and lr_final == 0.0):
            return 0.0
        if lr_delay_steps > 0:
            delay_rate = lr_delay_mult + (1 - lr_delay_mult) * np.sin(0.5 * np.pi * np.clip(step / lr_delay_steps, 0, 1))
        else:
            delay_rate = 1.0
        t = np.clip(step / max_steps, 0, 1)
        log_lerp = np.exp(np.log(lr_init) * (1 - t) + np.log(lr_final) * t)
        return delay_rate * log_lerp
    return helper


def build_rotation(r):
    """utils/general_utils.py:78-99: rotation matrices of the normalised quaternions (r, x, y, z)."""
    norm = torch.sqrt(r[:, 0] * r[:, 0] + r[:, 1] * r[:, 1] + r[:, 2] * r[:, 2] + r[:, 3] * r[:, 3])
    q = r / norm[:, None]
    R = torch.zeros((q.size(0), 3, 3), device=r.device)
    w, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    R[:, 0, 0] = 1 - 2 * (y * y + z * z)
    R[:, 0, 1] = 2 * (x * y - w * z)
    R[:, 0, 2] = 2 * (x * z + w * y)
    R[:, 1, 0] = 2 * (x * y + w * z)
    R[:, 1, 1] = 1 - 2 * (x * x + z * z)
    R[:, 1, 2] = 2 * (y * z - w * x)
    R[:, 2, 0] = 2 * (x * z - w * y)
    R[:, 2, 1] = 2 * (y * z + w * x)
    R[:, 2, 2] = 1 - 2 * (x * x + y * y)
    return R


SH_C0 = 0.28209479177387814


def rgb2sh(rgb):
    """utils/sh_utils.py:114-115"""
    return (rgb - 0.5) / SH_C0


def compute_plane_smoothness(t):
    """scene/regulation.py:22-28: mean squared second difference along dim 2 (time for time planes)."""
    h = t.shape[2]
    first = t[..., 1:, :] - t[..., :h - 1, :]
    second = first[..., 1:, :] - first[..., :h - 2, :]
    return torch.square(second).mean()


class GaussianModel:
    def __init__(self, sh_degree, args, fused=None):
        self.active_sh_degree = 0
        self.max_sh_degree = sh_degree
        self._deformation = DeformNetwork(args)
        self._xyz = torch.empty(0)
        self._features_dc = torch.empty(0)
        self._features_rest = torch.empty(0)
        self._scaling = torch.empty(0)
        self._rotation = torch.empty(0)
        self._opacity = torch.empty(0)
        self.max_radii2D = torch.empty(0)
        self.xyz_gradient_accum = torch.empty(0)
        self.denom = torch.empty(0)
        self.optimizer = None
        self.percent_dense = 0
        self.spatial_lr_scale = 0
        self._deformation_table = torch.empty(0)
        self.fused = torch.cuda.is_available() if fused is None else fused
        # gaussian_model.py:29-45
        self.scaling_activation = torch.exp
        self.scaling_inverse_activation = torch.log
        self.opacity_activation = torch.sigmoid
        self.inverse_opacity_activation = inverse_sigmoid
        self.rotation_activation = torch.nn.functional.normalize

    # ---- accessors (gaussian_model.py:108-131)
    @property
    def get_scaling(self):
        return self.scaling_activation(self._scaling)

    @property
    def get_rotation(self):
        return self.rotation_activation(self._rotation)

    @property
    def get_xyz(self):
        return self._xyz

    @property
    def get_features(self):
        return torch.cat((self._features_dc, self._features_rest), dim=1)

    @property
    def get_opacity(self):
        return self.opacity_activation(self._opacity)

    def oneupSHdegree(self):
        if self.active_sh_degree < self.max_sh_degree:
            self.active_sh_degree += 1

    # ---- checkpoints (gaussian_model.py:66-106; train.py:49-57 restores, :393-395 saves)
    def capture(self):
        """The reference's checkpoint tuple, in its order; saved as torch.save((capture(), iteration))."""
        return (self.active_sh_degree, self._xyz, self._deformation.state_dict(), self._deformation_table,
                self._features_dc, self._features_rest, self._scaling, self._rotation, self._opacity,
                self.max_radii2D, self.xyz_gradient_accum, self.denom, self.optimizer.state_dict(),
                self.spatial_lr_scale)

    def restore(self, model_args, training_args):
        """Inverse of capture(): parameters, deformation network, statistics, then a fresh optimizer
        (training_setup) loaded with the saved state -- torch.optim.Adam and FusedAdam state dicts are
        interchangeable."""
        (self.active_sh_degree, self._xyz, deform_state, self._deformation_table, self._features_dc,
         self._features_rest, self._scaling, self._rotation, self._opacity, self.max_radii2D, xyz_gradient_accum,
         denom, opt_dict, self.spatial_lr_scale) = model_args
        self._deformation.load_state_dict(deform_state)
        self.training_setup(training_args)
        self.xyz_gradient_accum = xyz_gradient_accum
        self.denom = denom
        self.optimizer.load_state_dict(opt_dict)

    # ---- initialisation (gaussian_model.py:137-163)
    def create_from_pcd(self, points, colors, spatial_lr_scale, device="cuda"):
        from simple_knn._C import distCUDA2
        self.spatial_lr_scale = spatial_lr_scale
        fused_point_cloud = torch.tensor(np.asarray(points)).float().to(device)
        fused_color = rgb2sh(torch.tensor(np.asarray(colors)).float().to(device))
        features = torch.zeros((fused_color.shape[0], 3, (self.max_sh_degree + 1) ** 2)).float().to(device)
        features[:, :3, 0] = fused_color
        features[:, 3:, 1:] = 0.0
        dist2 = torch.clamp_min(distCUDA2(torch.from_numpy(np.asarray(points)).float().to(device)), 0.0000001)
        scales = torch.log(torch.sqrt(dist2))[..., None].repeat(1, 3)
        rots = torch.zeros((fused_point_cloud.shape[0], 4), device=device)
        rots[:, 0] = 1
        opacities = inverse_sigmoid(0.1 * torch.ones((fused_point_cloud.shape[0], 1), dtype=torch.float, device=device))
        self._xyz = nn.Parameter(fused_point_cloud.requires_grad_(True))
        self._deformation = self._deformation.to(device)
        self._features_dc = nn.Parameter(features[:, :, 0:1].transpose(1, 2).contiguous().requires_grad_(True))
        self._features_rest = nn.Parameter(features[:, :, 1:].transpose(1, 2).contiguous().requires_grad_(True))
        self._scaling = nn.Parameter(scales.requires_grad_(True))
        self._rotation = nn.Parameter(rots.requires_grad_(True))
        self._opacity = nn.Parameter(opacities.requires_grad_(True))
        self.max_radii2D = torch.zeros((self.get_xyz.shape[0]), device=device)
        self._deformation_table = torch.gt(torch.ones((self.get_xyz.shape[0]), device=device), 0)

    # ---- optimizer (gaussian_model.py:165-212)
    def training_setup(self, training_args):
        dev = self._xyz.device
        self.percent_dense = training_args.percent_dense
        self.xyz_gradient_accum = torch.zeros((self.get_xyz.shape[0], 1), device=dev)
        self.denom = torch.zeros((self.get_xyz.shape[0], 1), device=dev)
        self._deformation_accum = torch.zeros((self.get_xyz.shape[0], 3), device=dev)
        s = self.spatial_lr_scale
        groups = [
            {"params": [self._xyz], "lr": training_args.position_lr_init * s, "name": "xyz"},
            {"params": list(self._deformation.get_mlp_parameters()), "lr": training_args.deformation_lr_init * s,
             "name": "deformation"},
            {"params": list(self._deformation.get_grid_parameters()), "lr": training_args.grid_lr_init * s,
             "name": "grid"},
            {"params": [self._features_dc], "lr": training_args.feature_lr, "name": "f_dc"},
            {"params": [self._features_rest], "lr": training_args.feature_lr / 20.0, "name": "f_rest"},
            {"params": [self._opacity], "lr": training_args.opacity_lr, "name": "opacity"},
            {"params": [self._scaling], "lr": training_args.scaling_lr, "name": "scaling"},
            {"params": [self._rotation], "lr": training_args.rotation_lr, "name": "rotation"},
        ]
        if self.fused:
            from .kernels import FusedAdam
            self.optimizer = FusedAdam(groups, lr=0.0, eps=1e-15)
        else:
            self.optimizer = torch.optim.Adam(groups, lr=0.0, eps=1e-15)
        self.xyz_scheduler_args = get_expon_lr_func(training_args.position_lr_init * s, training_args.position_lr_final * s,
                                                    lr_delay_mult=training_args.position_lr_delay_mult,
                                                    max_steps=training_args.position_lr_max_steps)
        self.deformation_scheduler_args = get_expon_lr_func(training_args.deformation_lr_init * s,
                                                            training_args.deformation_lr_final * s,
                                                            lr_delay_mult=training_args.deformation_lr_delay_mult,
                                                            max_steps=training_args.position_lr_max_steps)
        self.grid_scheduler_args = get_expon_lr_func(training_args.grid_lr_init * s, training_args.grid_lr_final * s,
                                                     lr_delay_mult=training_args.deformation_lr_delay_mult,
                                                     max_steps=training_args.position_lr_max_steps)

    def update_learning_rate(self, iteration):
        for g in self.optimizer.param_groups:
            if g["name"] == "xyz":
                g["lr"] = self.xyz_scheduler_args(iteration)
            if "grid" in g["name"]:
                g["lr"] = self.grid_scheduler_args(iteration)
            elif g["name"] == "deformation":
                g["lr"] = self.deformation_scheduler_args(iteration)

    # ---- densification statistics (gaussian_model.py:521-523, train.py:346-349)
    def add_densification_stats(self, viewspace_grad, update_filter, radii=None):
        """xyz_gradient_accum[f] += |grad[f, :2]|, denom[f] += 1 and (when radii is given, train.py:348)
        max_radii2D[f] = max(max_radii2D[f], radii[f]).  update_filter None: f = radii > 0 (train.py:229-232)."""
        if self.fused:
            from .kernels import densify_stats
            densify_stats(viewspace_grad, update_filter, radii, self.xyz_gradient_accum, self.denom, self.max_radii2D)
            return
        if update_filter is None:
            update_filter = radii > 0
        if radii is not None:
            self.max_radii2D[update_filter] = torch.max(self.max_radii2D[update_filter], radii[update_filter])
        self.xyz_gradient_accum[update_filter] += torch.norm(viewspace_grad[update_filter, :2], dim=-1, keepdim=True)
        self.denom[update_filter] += 1

    # ---- densification and pruning (gaussian_model.py:316-506) as row plans over the old rows (surgery.py):
    # every per-Gaussian tensor, its Adam moments and statistics rebuilt in one pass per event
    def _row_ids(self, mask):
        return torch.nonzero(mask, as_tuple=False).flatten()

    def prune_points(self, mask):
        """Drop the rows where mask is True; surviving rows keep their moments and statistics."""
        surgery.apply(self, surgery.RowPlan(keep=self._row_ids(~mask)))

    def _max_scale(self):
        return torch.max(self.get_scaling, dim=1).values

    def _clone_rows(self, grads, grad_threshold, scene_extent):
        """gaussian_model.py:443-457's choice: accumulated gradient at or above the threshold, small Gaussians."""
        hot = torch.norm(grads, dim=-1) >= grad_threshold
        return self._row_ids(hot & (self._max_scale() <= self.percent_dense * scene_extent))

    def _split_rows(self, grads, grad_threshold, scene_extent):
        """gaussian_model.py:415-423's choice: the same gradient test on large Gaussians.  (The reference pads the
        gradient with zeros for rows cloned just before, which therefore never split: only old rows can.)"""
        g = grads.reshape(-1)
        return self._row_ids((g >= grad_threshold) & (self._max_scale() > self.percent_dense * scene_extent))

    def _split_children(self, ids, N):
        """Positions and scales of the N children of each row in ids (gaussian_model.py:424-431), children
        ordered copy after copy; the sampling draws the same normals, in the same order, as the reference."""
        dev = self._xyz.device
        scale = self.get_scaling[ids].repeat(N, 1)
        offsets = torch.normal(mean=torch.zeros((scale.size(0), 3), device=dev), std=scale)
        # data-parallel replicas select the same Gaussians (their statistics are all-reduced) but draw
        # from their own RNGs: rank 0's draws are the ones every replica uses
        from . import dp
        if getattr(self, "data_parallel_step", False) and dp.world() > 1:
            torch.distributed.broadcast(offsets, src=0)
        rot = build_rotation(self._rotation[ids]).repeat(N, 1, 1)
        xyz = torch.bmm(rot, offsets.unsqueeze(-1)).squeeze(-1) + self.get_xyz[ids].repeat(N, 1)
        return xyz, self.scaling_inverse_activation(scale / (0.8 * N))

    def _grow(self, clone_ids, split_ids, N=2):
        """One plan for a clone pass followed by a split pass: the rows not split, the clones, the children.
        Statistics restart at zero (densification_postfix)."""
        dev = self._xyz.device
        keep = torch.ones(self._xyz.shape[0], dtype=torch.bool, device=dev)
        keep[split_ids] = False
        computed, n_split = {}, split_ids.numel()
        if n_split:
            computed["xyz"], computed["scaling"] = self._split_children(split_ids, N)
        plan = surgery.RowPlan(keep=self._row_ids(keep), append=torch.cat([clone_ids] + [split_ids] * N),
                               computed=computed, n_new=clone_ids.numel() + N * n_split, stats="reset")
        surgery.apply(self, plan)

    def densify_and_clone(self, grads, grad_threshold, scene_extent):
        """gaussian_model.py:443-457"""
        empty = self._row_ids(torch.zeros(0, dtype=torch.bool, device=self._xyz.device))
        self._grow(self._clone_rows(grads, grad_threshold, scene_extent), empty)

    def densify_and_split(self, grads, grad_threshold, scene_extent, N=2):
        """gaussian_model.py:415-441 (a no-op when nothing is selected, as there)"""
        ids = self._split_rows(grads[:self._xyz.shape[0]], grad_threshold, scene_extent)
        if ids.numel():
            self._grow(ids[:0], ids, N)

    def prune(self, max_grad, min_opacity, extent, max_screen_size):
        """gaussian_model.py:489-499"""
        drop = (self.get_opacity < min_opacity).squeeze()
        if max_screen_size:
            drop = drop | (self.max_radii2D > max_screen_size) | (self._max_scale() > 0.1 * extent)
        self.prune_points(drop)

    def densify(self, max_grad, min_opacity, extent, max_screen_size):
        """gaussian_model.py:501-506: clone then split, as ONE row plan (the two passes' combined result)."""
        grads = self.xyz_gradient_accum / self.denom
        grads[grads.isnan()] = 0.0
        self._grow(self._clone_rows(grads, max_grad, extent), self._split_rows(grads, max_grad, extent))

    def reset_opacity(self):
        """gaussian_model.py:269-272"""
        surgery.replace_param(self, "opacity",
                              inverse_sigmoid(torch.min(self.get_opacity, torch.ones_like(self.get_opacity) * 0.01)))

    # ---- HexPlane regularisers (gaussian_model.py:538-566)
    def compute_regulation(self, time_smoothness_weight, l1_time_planes_weight, plane_tv_weight):
        grids = self._deformation.deformation_net.grid.grids
        if self.fused:
            from .kernels import hexplane_regulation
            return hexplane_regulation([list(g) for g in grids], time_smoothness_weight, l1_time_planes_weight,
                                       plane_tv_weight)
        plane = sum(compute_plane_smoothness(g[i]) for g in grids for i in ([] if len(g) == 3 else [0, 1, 3]))
        time = sum(compute_plane_smoothness(g[i]) for g in grids for i in ([] if len(g) == 3 else [2, 4, 5]))
        l1 = sum(torch.abs(1 - g[i]).mean() for g in grids if len(g) != 3 for i in [2, 4, 5])
        return plane_tv_weight * plane + time_smoothness_weight * time + l1_time_planes_weight * l1

    def regulation_value(self, time_smoothness_weight, l1_time_planes_weight, plane_tv_weight):
        """compute_regulation's value with no autograd graph (fused path; see add_regulation_grad)."""
        from .kernels import hexplane_regulation_value
        grids = self._deformation.deformation_net.grid.grids
        return hexplane_regulation_value([list(g) for g in grids], time_smoothness_weight, l1_time_planes_weight,
                                         plane_tv_weight)

    def add_regulation_grad(self, time_smoothness_weight, l1_time_planes_weight, plane_tv_weight, scale=1.0,
                            with_value=False, base=None):
        """scale * d(compute_regulation)/d(plane) added to the planes' .grad in one launch: the gradient
        the loss's regulariser term contributes, applied after the rest of the backward.  with_value: returns
        compute_regulation's value too, from the same pass (regulation_value's number, bitwise); with base (a
        one-value device tensor), base + that value, added by the same launch."""
        from .kernels import hexplane_regulation_accumulate_grad
        grids = self._deformation.deformation_net.grid.grids
        return hexplane_regulation_accumulate_grad([list(g) for g in grids], time_smoothness_weight,
                                                   l1_time_planes_weight, plane_tv_weight, scale, with_value, base)

    # ---- on-disk formats (gaussian_model.py:214-314 and scene/__init__.py:143-150)
    def save_ply(self, path):
        from .ply import save_gaussians
        save_gaussians(path, self)

    def load_ply(self, path, device="cuda"):
        from .ply import load_gaussians
        load_gaussians(path, self, device)
