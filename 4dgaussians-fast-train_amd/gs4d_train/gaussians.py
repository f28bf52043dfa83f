"""The Gaussian model around the rasterizer: parameters, activations, optimizer, densification.

Restates scene/gaussian_model.py of the reference (the train-step tail) for the
fine-stage training path: the same parameter tensors and activations (:29-45), the Adam parameter
groups and learning-rate schedules (:165-212), the densification statistics (:521-523), the
clone / split / prune tensor surgery on the optimizer state (:316-505), opacity reset (:269-272),
the HexPlane regularisers (:538-566) and the PLY layout (:214-226, 250-314; see gs4d_train/ply.py).

Three places run libgs4d HIP kernels when `fused=True` (the default on a GPU): the optimizer step
(one multi-tensor Adam launch, kernels.FusedAdam), the densification statistics
(kernels.densify_stats) and the HexPlane regularisers (kernels.hexplane_regulation).  `fused=False` keeps the reference's torch formulation, which the parity
tests compare against.
"""
import math

import numpy as np
import torch
import torch.nn as nn

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

    # ---- optimizer-state surgery (gaussian_model.py:316-413)
    def replace_tensor_to_optimizer(self, tensor, name):
        out = {}
        for group in self.optimizer.param_groups:
            if group["name"] == name:
                stored = self.optimizer.state.get(group["params"][0], None)
                stored["exp_avg"] = torch.zeros_like(tensor)
                stored["exp_avg_sq"] = torch.zeros_like(tensor)
                del self.optimizer.state[group["params"][0]]
                group["params"][0] = nn.Parameter(tensor.requires_grad_(True))
                self.optimizer.state[group["params"][0]] = stored
                out[group["name"]] = group["params"][0]
        return out

    def _prune_optimizer(self, mask):
        out = {}
        for group in self.optimizer.param_groups:
            if len(group["params"]) > 1:
                continue
            stored = self.optimizer.state.get(group["params"][0], None)
            if stored is not None:
                stored["exp_avg"] = stored["exp_avg"][mask]
                stored["exp_avg_sq"] = stored["exp_avg_sq"][mask]
                del self.optimizer.state[group["params"][0]]
                group["params"][0] = nn.Parameter(group["params"][0][mask].requires_grad_(True))
                self.optimizer.state[group["params"][0]] = stored
            else:
                group["params"][0] = nn.Parameter(group["params"][0][mask].requires_grad_(True))
            out[group["name"]] = group["params"][0]
        return out

    def _take(self, t):
        self._xyz, self._features_dc, self._features_rest = t["xyz"], t["f_dc"], t["f_rest"]
        self._opacity, self._scaling, self._rotation = t["opacity"], t["scaling"], t["rotation"]

    def prune_points(self, mask):
        valid = ~mask
        self._take(self._prune_optimizer(valid))
        self._deformation_accum = self._deformation_accum[valid]
        self.xyz_gradient_accum = self.xyz_gradient_accum[valid]
        self._deformation_table = self._deformation_table[valid]
        self.denom = self.denom[valid]
        self.max_radii2D = self.max_radii2D[valid]

    def cat_tensors_to_optimizer(self, tensors_dict):
        out = {}
        for group in self.optimizer.param_groups:
            if len(group["params"]) > 1:
                continue
            ext = tensors_dict[group["name"]]
            stored = self.optimizer.state.get(group["params"][0], None)
            if stored is not None:
                stored["exp_avg"] = torch.cat((stored["exp_avg"], torch.zeros_like(ext)), dim=0)
                stored["exp_avg_sq"] = torch.cat((stored["exp_avg_sq"], torch.zeros_like(ext)), dim=0)
                del self.optimizer.state[group["params"][0]]
                group["params"][0] = nn.Parameter(torch.cat((group["params"][0], ext), dim=0).requires_grad_(True))
                self.optimizer.state[group["params"][0]] = stored
            else:
                group["params"][0] = nn.Parameter(torch.cat((group["params"][0], ext), dim=0).requires_grad_(True))
            out[group["name"]] = group["params"][0]
        return out

    def densification_postfix(self, new_xyz, new_features_dc, new_features_rest, new_opacities, new_scaling,
                              new_rotation, new_deformation_table):
        dev = self._xyz.device
        self._take(self.cat_tensors_to_optimizer({"xyz": new_xyz, "f_dc": new_features_dc,
                                                  "f_rest": new_features_rest, "opacity": new_opacities,
                                                  "scaling": new_scaling, "rotation": new_rotation}))
        self._deformation_table = torch.cat([self._deformation_table, new_deformation_table], -1)
        P = self.get_xyz.shape[0]
        self.xyz_gradient_accum = torch.zeros((P, 1), device=dev)
        self._deformation_accum = torch.zeros((P, 3), device=dev)
        self.denom = torch.zeros((P, 1), device=dev)
        self.max_radii2D = torch.zeros((P), device=dev)

    def densify_and_split(self, grads, grad_threshold, scene_extent, N=2):
        """gaussian_model.py:415-441"""
        dev = self._xyz.device
        n_init = self.get_xyz.shape[0]
        padded = torch.zeros((n_init), device=dev)
        padded[:grads.shape[0]] = grads.squeeze()
        sel = torch.where(padded >= grad_threshold, True, False)
        sel = torch.logical_and(sel, torch.max(self.get_scaling, dim=1).values > self.percent_dense * scene_extent)
        if not sel.any():
            return
        stds = self.get_scaling[sel].repeat(N, 1)
        samples = torch.normal(mean=torch.zeros((stds.size(0), 3), device=dev), std=stds)
        # data-parallel replicas select the same Gaussians (their statistics are all-reduced) but draw
        # from their own RNGs: rank 0's draws are the ones every replica uses
        from . import dp
        if getattr(self, "data_parallel_step", False) and dp.world() > 1:
            torch.distributed.broadcast(samples, src=0)
        rots = build_rotation(self._rotation[sel]).repeat(N, 1, 1)
        new_xyz = torch.bmm(rots, samples.unsqueeze(-1)).squeeze(-1) + self.get_xyz[sel].repeat(N, 1)
        new_scaling = self.scaling_inverse_activation(self.get_scaling[sel].repeat(N, 1) / (0.8 * N))
        self.densification_postfix(new_xyz, self._features_dc[sel].repeat(N, 1, 1),
                                   self._features_rest[sel].repeat(N, 1, 1), self._opacity[sel].repeat(N, 1),
                                   new_scaling, self._rotation[sel].repeat(N, 1), self._deformation_table[sel].repeat(N))
        prune_filter = torch.cat((sel, torch.zeros(N * sel.sum(), device=dev, dtype=bool)))
        self.prune_points(prune_filter)

    def densify_and_clone(self, grads, grad_threshold, scene_extent):
        """gaussian_model.py:443-457"""
        mask = torch.where(torch.norm(grads, dim=-1) >= grad_threshold, True, False)
        sel = torch.logical_and(mask, torch.max(self.get_scaling, dim=1).values <= self.percent_dense * scene_extent)
        self.densification_postfix(self._xyz[sel], self._features_dc[sel], self._features_rest[sel],
                                   self._opacity[sel], self._scaling[sel], self._rotation[sel],
                                   self._deformation_table[sel])

    def prune(self, max_grad, min_opacity, extent, max_screen_size):
        """gaussian_model.py:489-499"""
        prune_mask = (self.get_opacity < min_opacity).squeeze()
        if max_screen_size:
            big_vs = self.max_radii2D > max_screen_size
            big_ws = self.get_scaling.max(dim=1).values > 0.1 * extent
            prune_mask = torch.logical_or(torch.logical_or(prune_mask, big_vs), big_ws)
        self.prune_points(prune_mask)

    def densify(self, max_grad, min_opacity, extent, max_screen_size):
        """gaussian_model.py:501-506"""
        grads = self.xyz_gradient_accum / self.denom
        grads[grads.isnan()] = 0.0
        self.densify_and_clone(grads, max_grad, extent)
        self.densify_and_split(grads, max_grad, extent)

    def reset_opacity(self):
        """gaussian_model.py:269-272"""
        new = inverse_sigmoid(torch.min(self.get_opacity, torch.ones_like(self.get_opacity) * 0.01))
        self._opacity = self.replace_tensor_to_optimizer(new, "opacity")["opacity"]

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
