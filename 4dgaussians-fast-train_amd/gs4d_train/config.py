"""Hyper-parameter groups of the reference (arguments/__init__.py) as plain namespaces.

`model_hidden_params()` / `optimization_params()` return the reference defaults
(arguments/__init__.py:77-107 and :109-156); the per-dataset files of arguments/ override a few of
them, e.g. `DYNERF` mirrors arguments/dynerf/default.py (the BASELINE.json metric's camera size)
and `DNERF` arguments/dnerf/dnerf_default.py.
"""
from types import SimpleNamespace


def model_hidden_params(**over):
    d = dict(net_width=64, timebase_pe=4, defor_depth=1, posebase_pe=10, scale_rotation_pe=2, opacity_pe=2,
             timenet_width=64, timenet_output=32, bounds=1.6, plane_tv_weight=0.0001, time_smoothness_weight=0.01,
             l1_time_planes=0.0001,
             kplanes_config={"grid_dimensions": 2, "input_coordinate_dim": 4, "output_coordinate_dim": 32,
                             "resolution": [64, 64, 64, 25]},
             multires=[1, 2, 4, 8], no_dx=False, no_grid=False, no_ds=False, no_dr=False, no_do=True, no_dshs=True,
             empty_voxel=False, grid_pe=0, static_mlp=False, apply_rotation=False,
             mlp_dtype="fp32")  # this build's opt-in: "bf16" deformation MLP GEMMs (deformation.py)
    d.update(over)
    return SimpleNamespace(**d)


def optimization_params(**over):
    d = dict(dataloader=False, iterations=30_000, coarse_iterations=3000, position_lr_init=0.00016,
             position_lr_final=0.0000016, position_lr_delay_mult=0.01, position_lr_max_steps=20_000,
             deformation_lr_init=0.00016, deformation_lr_final=0.000016, deformation_lr_delay_mult=0.01,
             grid_lr_init=0.0016, grid_lr_final=0.00016, feature_lr=0.0025, opacity_lr=0.05, scaling_lr=0.005,
             rotation_lr=0.001, percent_dense=0.01, lambda_dssim=0, lambda_lpips=0, opacity_reset_interval=3000,
             densification_interval=100, densify_from_iter=500, densify_until_iter=15_000,
             densify_grad_threshold_coarse=0.0002, densify_grad_threshold_fine_init=0.0002,
             densify_grad_threshold_after=0.0002, pruning_from_iter=500, pruning_interval=100,
             opacity_threshold_coarse=0.005, opacity_threshold_fine_init=0.005, opacity_threshold_fine_after=0.005,
             batch_size=1, add_point=False)
    d.update(over)
    return SimpleNamespace(**d)


# arguments/dynerf/default.py
DYNERF_HIDDEN = dict(kplanes_config={"grid_dimensions": 2, "input_coordinate_dim": 4, "output_coordinate_dim": 16,
                                     "resolution": [64, 64, 64, 150]},
                     multires=[1, 2], defor_depth=0, net_width=128, plane_tv_weight=0.0002,
                     time_smoothness_weight=0.001, l1_time_planes=0.0001, no_do=False, no_dshs=False,
                     empty_voxel=False, static_mlp=False)
DYNERF_OPT = dict(dataloader=True, iterations=14000, batch_size=4, coarse_iterations=3000, densify_until_iter=10_000,
                  opacity_reset_interval=60000, opacity_threshold_coarse=0.005, opacity_threshold_fine_init=0.005,
                  opacity_threshold_fine_after=0.005)
# arguments/dnerf/dnerf_default.py
DNERF_HIDDEN = dict(multires=[1, 2], defor_depth=0, net_width=64, plane_tv_weight=0.0001,
                    time_smoothness_weight=0.01, l1_time_planes=0.0001, weight_decay_iteration=0, bounds=1.6)
DNERF_OPT = dict(coarse_iterations=3000, deformation_lr_init=0.00016, deformation_lr_final=0.0000016,
                 deformation_lr_delay_mult=0.01, grid_lr_init=0.0016, grid_lr_final=0.000016, iterations=20000,
                 pruning_interval=8000, percent_dense=0.01)


def dynerf():
    return model_hidden_params(**DYNERF_HIDDEN), optimization_params(**DYNERF_OPT)


def dnerf():
    return model_hidden_params(**DNERF_HIDDEN), optimization_params(**DNERF_OPT)
