"""Training quality: a synthetic stand-in for north_star's "matching reference PSNR on D-NeRF bouncingballs".

The reference quotes 38.327 dB on bouncingballs after 20k iterations (4DGaussians.ipynb:442; loop
train.py:110-401).  Neither the dataset nor the reference's CUDA build exists here, so the number itself
cannot be reproduced.  These tests check what can be: that the MI355X training path LEARNS a dynamic
scene, and that the fused HIP kernels train it as the reference's own PyTorch formulation does.

  * Scene: three coloured balls of Gaussians bouncing over t in [0, 1] (gs4d_train.synthetic.
    bouncing_balls), white background.  Ground-truth frames are rendered by the CPU ORACLE (the
    restatement of the reference rasterizer), not by the code under test: 24 training views and 6
    held-out test views, each camera at its own time and angle (the D-NeRF setup: one timestamp per
    image).
  * Training: the reference's schedule in miniature -- D-NeRF hyper-parameters (arguments/dnerf/
    dnerf_default.py), its random 2,000-point initialisation (scene/dataset_readers.py:364-370),
    a coarse stage without deformation and a fine stage with the HexPlane field + deformation MLP,
    densification every 100 iterations past 500, one random view per iteration (batch 1).
  * Fused (libgs4d HexPlane field, heads, L1, Adam, statistics kernels) against unfused (the
    reference's torch grid_sample / L1 / Adam formulation); both use the HIP rasterizer.

Training is chaotic in the rounding: the two formulations agree per step to ~1e-7 (test_train_gpu.py),
but Adam's first steps turn the sign of near-zero gradients into full-size updates and densification
thresholds accumulated gradients, so the trajectories of two formulations that differ only in rounding fan out.
What the tests can assert is therefore statistical, with bars set from measurements:
  * the fused arm is bitwise reproducible across processes (round 6: every kernel of the fused step sums in a
    fixed order, the MLP's large GEMMs included -- round 5's timing-tuned library GEMMs were not, and its
    per-seed bar failed on the driver); the unfused arm is not (torch's grid_sample backward sums with float
    atomics);
  * measured over 12 seeds at 200 + 200 iterations, two processes (tools/probes/conv_spread.py,
    profiles/r06/conv_spread_{a,b}.log): the unfused arm's run-to-run difference has sd 0.025-0.026 dB (so
    one run's sd is ~0.018), the fused-minus-unfused per-seed gap sd 0.052-0.054 dB with mean -0.009 / -0.020 dB
    and largest |gap| 0.136 dB;
  * short horizon (no densification, 200 + 200 iterations, SHORT_SEEDS = 12): each seed's gap within
    SHORT_RUN_DELTA = 0.25 dB (4.7 sigma of the measured gap: false failure ~3e-6 per seed, ~3e-5 over 12), the
    12-seed mean gap within SHORT_DELTA = 0.07 dB (4.6 sigma of the mean, sigma = 0.053 / sqrt(12): ~4e-6),
    and the last-50-iteration mean losses within 1 %;
  * long horizon (the full miniature schedule, 5 seeds each): every run converges (above RUN_FLOOR and
    PSNR_GAIN over its start), each formulation's median above PSNR_FLOOR, the median fused PSNR within
    PSNR_DELTA of the median unfused PSNR, and the same for the fused run with the opt-in bf16
    deformation MLP (3 seeds).  Medians, because a run now and then loses ~2 dB to an unlucky
    densification (an unfused run at 26.4 dB, train 31.9, among 28-29 dB runs): the claim is about the
    formulations, not one trajectory.
This file sorts after the parity suites (test_gpu_parity, test_knn, test_train_gpu): a statistical failure here
cannot hide their results under `pytest -x`.
"""
import copy
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

W, H = 160, 120
N_TRAIN, N_TEST = 24, 6
K_COARSE, K_FINE = 800, 2500   # no opacity reset in range (opacity_reset_interval = 3000)
PSNR_FLOOR = 27.0     # dB, median held-out PSNR after K_COARSE + K_FINE iterations (runs measured 26.4-29.5)
RUN_FLOOR = 25.0      # dB, every run
PSNR_GAIN = 15.0      # dB over the initial random point cloud (8.5-8.7 dB)
PSNR_DELTA = 1.0      # dB between the medians of the fused and the unfused runs
SEEDS = 5
SHORT_DELTA = 0.07    # dB, |mean over SHORT_SEEDS seeds of (fused - unfused)|: 4.6 sigma of the measured mean (docstring)
SHORT_RUN_DELTA = 0.25  # dB, |fused - unfused| at any one seed: 4.7 sigma of the measured per-seed gap (docstring)
SHORT_SEEDS = 12


def _cameras(n, seed, offset):
    from gs4d_train.synthetic import look_at_camera
    rng = np.random.default_rng(seed)
    cams = []
    for v in range(n):
        a = 2 * math.pi * ((v + offset) / n) + rng.uniform(-0.1, 0.1)
        elev = rng.uniform(0.15, 0.45)
        c = 4.0 * np.array([math.cos(elev) * math.sin(a), math.sin(elev), -math.cos(elev) * math.cos(a)])
        cams.append(look_at_camera(W, H, c, time=float(rng.uniform(0, 1))))
    return cams


@pytest.fixture(scope="module")
def dataset():
    if not torch.cuda.is_available():
        pytest.skip("needs an MI355X")
    return make_dataset()


def make_dataset():
    """GT images of the bouncing balls, rendered by the oracle at each camera's time."""
    from oracle import oracle as O
    from gs4d_train.synthetic import bouncing_balls
    canon, means_at = bouncing_balls(n_per_ball=1000, seed=3)
    bg = np.ones(3, np.float32)

    def gt(cam):
        nr, color, depth, radii, st = O.rasterize_forward(
            bg, means_at(cam.time), None, canon["opacities"], canon["scales"], canon["rotations"], 1.0, None,
            cam.world_view_transform.numpy().astype(np.float32), cam.full_proj_transform.numpy().astype(np.float32),
            cam.tanfovx, cam.tanfovy, H, W, canon["shs"], 0, cam.camera_center.numpy().astype(np.float32))
        return torch.tensor(color, device="cuda")
    train = [(c, gt(c)) for c in _cameras(N_TRAIN, seed=1, offset=0.0)]
    test = [(c, gt(c)) for c in _cameras(N_TEST, seed=2, offset=0.5)]
    return train, test


def _extent(views):
    """getNerfppNorm (scene/dataset_readers.py:86-107): 1.1 x the largest camera distance from their mean."""
    cs = np.stack([c.camera_center.numpy() for c, _ in views])
    return 1.1 * float(np.linalg.norm(cs - cs.mean(0), axis=1).max())


def _evaluate(g, views, bg):
    from gs4d_train.losses import psnr
    from gs4d_train.render import render
    with torch.no_grad():
        vals = [float(psnr(render(c, g, False, bg, stage="fine")["render"].unsqueeze(0).clamp(0, 1),
                           gt.unsqueeze(0))) for c, gt in views]
    return float(np.mean(vals))


def _train(dataset, fused, seed=0, k_coarse=K_COARSE, k_fine=K_FINE, densify=True, losses=None, mlp_dtype="fp32"):
    from gs4d_train import config
    from gs4d_train.gaussians import GaussianModel
    from gs4d_train.train import train_step
    train_views, test_views = dataset
    hyper, opt = config.dnerf()
    hyper.mlp_dtype = mlp_dtype
    opt_c, opt_f = copy.copy(opt), copy.copy(opt)
    opt_c.iterations, opt_f.iterations = k_coarse, k_fine
    if not densify:
        opt_c.densify_from_iter = opt_f.densify_from_iter = 10 ** 9
    extent = _extent(train_views)
    torch.manual_seed(seed)
    rng = np.random.default_rng(seed)
    # scene/dataset_readers.py:364-370: 2,000 uniform points in [-1.3, 1.3]^3, colours SH2RGB(U(0,1)/255)
    pts = (rng.random((2000, 3)) * 2.6 - 1.3).astype(np.float32)
    cols = ((rng.random((2000, 3)) / 255.0) * 0.28209479177387814 + 0.5).astype(np.float32)
    g = GaussianModel(3, hyper, fused=fused)
    g.create_from_pcd(pts, cols, spatial_lr_scale=extent, device="cuda")
    g.cameras_extent = extent
    g._deformation.deformation_net.grid.fused = fused
    g._deformation.deformation_net.fused_heads = fused
    bg = torch.ones(3, device="cuda")
    init_psnr = _evaluate(g, test_views, bg)
    for stage, o, K in (("coarse", opt_c, k_coarse), ("fine", opt_f, k_fine)):
        g.training_setup(o)  # train.py: scene_reconstruction sets the optimizer up per stage
        for it in range(1, K + 1):
            v = int(rng.integers(len(train_views)))
            loss = train_step(g, [train_views[v]], o, hyper, it, bg, stage=stage)
            if losses is not None and stage == "fine":
                losses.append(loss)
    torch.cuda.synchronize()
    return init_psnr, _evaluate(g, test_views, bg), _evaluate(g, train_views, bg), g.get_xyz.shape[0]


def test_short_horizon_fused_matches_unfused(dataset):
    test = {True: [], False: []}
    for seed in range(SHORT_SEEDS):
        res, curves = {}, {}
        for fused in (True, False):
            curves[fused] = []
            res[fused] = _train(dataset, fused, seed=seed, k_coarse=200, k_fine=200, densify=False,
                                losses=curves[fused])
            test[fused].append(res[fused][1])
            print(f"short seed {seed} fused={fused}: init {res[fused][0]:.3f} dB -> test {res[fused][1]:.3f} dB, "
                  f"train {res[fused][2]:.3f} dB")
        la = float(torch.stack(curves[True][-50:]).mean())
        lb = float(torch.stack(curves[False][-50:]).mean())
        assert abs(res[True][0] - res[False][0]) < 1e-3   # same initial model
        assert abs(la - lb) <= 0.01 * lb, (seed, la, lb)
        assert abs(res[True][1] - res[False][1]) <= SHORT_RUN_DELTA, (seed, res[True][1], res[False][1])
    mf, mu = float(np.mean(test[True])), float(np.mean(test[False]))
    gaps = np.array(test[True]) - np.array(test[False])
    print(f"short mean test PSNR: fused {mf:.3f} dB, unfused {mu:.3f} dB; per-seed gap sd {gaps.std(ddof=1):.3f} dB")
    assert abs(mf - mu) <= SHORT_DELTA, (mf, mu)


def test_long_horizon_psnr(dataset):
    res = {True: [], False: []}
    for seed in range(SEEDS):
        for fused in (True, False):
            r = _train(dataset, fused, seed=seed)
            res[fused].append(r)
            print(f"seed {seed} fused={fused}: init {r[0]:.2f} dB -> test {r[1]:.2f} dB, train {r[2]:.2f} dB, "
                  f"{r[3]} Gaussians")
    for fused in (True, False):
        for init, test, train, n in res[fused]:
            assert test >= RUN_FLOOR, (fused, test)
            assert test >= init + PSNR_GAIN, (fused, init, test)
    mf = float(np.median([r[1] for r in res[True]]))
    mu = float(np.median([r[1] for r in res[False]]))
    # the opt-in bf16 deformation MLP (BASELINE C3's "bf16/fp32") trains the same scene as well
    rb = [_train(dataset, True, seed=seed, mlp_dtype="bf16") for seed in range(3)]
    mb = float(np.median([r[1] for r in rb]))
    print(f"median test PSNR: fused {mf:.2f} dB, unfused {mu:.2f} dB, fused + bf16 MLP {mb:.2f} dB "
          f"({', '.join(f'{r[1]:.2f}' for r in rb)})")
    assert mf >= PSNR_FLOOR and mu >= PSNR_FLOOR, (mf, mu)
    assert abs(mf - mu) <= PSNR_DELTA, (mf, mu)
    assert min(r[1] for r in rb) >= RUN_FLOOR, [r[1] for r in rb]
    assert mb >= PSNR_FLOOR and abs(mb - mf) <= PSNR_DELTA, (mb, mf)
