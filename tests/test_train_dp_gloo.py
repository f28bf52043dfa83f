"""Multi-process (gloo, world size 2, CPU) tests of the data-parallel train step (gs4d_train.train).

train_step(..., data_parallel=True) shards a batch's views over the ranks and reduces gradients and
densification statistics so that every replica takes the single-process step.  The
rasterizer is replaced by a small differentiable torch splatter with render()'s return dict (the HIP
path needs a GPU); the model, the optimizer, the statistics and the densification are the real
gs4d_train code on CPU (fused=False: torch.optim.Adam and the torch formulations).

Covered: a rank that receives no view of the batch (1 view on 2 ranks, coarse stage: no regulariser,
so that rank's loss is a constant), and a step that crosses a densification iteration (clone + split,
whose split samples come from each rank's own RNG unless shared).
"""
import os
import socket
from types import SimpleNamespace

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gs4d_train import config
from gs4d_train.gaussians import GaussianModel

H = W = 6


def make_model(P=200, seed=0):
    hyper, opt = config.dnerf()
    torch.manual_seed(seed)
    g = GaussianModel(3, hyper, fused=False)
    rng = np.random.default_rng(seed)
    f32 = lambda a: torch.tensor(a, dtype=torch.float32)
    g._xyz = torch.nn.Parameter(f32(rng.normal(size=(P, 3))))
    g._features_dc = torch.nn.Parameter(f32(rng.normal(size=(P, 1, 3))))
    g._features_rest = torch.nn.Parameter(f32(rng.normal(size=(P, 15, 3))))
    sc = rng.normal(-3, 0.5, size=(P, 3))
    sc[::4] = -6.0                       # a quarter small enough to clone instead of split
    g._scaling = torch.nn.Parameter(f32(sc))
    g._rotation = torch.nn.Parameter(f32(rng.normal(size=(P, 4))))
    g._opacity = torch.nn.Parameter(f32(rng.normal(size=(P, 1))))
    g.max_radii2D = torch.zeros(P)
    g._deformation_table = torch.ones(P, dtype=torch.bool)
    g.spatial_lr_scale = 1.0
    opt.densify_grad_threshold_coarse = 1e-9
    g.training_setup(opt)
    return g, hyper, opt


def make_views(n):
    g = torch.Generator().manual_seed(7)
    views = []
    for i in range(n):
        cam = SimpleNamespace(A=torch.randn(3, 2, generator=g) + 2.0, time=i / max(n, 1))
        views.append((cam, torch.rand(3, H, W, generator=g)))
    return views


def splat_render(cam, pc, debug, bg, stage="coarse"):
    """render()'s dict from a differentiable isotropic splatter (a stand-in for the rasterizer)."""
    xyz = pc.get_xyz
    ss = torch.zeros_like(xyz, requires_grad=True) + 0
    ss.retain_grad()
    m2 = xyz @ cam.A + ss[:, :2]
    s = pc.get_scaling.max(dim=1).values * 20
    op = pc.get_opacity[:, 0]
    col = pc.get_features[:, 0, :] * 0.28 + 0.5
    yy, xx = torch.meshgrid(torch.arange(H, dtype=torch.float32), torch.arange(W, dtype=torch.float32),
                            indexing="ij")
    pix = torch.stack([xx.reshape(-1), yy.reshape(-1)], 1)
    vis = xyz[:, 2] > 0
    wgt = (op * vis)[:, None] * torch.exp(-((pix[None] - m2[:, None]) ** 2).sum(-1) / (2 * s[:, None] ** 2 + 1))
    img = (wgt[:, :, None] * col[:, None, :]).sum(0) / (1 + wgt.sum(0)[:, None])
    radii = (torch.ceil(3 * s).to(torch.int32) * vis).to(torch.int32)
    return {"render": img.t().reshape(3, H, W), "viewspace_points": ss, "visibility_filter": radii > 0,
            "radii": radii, "depth": torch.zeros(1, H, W)}


def run_step(g, hyper, opt, views, iteration, data_parallel):
    from gs4d_train.train import train_step
    bg = torch.ones(3)
    return train_step(g, views, opt, hyper, iteration, bg, stage="coarse", data_parallel=data_parallel,
                      render_fn=splat_render)


def snapshot(g):
    out = {k: getattr(g, k).detach().clone() for k in ("_xyz", "_features_dc", "_features_rest", "_scaling",
                                                      "_rotation", "_opacity")}
    out["max_radii2D"] = g.max_radii2D.clone()
    out["denom"] = g.denom.clone()
    out["steps"] = [float(st["step"]) for st in g.optimizer.state.values()]
    return out


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(r, w, port, n_views, iteration, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=r, world_size=w)
    try:
        g, hyper, opt = make_model()
        torch.manual_seed(100 + r)       # replicas' RNGs differ on purpose
        loss = run_step(g, hyper, opt, make_views(n_views), iteration, True)
        out[r] = (float(loss), snapshot(g))
    finally:
        dist.destroy_process_group()


def single_process(n_views, iteration):
    g, hyper, opt = make_model()
    torch.manual_seed(100)               # rank 0's seed: its split samples are the ones every replica uses
    loss = run_step(g, hyper, opt, make_views(n_views), iteration, False)
    return float(loss), snapshot(g)


def _launch(n_views, iteration):
    mgr = mp.Manager()
    out = mgr.dict()
    mp.start_processes(_worker, args=(2, _free_port(), n_views, iteration, out), nprocs=2, join=True,
                       start_method="spawn")
    assert set(out.keys()) == {0, 1}
    return out[0], out[1]


def _check(ref, a, b):
    ref_loss, ref_s = ref
    for loss, s in (a, b):
        assert abs(loss - ref_loss) <= 1e-6 * max(1.0, abs(ref_loss))
        assert s["steps"] == ref_s["steps"]
        for k, v in ref_s.items():
            if k == "steps":
                continue
            assert s[k].shape == v.shape, k
            torch.testing.assert_close(s[k], v, rtol=1e-5, atol=1e-6, msg=k)
    for k in ref_s:                      # the replicas are bit-identical
        if k != "steps":
            assert torch.equal(a[1][k], b[1][k]), k


@pytest.mark.timeout(180)
def test_rank_without_views_coarse_stage():
    """1 view, 2 ranks: rank 1 renders nothing and has no regulariser (coarse); it must not call
    backward on a constant, and both replicas take the single-process step."""
    ref = single_process(1, 3001)
    a, b = _launch(1, 3001)
    _check(ref, a, b)


@pytest.mark.timeout(180)
def test_densification_keeps_replicas_identical():
    """A batch step at a densification iteration (600: clone + split): the split samples are drawn
    from rank 0's RNG on every replica, so replicas match each other and the single-process step."""
    ref = single_process(3, 600)
    P0 = 200
    assert ref[1]["_xyz"].shape[0] > P0      # densification did happen
    a, b = _launch(3, 600)
    _check(ref, a, b)
