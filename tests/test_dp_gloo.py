"""Multi-process (gloo, world_size 2, CPU) tests of the data-parallel view sharding (gs4d_train/dp.py).

The renderer is a parameter of dp.batch_step; here a small differentiable torch stand-in is used, since
the HIP path needs a GPU.  The property checked is the DP contract of SURVEY §8e: every rank ends with
the batch loss and parameter gradients of the single-process batch.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gs4d_train import dp

NUM_VIEWS = 5


def make_params():
    g = torch.Generator().manual_seed(0)
    return {"means3D": torch.randn(64, 3, generator=g), "opacities": torch.rand(64, 1, generator=g),
            "shs": torch.randn(64, 16, 3, generator=g)}


def make_views():
    g = torch.Generator().manual_seed(1)
    return [{"A": torch.randn(3, 4, generator=g), "gt": torch.rand(64, 4, generator=g)} for _ in range(NUM_VIEWS)]


def render_loss(p, v):
    img = torch.sigmoid(p["means3D"] @ v["A"]) * p["opacities"] + p["shs"][:, 0, :1]
    return (img - v["gt"]).abs().mean()


def reference():
    params = {k: t.clone().requires_grad_(True) for k, t in make_params().items()}
    views = make_views()
    loss = sum(render_loss(params, v) for v in views) / NUM_VIEWS
    loss.backward()
    return loss.detach(), {k: t.grad.clone() for k, t in params.items()}


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(r, w, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=r, world_size=w)
    try:
        params = {k: t.clone().requires_grad_(True) for k, t in make_params().items()}
        loss = dp.batch_step(params, make_views(), render_loss, NUM_VIEWS, bucket_mb=0.01)
        out[r] = (loss.clone(), {k: t.grad.clone() for k, t in params.items()}, dp.shard_views(NUM_VIEWS))
    finally:
        dist.destroy_process_group()


def test_shard_views_partition():
    for w in (1, 2, 3, 8):
        got = sorted(v for r in range(w) for v in dp.shard_views(17, r, w))
        assert got == list(range(17))
        sizes = [len(dp.shard_views(17, r, w)) for r in range(w)]
        assert max(sizes) - min(sizes) <= 1


def test_allreduce_single_process_is_identity():
    t = [torch.arange(5.0), torch.ones(3, 2)]
    before = [x.clone() for x in t]
    dp.allreduce_sum_(t)
    assert all(torch.equal(a, b) for a, b in zip(t, before))


@pytest.mark.timeout(120)
def test_batch_step_world2_matches_single_process():
    ref_loss, ref_grads = reference()
    mgr = mp.Manager()
    out = mgr.dict()
    port = _free_port()
    mp.start_processes(_worker, args=(2, port, out), nprocs=2, join=True, start_method="spawn")
    assert set(out.keys()) == {0, 1}
    assert out[0][2] == [0, 2, 4] and out[1][2] == [1, 3]
    for r in (0, 1):
        loss, grads, _ = out[r]
        torch.testing.assert_close(loss.reshape(()), ref_loss, rtol=1e-6, atol=1e-7)
        for k, g in ref_grads.items():
            torch.testing.assert_close(grads[k], g, rtol=1e-5, atol=1e-7)
    # both replicas hold bit-identical gradients (the all-reduce result is shared)
    for k in ref_grads:
        assert torch.equal(out[0][1][k], out[1][1][k])
