"""CPU tests of the train-step harness around the rasterizer, no GPU calls:

* the HexPlane field's torch graph (gs4d_train.deformation, the parity reference of the fused HIP
  kernel) against an independent numpy restatement of grid_sample(bilinear, align_corners=True,
  border) and the per-level plane product of scene/hexplane.py:75-110;
* state-dict names and shapes of the deformation network as scene/deformation.py builds them, so a
  reference deformation.pth loads;
* the PLY layout of scene/gaussian_model.py:214-314 (header, attribute order, round trip);
* the optimizer-state surgery of densify / prune / reset_opacity with torch.optim.Adam;
* the learning-rate schedule of utils/general_utils.get_expon_lr_func.
"""
import itertools
import math
import os

import numpy as np
import pytest
import torch

from gs4d_train import config
from gs4d_train.deformation import DeformNetwork, HexPlaneField, interpolate_ms_features
from gs4d_train.gaussians import GaussianModel, get_expon_lr_func
from gs4d_train import ply


def np_grid_sample_border(plane, x, y):
    """plane (F, H, W); x, y in [-1, 1] (clipped): bilinear, align_corners=True, border padding."""
    F, H, W = plane.shape
    ix = np.clip((x + 1) / 2 * (W - 1), 0, W - 1)
    iy = np.clip((y + 1) / 2 * (H - 1), 0, H - 1)
    x0, y0 = np.floor(ix).astype(int), np.floor(iy).astype(int)
    x1, y1 = x0 + 1, y0 + 1
    out = np.zeros((len(x), F))
    for xx, yy, w in ((x0, y0, (x1 - ix) * (y1 - iy)), (x1, y0, (ix - x0) * (y1 - iy)),
                      (x0, y1, (x1 - ix) * (iy - y0)), (x1, y1, (ix - x0) * (iy - y0))):
        ok = (xx >= 0) & (xx < W) & (yy >= 0) & (yy < H)
        out[ok] += plane[:, yy[ok], xx[ok]].T * w[ok, None]
    return out


def test_hexplane_torch_graph_matches_numpy():
    torch.manual_seed(0)
    f = HexPlaneField(1.6, {"grid_dimensions": 2, "input_coordinate_dim": 4, "output_coordinate_dim": 8,
                            "resolution": [16, 12, 10, 7]}, [1, 2])
    with torch.no_grad():
        for level in f.grids:
            for p in level:
                p.uniform_(0.2, 1.1)
    rng = np.random.default_rng(1)
    pts = rng.uniform(-1.2, 1.2, (500, 4)).astype(np.float32)
    out = interpolate_ms_features(torch.tensor(pts), f.grids).detach().numpy()
    ref = []
    for level in f.grids:
        prod = np.ones((500, 8))
        for ci, (a, b) in enumerate(itertools.combinations(range(4), 2)):
            prod = prod * np_grid_sample_border(level[ci].detach().numpy()[0].astype(np.float64), pts[:, a], pts[:, b])
        ref.append(prod)
    np.testing.assert_allclose(out, np.concatenate(ref, 1), rtol=2e-5, atol=1e-6)
    # plane shapes: (1, F, reso[c1], reso[c0]) with the spatial resolution scaled per level
    assert tuple(f.grids[0][0].shape) == (1, 8, 12, 16) and tuple(f.grids[1][2].shape) == (1, 8, 7, 32)
    # time planes start at 1 only when initialised fresh
    g = HexPlaneField(1.6, {"grid_dimensions": 2, "input_coordinate_dim": 4, "output_coordinate_dim": 4,
                            "resolution": [8, 8, 8, 5]}, [1])
    assert torch.all(g.grids[0][2] == 1) and not torch.all(g.grids[0][0] == 1)


def test_deformation_state_dict_matches_reference_names():
    hyper, _ = config.dynerf()
    sd = DeformNetwork(hyper).state_dict()
    expect = {
        "deformation_net.grid.aabb": (2, 3),
        "deformation_net.grid.grids.0.0": (1, 16, 64, 64),
        "deformation_net.grid.grids.0.2": (1, 16, 150, 64),
        "deformation_net.grid.grids.1.5": (1, 16, 150, 128),
        "deformation_net.feature_out.0.weight": (128, 32),
        "deformation_net.pos_deform.1.weight": (128, 128),
        "deformation_net.pos_deform.3.weight": (3, 128),
        "deformation_net.rotations_deform.3.weight": (4, 128),
        "deformation_net.shs_deform.3.bias": (48,),
        "timenet.0.weight": (64, 9),
        "time_poc": (4,),
        "pos_poc": (10,),
    }
    for k, shape in expect.items():
        assert k in sd, k
        assert tuple(sd[k].shape) == shape, (k, tuple(sd[k].shape))
    assert sum(v.numel() for k, v in sd.items() if "grid" in k and "aabb" not in k) == \
        16 * (3 * 64 * 64 + 3 * 64 * 150 + 3 * 128 * 128 + 3 * 128 * 150)


def _cpu_model(P=300, seed=0):
    hyper, opt = config.dnerf()
    torch.manual_seed(seed)
    g = GaussianModel(3, hyper, fused=False)
    rng = np.random.default_rng(seed)
    g._xyz = torch.nn.Parameter(torch.tensor(rng.normal(size=(P, 3)), dtype=torch.float32))
    g._features_dc = torch.nn.Parameter(torch.tensor(rng.normal(size=(P, 1, 3)), dtype=torch.float32))
    g._features_rest = torch.nn.Parameter(torch.tensor(rng.normal(size=(P, 15, 3)), dtype=torch.float32))
    g._scaling = torch.nn.Parameter(torch.tensor(rng.normal(-3, 0.5, size=(P, 3)), dtype=torch.float32))
    g._rotation = torch.nn.Parameter(torch.tensor(rng.normal(size=(P, 4)), dtype=torch.float32))
    g._opacity = torch.nn.Parameter(torch.tensor(rng.normal(size=(P, 1)), dtype=torch.float32))
    g.max_radii2D = torch.zeros(P)
    g._deformation_table = torch.ones(P, dtype=torch.bool)
    g.spatial_lr_scale = 1.0
    return g, opt


def test_ply_round_trip_and_layout(tmp_path):
    g, _ = _cpu_model()
    path = os.path.join(tmp_path, "point_cloud", "iteration_7", "point_cloud.ply")
    g.save_ply(path)
    head = open(path, "rb").read(4096).split(b"end_header\n")[0].decode()
    names = [l.split()[-1] for l in head.splitlines() if l.startswith("property")]
    assert names == ply.attribute_names(3, 45)
    assert "format binary_little_endian 1.0" in head and "element vertex 300" in head
    assert all(l.startswith("property float ") for l in head.splitlines() if l.startswith("property"))
    el = ply.read_ply(path)
    # f_rest is channel-major: f_rest_{c*15 + k} = features_rest[:, k, c]
    np.testing.assert_array_equal(el["f_rest_16"], g._features_rest.detach().numpy()[:, 1, 1])
    np.testing.assert_array_equal(el["nx"], 0)
    h, _ = _cpu_model(seed=1)
    h.load_ply(path, device="cpu")
    for k in ("_xyz", "_features_dc", "_features_rest", "_scaling", "_rotation", "_opacity"):
        torch.testing.assert_close(getattr(h, k), getattr(g, k), rtol=0, atol=0)
    assert h.active_sh_degree == 3


def test_ply_reader_handles_ascii_and_shuffled_suffixes(tmp_path):
    p = os.path.join(tmp_path, "a.ply")
    with open(p, "w") as f:
        f.write("ply\nformat ascii 1.0\ncomment x\nelement vertex 2\nproperty float x\nproperty double y\n"
                "property uchar z\nend_header\n1.5 2.5 3\n-1 0.25 7\n")
    el = ply.read_ply(p)
    np.testing.assert_allclose(el["x"], [1.5, -1.0])
    np.testing.assert_allclose(el["y"], [2.5, 0.25])
    np.testing.assert_array_equal(el["z"], [3, 7])


def test_deformation_checkpoint_round_trip(tmp_path):
    g, _ = _cpu_model()
    g._deformation_accum = torch.rand(300, 3)
    ply.save_model(str(tmp_path), 100, g)
    h, _ = _cpu_model(seed=2)
    ply.load_model(str(tmp_path), 100, h, device="cpu")
    for (ka, a), (kb, b) in zip(g._deformation.state_dict().items(), h._deformation.state_dict().items()):
        assert ka == kb
        torch.testing.assert_close(a, b, rtol=0, atol=0)
    torch.testing.assert_close(h._deformation_accum, g._deformation_accum)


def test_densify_prune_keep_optimizer_state_aligned():
    g, opt = _cpu_model(P=400)
    g.training_setup(opt)
    P0 = g.get_xyz.shape[0]
    # give every parameter a gradient and take one Adam step so the state exists
    loss = sum((p ** 2).sum() for grp in g.optimizer.param_groups for p in grp["params"])
    loss.backward()
    g.optimizer.step()
    g.xyz_gradient_accum = torch.rand(P0, 1) * 1e-3
    g.denom = torch.ones(P0, 1)
    g.percent_dense = 0.05
    torch.manual_seed(3)
    g.densify(5e-4, 0.005, 1.0, None)
    P1 = g.get_xyz.shape[0]
    assert P1 != P0
    for grp in g.optimizer.param_groups:
        if len(grp["params"]) > 1 or grp["name"] in ("deformation", "grid"):
            continue
        p = grp["params"][0]
        st = g.optimizer.state[p]
        assert p.shape[0] == P1 and st["exp_avg"].shape == p.shape and st["exp_avg_sq"].shape == p.shape
    assert g.max_radii2D.shape[0] == P1 and g.denom.shape[0] == P1 and g._deformation_table.shape[0] == P1
    g.prune(5e-4, 0.4, 1.0, None)
    P2 = g.get_xyz.shape[0]
    assert P2 < P1 and bool((g.get_opacity >= 0.4).all())
    g.reset_opacity()
    assert float(g.get_opacity.detach().max()) <= 0.01 + 1e-6
    st = g.optimizer.state[g._opacity]
    assert float(st["exp_avg"].abs().sum()) == 0.0


def _stepped_model(P=400, seed=0):
    """A CPU model whose optimizer has state (one Adam step), with statistics set and a mixed deformation table."""
    g, opt = _cpu_model(P=P, seed=seed)
    g.training_setup(opt)
    loss = sum((p ** 2).sum() for grp in g.optimizer.param_groups for p in grp["params"])
    loss.backward()
    g.optimizer.step()
    gen = torch.Generator().manual_seed(seed + 1)
    g.xyz_gradient_accum = torch.rand(P, 1, generator=gen) * 1e-3
    g.denom = torch.ones(P, 1)
    g.max_radii2D = torch.rand(P, generator=gen) * 10
    g._deformation_accum = torch.rand(P, 3, generator=gen)
    g._deformation_table = torch.rand(P, generator=gen) > 0.3
    g.percent_dense = 0.05
    return g


def _rows(g):
    names = {"xyz": "_xyz", "f_dc": "_features_dc", "f_rest": "_features_rest", "opacity": "_opacity",
             "scaling": "_scaling", "rotation": "_rotation"}
    out = {}
    for n, a in names.items():
        p = getattr(g, a)
        st = g.optimizer.state[p]
        out[n] = (p.detach().clone(), st["exp_avg"].clone(), st["exp_avg_sq"].clone(), st["step"])
    return out


def test_densify_rows_follow_reference_order():
    """densify (gaussian_model.py:501-506 = clone :443-457 then split :415-441) as one row plan: checked element
    by element against the row order the reference's two passes produce -- old rows not split (values and
    moments kept), then clones (copies, zero moments), then the two children of each split row copy after
    copy (copied attributes; scale log(s / 1.6); positions from the same normal draws); every statistic zero;
    the table follows the rows; each optimizer state keeps its step."""
    g = _stepped_model()
    before = _rows(g)
    P = before["xyz"][0].shape[0]
    grads = g.xyz_gradient_accum / g.denom
    smax = torch.exp(before["scaling"][0]).max(dim=1).values
    hot = grads[:, 0] >= 5e-4
    clone = torch.nonzero(hot & (smax <= 0.05)).flatten()
    split = torch.nonzero(hot & (smax > 0.05)).flatten()
    assert clone.numel() > 5 and split.numel() > 5
    kept = torch.nonzero(~torch.isin(torch.arange(P), split)).flatten()
    table0 = g._deformation_table.clone()
    torch.manual_seed(9)
    g.densify(5e-4, 0.005, 1.0, None)
    torch.manual_seed(9)
    s_split = torch.exp(before["scaling"][0][split]).repeat(2, 1)
    draws = torch.normal(mean=torch.zeros((s_split.size(0), 3)), std=s_split)
    K, C, S = kept.numel(), clone.numel(), split.numel()
    after = _rows(g)
    for n, (p0, m0, v0, step0) in before.items():
        p1, m1, v1, step1 = after[n]
        assert p1.shape[0] == K + C + 2 * S and step1 is step0
        assert torch.equal(p1[:K], p0[kept]) and torch.equal(m1[:K], m0[kept]) and torch.equal(v1[:K], v0[kept])
        assert torch.equal(p1[K:K + C], p0[clone])
        assert not m1[K:].any() and not v1[K:].any()
        if n not in ("xyz", "scaling"):
            assert torch.equal(p1[K + C:], p0[split].repeat(2, *([1] * (p0.dim() - 1))))
    sc = after["scaling"][0][K + C:]
    assert torch.equal(sc, torch.log(s_split / (0.8 * 2)))
    from gs4d_train.gaussians import build_rotation
    rot = build_rotation(before["rotation"][0][split]).repeat(2, 1, 1)
    xyz = torch.bmm(rot, draws.unsqueeze(-1)).squeeze(-1) + before["xyz"][0][split].repeat(2, 1)
    assert torch.equal(after["xyz"][0][K + C:], xyz)
    assert torch.equal(g._deformation_table, torch.cat([table0[kept], table0[clone], table0[split].repeat(2)]))
    for name, shape in (("xyz_gradient_accum", (K + C + 2 * S, 1)), ("denom", (K + C + 2 * S, 1)),
                        ("max_radii2D", (K + C + 2 * S,)), ("_deformation_accum", (K + C + 2 * S, 3))):
        t = getattr(g, name)
        assert t.shape == shape and not t.any(), name
    # prune: surviving rows keep values, moments and statistics, in order
    g.xyz_gradient_accum = torch.rand(K + C + 2 * S, 1)
    acc0, before = g.xyz_gradient_accum.clone(), _rows(g)
    live = (torch.sigmoid(before["opacity"][0]) >= 0.4).flatten()
    g.prune(5e-4, 0.4, 1.0, None)
    after = _rows(g)
    for n, (p0, m0, v0, step0) in before.items():
        p1, m1, v1, step1 = after[n]
        assert torch.equal(p1, p0[live]) and torch.equal(m1, m0[live]) and torch.equal(v1, v0[live]) and step1 is step0
    assert torch.equal(g.xyz_gradient_accum, acc0[live])


def test_expon_lr_schedule():
    f = get_expon_lr_func(1.6e-4, 1.6e-6, lr_delay_mult=0.01, max_steps=20000)
    assert math.isclose(f(0), 1.6e-4)
    assert math.isclose(f(20000), 1.6e-6, rel_tol=1e-9)
    assert math.isclose(f(10000), math.sqrt(1.6e-4 * 1.6e-6), rel_tol=1e-9)
    d = get_expon_lr_func(1.0, 1.0, lr_delay_steps=100, lr_delay_mult=0.1)
    assert math.isclose(d(0), 0.1) and math.isclose(d(100), 1.0)
    assert f(-1) == 0.0


def test_regularisers_run_and_are_zero_at_init():
    hyper, _ = config.dynerf()
    g = GaussianModel(3, hyper, fused=False)
    # time planes initialise to 1: second differences and |1 - plane| vanish on them
    assert float(g.compute_regulation(0.0, 1.0, 0.0)) == 0.0
    assert float(g.compute_regulation(1.0, 0.0, 0.0)) == 0.0
    assert float(g.compute_regulation(0.0, 0.0, 1.0)) > 0.0


def test_deform_heads_block_matches_separate_heads():
    """gs4d_train.deformation._DeformHeads (the 5 heads as one block: concatenated first layers, column
    slices for the second) against the reference's separate nn.Sequential heads
    (scene/deformation.py:73-78), float64 on CPU: outputs and every gradient to 1e-10."""
    import torch
    from gs4d_train.deformation import _DeformHeads
    torch.manual_seed(0)
    P, W, ns = 2500, 16, [3, 3, 4, 1, 48]   # P > 2 * 1024: exercises the split-K weight gradients
    hid = torch.randn(P, W, dtype=torch.float64, requires_grad=True)
    w1 = [torch.randn(W, W, dtype=torch.float64, requires_grad=True) for _ in ns]
    b1 = [torch.randn(W, dtype=torch.float64, requires_grad=True) for _ in ns]
    w2 = [torch.randn(n, W, dtype=torch.float64, requires_grad=True) for n in ns]
    b2 = [torch.randn(n, dtype=torch.float64, requires_grad=True) for n in ns]
    ups = [torch.randn(P, n, dtype=torch.float64) for n in ns]
    leaves = [hid] + w1 + b1 + w2 + b2
    outs = _DeformHeads.apply(False, hid, torch.cat(w1), torch.cat(b1), *[t for i in range(5) for t in (w2[i], b2[i])])
    ga = torch.autograd.grad(sum((o * u).sum() for o, u in zip(outs, ups)), leaves)
    F = torch.nn.functional
    ref = [F.linear(torch.relu(F.linear(torch.relu(hid), w1[i], b1[i])), w2[i], b2[i]) for i in range(5)]
    gb = torch.autograd.grad(sum((o * u).sum() for o, u in zip(ref, ups)), leaves)
    for a, b in zip(outs, ref):
        torch.testing.assert_close(a, b, rtol=1e-10, atol=1e-10)
    for a, b in zip(ga, gb):
        torch.testing.assert_close(a, b, rtol=1e-10, atol=1e-10)


def test_checkpoint_capture_restore_round_trip(tmp_path):
    """gaussian_model.py:66-106: capture() -> torch.save((capture(), iteration)) -> restore(); the
    optimizer state comes back bound to the restored parameters (train.py:49-57, 393-395)."""
    g, opt = _cpu_model(P=120)
    g.training_setup(opt)
    loss = sum((p ** 2).sum() for grp in g.optimizer.param_groups for p in grp["params"])
    loss.backward()
    g.optimizer.step()
    g.xyz_gradient_accum = torch.rand(120, 1)
    g.denom = torch.ones(120, 1) * 3
    g.active_sh_degree = 2
    path = os.path.join(tmp_path, "chkpnt_fine_7.pth")
    torch.save((g.capture(), 7), path)
    model_args, it = torch.load(path, weights_only=True)
    assert it == 7
    h, _ = _cpu_model(P=5, seed=4)
    h.restore(model_args, opt)
    assert h.active_sh_degree == 2 and h.spatial_lr_scale == g.spatial_lr_scale
    for k in ("_xyz", "_features_dc", "_features_rest", "_scaling", "_rotation", "_opacity", "xyz_gradient_accum",
              "denom", "max_radii2D"):
        torch.testing.assert_close(getattr(h, k), getattr(g, k), rtol=0, atol=0)
    for (ka, a), (kb, b) in zip(g._deformation.state_dict().items(), h._deformation.state_dict().items()):
        assert ka == kb and torch.equal(a, b)
    for pa, pb in zip([p for grp in g.optimizer.param_groups for p in grp["params"]],
                      [p for grp in h.optimizer.param_groups for p in grp["params"]]):
        sa, sb = g.optimizer.state[pa], h.optimizer.state[pb]
        if not pa.requires_grad:          # the HexPlane aabb buffer-parameter never steps
            assert len(sa) == len(sb) == 0
            continue
        assert torch.equal(sa["exp_avg"], sb["exp_avg"]) and torch.equal(sa["exp_avg_sq"], sb["exp_avg_sq"])
        assert float(sa["step"]) == float(sb["step"]) == 1.0


def test_fused_adam_state_dict_interchanges_with_torch_adam():
    """kernels.FusedAdam keeps torch.optim.Adam's state layout: a state dict saved by either loads
    into the other (the reference's checkpoints hold torch.optim.Adam state), with no kernel call."""
    from gs4d_train.kernels import FusedAdam
    torch.manual_seed(0)
    ps = [torch.nn.Parameter(torch.randn(5, 3)), torch.nn.Parameter(torch.randn(7))]
    adam = torch.optim.Adam([{"params": [ps[0]], "lr": 1e-2, "name": "a"},
                             {"params": [ps[1]], "lr": 1e-3, "name": "b"}], lr=0.0, eps=1e-15)
    (ps[0].sum() ** 2 + (ps[1] ** 3).sum()).backward()
    adam.step()
    sd = adam.state_dict()
    qs = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    fused = FusedAdam([{"params": [qs[0]], "lr": 0.5, "name": "a"}, {"params": [qs[1]], "lr": 0.5, "name": "b"}],
                      lr=0.0, eps=1e-15)
    fused.load_state_dict(sd)
    assert [g["lr"] for g in fused.param_groups] == [1e-2, 1e-3]
    assert [g["name"] for g in fused.param_groups] == ["a", "b"]
    for p, q in zip(ps, qs):
        a, b = adam.state[p], fused.state[q]
        assert torch.equal(a["exp_avg"], b["exp_avg"]) and torch.equal(a["exp_avg_sq"], b["exp_avg_sq"])
        assert float(b["step"]) == 1.0 and b["step"].dtype == torch.float32
    # and back: FusedAdam's state dict into a fresh torch Adam, which then steps normally
    back = torch.optim.Adam([{"params": [p], "lr": 0.0, "name": n} for p, n in zip(ps, "ab")], lr=0.0, eps=1e-15)
    back.load_state_dict(fused.state_dict())
    assert back.param_groups[0]["amsgrad"] is False and back.param_groups[1]["lr"] == 1e-3
    (ps[0].sum() ** 2 + (ps[1] ** 3).sum()).backward()
    back.step()
    assert float(back.state[ps[0]]["step"]) == 2.0


def test_fused_adam_host_step_counts(monkeypatch):
    """FusedAdam keeps its step counts on the host (no per-parameter tensor op / .item() per step): the scalars
    it passes to the launch follow torch's bias corrections for the right step, across the reference's
    optimizer-state surgery (the state dict moved to a replacement parameter, gaussian_model.py:316-388) and a
    state_dict() / load_state_dict() round trip, and the state's step tensors hold the count when read."""
    import math
    from gs4d_train import kernels as K
    calls = []
    monkeypatch.setattr(K, "_C", type("Fake", (), {"adam_step": staticmethod(lambda *a: calls.append(a))}))
    ps = [torch.nn.Parameter(torch.randn(4)) for _ in range(3)]
    for p in ps:
        p.grad = torch.randn(4)
    opt = K.FusedAdam([{"params": [p], "lr": 0.1} for p in ps], betas=(0.9, 0.99))
    for _ in range(5):
        opt.step()
    check = lambda n: (abs(calls[-1][4][0] + 0.1 / (1 - 0.9 ** n)) < 1e-12 and
                       abs(calls[-1][5][0] - math.sqrt(1 - 0.99 ** n)) < 1e-12)
    assert check(5)
    st = opt.state.pop(ps[0])  # surgery: the state follows a new tensor for the same group
    q = torch.nn.Parameter(torch.randn(6))
    q.grad = torch.randn(6)
    st["exp_avg"], st["exp_avg_sq"] = torch.zeros(6), torch.zeros(6)
    opt.param_groups[0]["params"][0] = q
    opt.state[q] = st
    opt.step()
    assert check(6)
    sd = opt.state_dict()
    assert [float(v["step"]) for v in sd["state"].values()] == [6.0, 6.0, 6.0]
    assert float(opt.state[q]["step"]) == 6.0
    opt2 = K.FusedAdam([{"params": [p], "lr": 0.1} for p in [q] + ps[1:]], betas=(0.9, 0.99))
    opt2.load_state_dict(sd)
    opt2.step()
    assert check(7)
    assert float(opt2.state_dict()["state"][0]["step"]) == 7.0
    # an in-place edit of a step tensor (a manual reset) is seen: the next step is step 1
    for st in opt2.state.values():
        st["step"].zero_()
    opt2.step()
    assert check(1)


def test_fused_adam_rejected_update_keeps_step_counts_and_frees_without_gc(monkeypatch):
    """A launch the extension rejects (a wrong dtype, size or device) leaves every step count as it was, so the
    bias corrections of the next accepted step are those of the right step; and an optimizer holds no reference
    to itself, so dropping the last reference frees it (and its moment buffers) without the cyclic GC."""
    import gc
    import weakref
    from gs4d_train import kernels as K
    calls = []

    def adam_step(*a):
        if any(p.numel() == 5 for p in a[0]):
            raise RuntimeError("adam_step: rejected")
        calls.append(a)
    monkeypatch.setattr(K, "_C", type("Fake", (), {"adam_step": staticmethod(adam_step)}))
    ps = [torch.nn.Parameter(torch.randn(4)) for _ in range(2)]
    for p in ps:
        p.grad = torch.randn(4)
    opt = K.FusedAdam([{"params": ps, "lr": 0.1}])
    opt.step()
    bad = torch.nn.Parameter(torch.randn(5))
    bad.grad = torch.randn(5)
    opt.param_groups[0]["params"].append(bad)
    with pytest.raises(RuntimeError):
        opt.step()
    assert [float(opt.state[p]["step"]) for p in ps] == [1.0, 1.0]
    opt.param_groups[0]["params"].pop()
    opt.step()
    assert [float(opt.state[p]["step"]) for p in ps] == [2.0, 2.0]
    assert abs(calls[-1][4][0] + 0.1 / (1 - 0.9 ** 2)) < 1e-12
    gc.disable()
    try:
        ref = weakref.ref(opt)
        del opt
        assert ref() is None, "FusedAdam must be freed by reference counting alone"
    finally:
        gc.enable()


def test_fused_adam_hooks_and_profiler_take_the_wrapped_step(monkeypatch):
    """FusedAdam's instance step skips torch's profiler/hook wrapper only while nothing is registered: step
    pre/post hooks (per optimizer and global) still fire, a profiler still sees the "Optimizer.step#..." range,
    an LR scheduler still wraps it, and parameters of groups with different betas go out in separate batches."""
    from gs4d_train import kernels as K
    calls = []
    monkeypatch.setattr(K, "_C", type("Fake", (), {"adam_step": staticmethod(lambda *a: calls.append(a))}))
    ps = [torch.nn.Parameter(torch.randn(3)) for _ in range(3)]
    for p in ps:
        p.grad = torch.randn(3)
    ps[2].grad = None  # no gradient: skipped, no state
    opt = K.FusedAdam([{"params": ps[:1], "lr": 0.1}, {"params": ps[1:], "lr": 0.2, "betas": (0.8, 0.9)}])
    seen = []
    h1 = opt.register_step_pre_hook(lambda o, a, k: seen.append("pre"))
    h2 = opt.register_step_post_hook(lambda o, a, k: seen.append("post"))
    from torch.optim.optimizer import register_optimizer_step_pre_hook
    h3 = register_optimizer_step_pre_hook(lambda o, a, k: seen.append("global"))
    opt.step()
    assert seen == ["global", "pre", "post"]
    for h in (h1, h2, h3):
        h.remove()
    opt.step()
    assert seen == ["global", "pre", "post"] and len(calls) == 4
    assert [len(c[0]) for c in calls[-2:]] == [1, 1] and {c[6] for c in calls[-2:]} == {0.9, 0.8}
    assert ps[2] not in opt.state and float(opt.state[ps[1]]["step"]) == 2.0
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU]) as prof:
        opt.step()
    assert any(e.name == "Optimizer.step#FusedAdam.step" for e in prof.events())
    sched = torch.optim.lr_scheduler.StepLR(opt, step_size=1, gamma=0.5)
    opt.step()
    sched.step()
    assert opt.param_groups[0]["lr"] == 0.05 and float(opt.state[ps[0]]["step"]) == 4.0


def test_ssim_restatement():
    """utils/loss_utils.py:26-66: window taps, ssim(x, x) = 1, and a direct float64 evaluation of the
    same formula (zero-padded 11x11 Gaussian window) on a small image."""
    from gs4d_train.losses import create_window, gaussian, ssim
    g = gaussian(11, 1.5)
    assert abs(float(g.sum()) - 1) < 1e-6 and int(g.argmax()) == 5
    w = create_window(11, 3)
    assert tuple(w.shape) == (3, 1, 11, 11)
    rng = np.random.default_rng(0)
    a = rng.uniform(size=(1, 3, 13, 17)).astype(np.float32)
    b = np.clip(a + rng.normal(0, 0.1, a.shape), 0, 1).astype(np.float32)
    assert abs(float(ssim(torch.tensor(a), torch.tensor(a))) - 1) < 1e-5
    k = w[0, 0].double().numpy()

    def filt(x):
        pad = np.pad(x, ((0, 0), (5, 5), (5, 5)))
        out = np.zeros_like(x)
        for i in range(x.shape[1]):
            for j in range(x.shape[2]):
                out[:, i, j] = (pad[:, i:i + 11, j:j + 11] * k).sum((1, 2))
        return out

    x, y = a[0].astype(np.float64), b[0].astype(np.float64)
    m1, m2 = filt(x), filt(y)
    s1, s2, s12 = filt(x * x) - m1 ** 2, filt(y * y) - m2 ** 2, filt(x * y) - m1 * m2
    C1, C2 = 0.01 ** 2, 0.03 ** 2
    ref = (((2 * m1 * m2 + C1) * (2 * s12 + C2)) / ((m1 ** 2 + m2 ** 2 + C1) * (s1 + s2 + C2))).mean()
    assert abs(float(ssim(torch.tensor(a), torch.tensor(b))) - ref) < 1e-5
    per_image = ssim(torch.tensor(a), torch.tensor(b), size_average=False)
    assert per_image.shape == (1,)


def _ref_hexplane_field(device="cpu"):
    """Our HexPlaneField (gs4d_train/deformation.py) holding the planes of tests/golden/ref_hexplane_vectors.npz,
    which the reference's own scene/hexplane.py produced (tests/golden/make_reference_vectors.py)."""
    import numpy as np
    import torch
    from gs4d_train.deformation import HexPlaneField
    v = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_hexplane_vectors.npz"))
    cfg = {"grid_dimensions": 2, "input_coordinate_dim": 4, "output_coordinate_dim": 4, "resolution": [8, 6, 10, 5]}
    field = HexPlaneField(1.6, cfg, [1, 2]).to(device)
    with torch.no_grad():
        for li, level in enumerate(field.grids):
            for pi, pl in enumerate(level):
                pl.copy_(torch.from_numpy(v[f"plane_{li}_{pi}"]))
    return field, v


def test_hexplane_field_matches_reference_module():
    """The restated HexPlane field (scene/hexplane.py restated in gs4d_train/deformation.py) against vectors
    made by RUNNING the reference's scene/hexplane.py: features, point gradients and plane gradients bitwise
    (the same grid_sample graph), and scene/regulation.py's compute_plane_smoothness per plane."""
    import numpy as np
    import torch
    from gs4d_train.gaussians import compute_plane_smoothness
    field, v = _ref_hexplane_field()
    pts = torch.from_numpy(v["pts"]).requires_grad_(True)
    feat = field(pts, torch.from_numpy(v["times"]))
    np.testing.assert_array_equal(feat.detach().numpy(), v["feat"])
    (feat * torch.from_numpy(v["G"])).sum().backward()
    np.testing.assert_array_equal(pts.grad.numpy(), v["gpts"])
    for li, level in enumerate(field.grids):
        for pi, pl in enumerate(level):
            np.testing.assert_array_equal(pl.grad.numpy(), v[f"gplane_{li}_{pi}"])
            assert float(compute_plane_smoothness(pl.detach())) == float(v[f"smooth_{li}_{pi}"])


def test_lr_schedule_matches_reference():
    """gs4d_train.gaussians.get_expon_lr_func against utils/general_utils.py:35-68 run by
    tests/golden/make_reference_vectors.py: the same float64 values at every step (warm-up, decay, clamp)."""
    import numpy as np
    from gs4d_train.gaussians import get_expon_lr_func
    v = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_lr_vectors.npz"))
    i = 0
    while f"lr_{i}" in v:
        a0, a1, dm, ms = v[f"args_{i}"]
        f = get_expon_lr_func(float(a0), float(a1), lr_delay_mult=float(dm), max_steps=int(ms))
        got = np.array([f(int(k)) for k in v["steps"]], np.float64)
        np.testing.assert_array_equal(got, v[f"lr_{i}"])
        i += 1
    assert i == 5


def test_splitk_chunk_rows_divides_p_or_falls_back():
    """deformation._chunk_rows: the largest multiple of 8 in [3/4, 2] x kChunk that divides P (no remainder GEMM),
    else kChunk (the remainder path)."""
    from gs4d_train.deformation import _LinearSplitK, _chunk_rows
    c0 = _LinearSplitK.kChunk
    for P in (100_000, 300_000, 1_000_000, 4096, 65_536, 100_003, 50_001, 7, 0):
        c = _chunk_rows(P)
        if c != c0 or P % c0 == 0:
            assert P % c == 0 and c % 8 == 0 and (3 * c0) // 4 <= c <= 2 * c0, (P, c)
            assert not any(P % d == 0 for d in range(c + 8, 2 * c0 + 1, 8) if d % 8 == 0), (P, c)
        else:
            assert not any(P % d == 0 for d in range((3 * c0) // 4, 2 * c0 + 1) if d % 8 == 0), (P, c)
    assert _chunk_rows(100_000) == 2000
