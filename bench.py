"""Benchmark of the MI355X rasterizer hot path (BASELINE.json metric).

One "step" = one forward + backward of the differentiable rasterizer (K1-K9) over one view of a
synthetic scene of the metric configuration (100k Gaussians, SH degree 3, 1352x1014), inputs already
resident in HBM, plus the per-step loss all-reduce of the data-parallel harness when N > 1.  Each
rank renders its own view (independent views/timesteps shard across GPUs), so per-GPU
work is fixed as N grows ("weak" scaling).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config metric] [--no-cpu-baseline]
  multi-GPU: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Rank 0 prints ONE JSON line (see the contract in the task statement): value = whole-job
MGaussians/s = N * P * K / max-over-ranks(timed seconds) / 1e6.
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "4dgaussians-fast-train_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

# BASELINE.json's metric; value = the rasterizer fwd+bwd MGaussians/s, train_step.ms = the train-step ms
BASELINE_METRIC = "train-step ms + rasterizer fwd+bwd MGaussians/s @100k pts, 1352\u00d71014"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table: 8.0 TB/s spec
# VALU issue peak: 256 CUs x 4 SIMDs, one wave64 VALU instruction per 4 cycles per SIMD at 2.4 GHz
# (MI355X_MICROARCH.md: v_fma_f32 issue cost 4 cycles)
VALU_PEAK_GINST = 256 * 4 * 2.4 / 4


def algorithmic_bytes(P, L, W, H, K=16):
    """Compulsory HBM bytes.  Returns dict per stage and totals."""
    T = ((W + 15) // 16) * ((H + 15) // 16)
    Npix = W * H
    render_bwd = 40 * L + 20 * Npix + 8 * T + 44 * P      # K7: instance reads + pixel state + accumulators
    b_fwd = P * (147 + 12 * K) + 88 * L + 24 * Npix + 24 * T
    b_bwd = P * (327 + 24 * K) + 40 * L + 20 * Npix + 8 * T
    return dict(render_backward=render_bwd, render=44 * L + 8 * T + 24 * Npix, fwd=b_fwd, bwd=b_bwd,
                step=b_fwd + b_bwd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="metric")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-train-step", action="store_true", help="skip the full train-step timing")
    ap.add_argument("--train-steps", type=int, default=20)
    args = ap.parse_args()

    from gs4d_train.synthetic import CONFIGS, make_scene, make_upstream_grad
    import diff_gaussian_rasterization as dgr

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if dist:
        import torch.distributed as tdist
        tdist.init_process_group("nccl", device_id=dev)

    P, W, H = CONFIGS[args.config]
    # rank r renders its own view: same scene statistics, per-rank seed
    s = make_scene(P, W, H, seed=rank)
    t = lambda a: torch.tensor(np.asarray(a), device=dev)
    bg, vm, pm, cp = t(s["bg"]), t(s["viewmatrix"]), t(s["projmatrix"]), t(s["campos"])
    means3D, opac, scales, rots, shs = (t(s[k]) for k in ("means3D", "opacities", "scales", "rotations", "shs"))
    e = torch.empty(0, device=dev)
    C = dgr._C
    from gs4d_train import _C as TC
    one = torch.ones(1, device=dev)
    gt = t(np.random.default_rng(rank + 1).uniform(0, 1, (3, H, W)).astype(np.float32))

    def step():
        fwd = C.rasterize_gaussians(bg, means3D, e, opac, scales, rots, 1.0, e, vm, pm, s["tanfovx"], s["tanfovy"],
                                    H, W, shs, 3, cp, False, False)
        nr, color, depth, radii, gb, bb, ib = fwd
        # train.py:244 L1 loss and its gradient sign(color - gt) / N (fused kernels, csrc/train_tail.hip)
        loss, sgn = TC.l1_forward(color, gt)
        grad = TC.l1_backward(sgn, one)
        grads = C.rasterize_gaussians_backward(bg, means3D, radii, e, scales, rots, 1.0, e, vm, pm, s["tanfovx"],
                                               s["tanfovy"], grad, shs, 3, cp, gb, nr, bb, ib, False)
        if dist:
            tdist.all_reduce(loss)                    # the harness's loss all-reduce over RCCL
        return nr, loss, grads

    for _ in range(args.warmup):
        nr, loss, grads = step()
    torch.cuda.synchronize()
    if dist:
        tdist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        nr, loss, grads = step()
    torch.cuda.synchronize()
    if dist:
        tdist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dist:
        et = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        tdist.all_reduce(et, op=tdist.ReduceOp.MAX)
        elapsed = float(et.item())
    ms_per_step = elapsed / args.steps * 1e3
    value = world * P * args.steps / elapsed / 1e6

    # ---- per-kernel timing with hipEvents on the launch stream (same workload, K more steps) ----
    C.set_profiling(True)
    stage_ms = {}
    for _ in range(max(5, min(args.steps, 20))):
        nr, color, depth, radii, gb, bb, ib = C.rasterize_gaussians(bg, means3D, e, opac, scales, rots, 1.0, e, vm, pm,
                                                                    s["tanfovx"], s["tanfovy"], H, W, shs, 3, cp,
                                                                    False, False)
        for name, ms in C.last_timings():
            stage_ms.setdefault("fwd." + name, []).append(ms)
        grad = torch.sign(color - gt) / color.numel()
        C.rasterize_gaussians_backward(bg, means3D, radii, e, scales, rots, 1.0, e, vm, pm, s["tanfovx"], s["tanfovy"],
                                       grad, shs, 3, cp, gb, nr, bb, ib, False)
        for name, ms in C.last_timings():
            stage_ms.setdefault("bwd." + name, []).append(ms)
    C.set_profiling(False)
    stage_avg = {k: float(np.mean(v)) for k, v in stage_ms.items()}

    # ---- the full fine-stage train step (the metric's "train-step ms") ----
    train = None if args.no_train_step else train_step_timing(P, W, H, dev, world, rank, args.train_steps,
                                                              args.warmup, dist)

    if rank == 0:
        L = int(nr)
        ab = algorithmic_bytes(P, L, W, H)
        dom = max(stage_avg, key=stage_avg.get)
        dom_ms = stage_avg[dom]
        dom_bytes = ab["render_backward"] if dom == "bwd.render_backward" else (
            ab["render"] if dom == "fwd.render" else None)
        achieved = dom_bytes / (dom_ms * 1e-3) / 1e9 if dom_bytes else None
        def pmc(name):
            path = os.path.join(ROOT, "profiles", name)
            try:
                return json.load(open(path)).get(dom.split(".", 1)[1], None)
            except Exception:
                return None
        traffic = pmc("pmc_traffic.json")
        traffic_raw = pmc("pmc_traffic_raw.json")
        valu = pmc("pmc_valu.json")
        out = {
            "metric": BASELINE_METRIC,
            "value": round(value, 3), "unit": "MGaussians/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic (seeded, SURVEY §8d)",
            "config": {"workload": f"{args.config}: P={P} Gaussians, {W}x{H}, SH deg 3, 1 view/GPU/step, fwd+bwd",
                       "global_batch": world, "parallelism": f"views x{world} (independent views + RCCL loss all-reduce)"},
            "num_rendered": L,
            "stage_ms": {k: round(v, 4) for k, v in stage_avg.items()},
            "roofline": {"kernel": dom, "bound": "hbm", "achieved": round(achieved, 2) if achieved else None,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5) if achieved else None, "traffic": traffic,
                         "traffic_raw": traffic_raw,
                         "traffic_note": "PMC bytes per launch (profiles/r02_pmc.json): traffic = 2 x FETCH_SIZE + "
                                         "WRITE_SIZE (gfx950 wide-read correction), traffic_raw = FETCH_SIZE + "
                                         "WRITE_SIZE; the kernel's reads are mostly gathers, so the truth lies between",
                         "algorithmic_bytes": dom_bytes, "avg_ms": round(dom_ms, 4)},
            # the blend kernels are VALU-issue bound, not HBM bound: instruction rate vs the issue peak
            "valu_issue": {"kernel": dom, "insts_per_launch": valu,
                           "achieved_Ginst_s": round(valu / (dom_ms * 1e-3) / 1e9, 1) if valu else None,
                           "peak_Ginst_s": VALU_PEAK_GINST,
                           "frac": round(valu / (dom_ms * 1e-3) / 1e9 / VALU_PEAK_GINST, 4) if valu else None,
                           "source": "SQ_INSTS_VALU per launch, profiles/pmc_valu.json (rocprofv3 --pmc)"},
            "step_roofline": {"algorithmic_bytes": ab["step"],
                              "achieved_GBs": round(ab["step"] / (ms_per_step * 1e-3) / 1e9, 2),
                              "frac": round(ab["step"] / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)},
        }
        if train is not None:
            out["train_step"] = train
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(s, args.cpu_seconds)
        print(json.dumps(out), flush=True)
    if dist:
        tdist.destroy_process_group()


def train_step_timing(P, W, H, dev, world, rank, steps, warmup, dist, unfused=True):
    """One fine-stage training iteration of train.py (gs4d_train.train.train_step): HexPlane deformation
    + rasterizer fwd/bwd + L1 + HexPlane regularisers + backward + densification statistics + Adam, for
    one synthetic view per GPU (global batch = world; views shard across ranks, gradients all-reduced
    over RCCL).  Timed like the rasterizer steps: barrier + synchronize around K steps, max over ranks.
    With unfused=True (rank 0, single GPU) the reference's PyTorch tail (grid_sample HexPlane, torch
    L1 / Adam / statistics) is timed the same way for comparison."""
    import torch.distributed as tdist
    from gs4d_train import config
    from gs4d_train.gaussians import GaussianModel
    from gs4d_train.synthetic import make_point_cloud, make_training_views
    from gs4d_train.train import train_step

    def run(fused, n_steps, n_warm):
        hyper, opt = config.dynerf()
        torch.manual_seed(0)
        g = GaussianModel(3, hyper, fused=fused)
        pts, cols = make_point_cloud(P, seed=0)
        g.create_from_pcd(pts, cols, spatial_lr_scale=1.0, device=dev)
        g._deformation.deformation_net.grid.fused = fused
        g._deformation.deformation_net.fused_heads = fused
        g.training_setup(opt)
        g.active_sh_degree = 3
        views = make_training_views(world, W, H, seed=1, device=dev)
        bg = torch.ones(3, device=dev)
        it0 = 3001  # fine stage, densification statistics on, no densify/prune/reset iteration in range
        for i in range(n_warm):
            train_step(g, views, opt, hyper, it0 + i, bg, data_parallel=dist)
        torch.cuda.synchronize()
        if dist:
            tdist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(n_steps):
            loss = train_step(g, views, opt, hyper, it0 + n_warm + i, bg, data_parallel=dist)
        torch.cuda.synchronize()
        if dist:
            tdist.barrier()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        if dist:
            et = torch.tensor([el], device=dev, dtype=torch.float64)
            tdist.all_reduce(et, op=tdist.ReduceOp.MAX)
            el = float(et.item())
        return el / n_steps * 1e3, float(loss)

    ms, loss = run(True, steps, warmup)
    res = {"ms": round(ms, 3), "views_per_gpu": 1, "global_batch": world, "gaussians": P,
           "image": f"{W}x{H}", "loss": round(loss, 6),
           "config": "arguments/dynerf/default.py (HexPlane 16 x [64,64,64,150], multires [1,2], MLP width 128, "
                     "opacity+SH deform), fused libgs4d HexPlane field + regularisers / L1 / densification stats / Adam kernels, deformation heads as one GEMM block with their second-layer backward in HIP (gs4d_heads_backward)"}
    if unfused and world == 1:
        ums, _ = run(False, max(3, steps // 4), 2)
        res["reference_torch_tail_ms"] = round(ums, 3)
    return res


def cpu_baseline(s, budget_s):
    """The oracle (C restatement, OpenMP) on the host cores: same scene, full fwd+bwd per sample."""
    from oracle import oracle as O
    from gs4d_train.synthetic import make_upstream_grad
    try:
        cores = len(os.sched_getaffinity(0))
    except Exception:
        cores = os.cpu_count() or 1
    cores = min(cores, 16)   # the GPU box gives this job a 16-CPU share
    O.set_threads(cores)
    P, W, H = s["means3D"].shape[0], s["W"], s["H"]
    times = []
    t_start = time.perf_counter()
    while True:
        t0 = time.perf_counter()
        nr, color, depth, radii, st = O.rasterize_forward(
            s["bg"], s["means3D"], None, s["opacities"], s["scales"], s["rotations"], 1.0, None, s["viewmatrix"],
            s["projmatrix"], s["tanfovx"], s["tanfovy"], H, W, s["shs"], 3, s["campos"])
        g, _ = make_upstream_grad(color)
        O.rasterize_backward(st, s["bg"], s["means3D"], radii, None, s["scales"], s["rotations"], 1.0, None,
                             s["viewmatrix"], s["projmatrix"], s["tanfovx"], s["tanfovy"], g, s["shs"], 3, s["campos"])
        times.append(time.perf_counter() - t0)
        if time.perf_counter() - t_start > budget_s or len(times) >= 20:
            break
    med = float(np.median(times))
    return {"value": round(P / med / 1e6, 4), "unit": "MGaussians/s", "cores": cores, "kind": "port",
            "sample": f"{len(times)} full fwd+bwd of the same metric view (P={P}, {W}x{H}) by the OpenMP C oracle, "
                      f"median {med * 1e3:.1f} ms"}


if __name__ == "__main__":
    main()
