"""Benchmark of the MI355X rasterizer hot path (BASELINE.json metric).

One "step" = one forward + backward of the differentiable rasterizer (K1-K9) over one view of a
synthetic scene of the metric configuration (100k Gaussians, SH degree 3, 1352x1014), inputs already
resident in HBM, plus the per-step loss all-reduce of the data-parallel harness when N > 1.  Each
rank renders its own view (independent views/timesteps shard across GPUs), so per-GPU
work is fixed as N grows ("weak" scaling).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config metric] [--no-cpu-baseline]

With --gpus N > 1 and no WORLD_SIZE in the environment, bench.py launches its own N ranks
(`torch.distributed.run`, 127.0.0.1) as a child process before anything touches the GPU, and exits
with the child's status; under a launcher (WORLD_SIZE set) it refuses to run unless WORLD_SIZE == N,
so a multi-GPU run can never silently measure one rank.  `--dry-run` goes through the same launcher
and rendezvous over gloo on the CPU, with a stand-in step instead of the HIP calls (the CPU test of the
launcher path, tests/test_bench_launcher.py).

Rank 0 prints ONE JSON line (see the contract in the task statement): value = whole-job
MGaussians/s = N * P * K / max-over-ranks(timed seconds) / 1e6.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "4dgaussians-fast-train_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

# BASELINE.json's metric; value = the rasterizer fwd+bwd MGaussians/s, train_step.ms = the train-step ms
BASELINE_METRIC = "train-step ms + rasterizer fwd+bwd MGaussians/s @100k pts, 1352×1014"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table: 8.0 TB/s spec
KERNEL_REPEATS = 10    # back-to-back launches per event bracket for the blend kernels' own durations


def algorithmic_bytes(P, L, W, H, K=16):
    """Compulsory HBM bytes.  Returns dict per stage and totals."""
    T = ((W + 15) // 16) * ((H + 15) // 16)
    Npix = W * H
    render_bwd = 40 * L + 20 * Npix + 8 * T + 44 * P      # K7: instance reads + pixel state + accumulators
    b_fwd = P * (147 + 12 * K) + 88 * L + 24 * Npix + 24 * T
    b_bwd = P * (327 + 24 * K) + 40 * L + 20 * Npix + 8 * T
    return dict(render_backward=render_bwd, render=44 * L + 8 * T + 24 * Npix, fwd=b_fwd, bwd=b_bwd,
                step=b_fwd + b_bwd)


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="metric")
    ap.add_argument("--scene", default="synthetic", choices=["synthetic", "train_like"],
                    help="synthetic: the SURVEY §8d scene (the metric); train_like: make_train_like_scene "
                         "(profiling of the second workload)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-train-step", action="store_true", help="skip the full train-step timing")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the autograd-wrapper and training-like-scene timings")
    ap.add_argument("--train-steps", type=int, default=20)
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher/rendezvous check on the CPU (gloo, no HIP call); not a measurement")
    return ap.parse_args(argv)


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args, argv):
    """Start N ranks of this script under torch.distributed.run (a child process: nothing in this
    process has touched the GPU) and return the child's exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__), *argv]
    return subprocess.call(cmd, cwd=ROOT)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    if args.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args, argv))
    world = int(env_world or "1")
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: refusing to measure a different "
                 f"number of ranks than asked for")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        return dry_run(args, world, rank)

    from gs4d_train.synthetic import CONFIGS, make_scene
    import diff_gaussian_rasterization as dgr
    import torch.distributed as tdist

    dist = world > 1
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if dist:
        tdist.init_process_group("nccl", device_id=dev)
        assert tdist.get_world_size() == args.gpus, (tdist.get_world_size(), args.gpus)

    P, W, H = CONFIGS[args.config]
    # rank r renders its own view: same scene statistics, per-rank seed
    if args.scene == "train_like":
        from gs4d_train.synthetic import make_train_like_scene
        s = make_train_like_scene(P, W, H, seed=rank)
    else:
        s = make_scene(P, W, H, seed=rank)
    scene = upload_scene(s, dev)
    step = make_step(scene, dev, rank, dgr._C, dist)
    elapsed, nr = timed_steps(step, args.steps, args.warmup, dist)
    my_ms = elapsed / args.steps * 1e3
    per_rank = gather_per_rank([float(nr), my_ms], world, dev, dist)
    elapsed = max(r[1] for r in per_rank) * args.steps / 1e3   # max over ranks
    ms_per_step = elapsed / args.steps * 1e3
    value = world * P * args.steps / elapsed / 1e6

    stage_avg = stage_timings(scene, dgr._C, args.steps)
    kernel_avg = stage_timings(scene, dgr._C, args.steps, repeats=KERNEL_REPEATS)

    # ---- the full fine-stage train step (the metric's "train-step ms"), before the extras: run after their
    # large scenes, the host-heavier bf16 leg measured 1.62-2.29 ms instead of 1.50-1.52 (fp32 unaffected)
    train = None if args.no_train_step else train_step_timing(P, W, H, dev, world, rank, args.train_steps,
                                                              args.warmup, dist)

    extras = {}
    if not args.no_extras:
        extras["forward_only"] = forward_timing(scene, dgr._C, args.steps, args.warmup)
        extras["autograd_wrapper"] = autograd_timing(scene, dgr, args.steps, args.warmup, P)
        extras["train_like_scene"] = train_like_timing(P, W, H, dev, args.steps, args.warmup, dgr._C, rank)
        extras["configs"] = config_timings(dev, args.steps, args.warmup, dgr._C)

    if rank == 0:
        L = int(nr)
        ab = algorithmic_bytes(P, L, W, H)
        dom = max(stage_avg, key=stage_avg.get)
        # the kernel's own duration: back-to-back launches between two events (agrees with rocprofv3's
        # kernel-trace average; the per-stage brackets of stage_ms add their gaps)
        dom_ms = kernel_avg.get(dom, stage_avg[dom])
        dom_bytes = ab["render_backward"] if dom == "bwd.render_backward" else (
            ab["render"] if dom == "fwd.render" else None)
        achieved = dom_bytes / (dom_ms * 1e-3) / 1e9 if dom_bytes else None
        prof = load_profile_summary(dom.split(".", 1)[1])
        out = {
            "metric": BASELINE_METRIC,
            "value": round(value, 3), "unit": "MGaussians/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic (seeded, SURVEY §8d)",
            "config": {"workload": f"{args.config}: P={P} Gaussians, {W}x{H}, SH deg 3, 1 view/GPU/step, fwd+bwd",
                       "global_batch": world, "parallelism": f"views x{world} (independent views + RCCL loss all-reduce)"},
            "num_rendered": L,
            "per_rank": [{"rank": i, "num_rendered": int(r[0]), "ms_per_step": round(r[1], 4)}
                         for i, r in enumerate(per_rank)],
            "stage_ms": {k: round(v, 4) for k, v in stage_avg.items()},
            "roofline": {"kernel": dom, "bound": "hbm", "achieved": round(achieved, 2) if achieved else None,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5) if achieved else None,
                         "traffic": prof.get("traffic"), "traffic_raw": prof.get("traffic_raw"),
                         "traffic_note": "PMC bytes per launch (profiles/pmc_traffic.json): traffic = 2 x FETCH_SIZE + "
                                         "WRITE_SIZE (gfx950 wide-read correction), traffic_raw = FETCH_SIZE + "
                                         "WRITE_SIZE; the kernel's reads are mostly gathers, so the truth lies between",
                         "algorithmic_bytes": dom_bytes, "avg_ms": round(dom_ms, 4),
                         "avg_ms_note": f"hipEvent average over {KERNEL_REPEATS} back-to-back launches on the "
                                        f"launch stream; stage_ms (one launch per event bracket) reads "
                                        f"{stage_avg[dom]:.4f}"},
            "kernel_ms": {k: round(v, 4) for k, v in kernel_avg.items()},
            "step_roofline": {"algorithmic_bytes": ab["step"],
                              "achieved_GBs": round(ab["step"] / (ms_per_step * 1e-3) / 1e9, 2),
                              "frac": round(ab["step"] / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)},
        }
        if prof.get("valu") is not None:
            # the blend kernels are VALU-issue bound, not HBM bound: measured VALU busy fraction
            out["valu_utilisation"] = prof["valu"]
        out.update(extras)
        if train is not None:
            out["train_step"] = train
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(s, args.cpu_seconds)
        print(json.dumps(out), flush=True)
    if dist:
        tdist.destroy_process_group()


def upload_scene(s, dev):
    t = lambda a: torch.tensor(np.asarray(a), device=dev)
    d = {k: t(s[k]) for k in ("bg", "viewmatrix", "projmatrix", "campos", "means3D", "opacities", "scales",
                              "rotations", "shs")}
    d.update(W=s["W"], H=s["H"], tanfovx=s["tanfovx"], tanfovy=s["tanfovy"], e=torch.empty(0, device=dev))
    return d


def _fwd(C, d):
    return C.rasterize_gaussians(d["bg"], d["means3D"], d["e"], d["opacities"], d["scales"], d["rotations"], 1.0,
                                 d["e"], d["viewmatrix"], d["projmatrix"], d["tanfovx"], d["tanfovy"], d["H"], d["W"],
                                 d["shs"], 3, d["campos"], False, False)


def _bwd(C, d, radii, grad, gb, nr, bb, ib):
    return C.rasterize_gaussians_backward(d["bg"], d["means3D"], radii, d["e"], d["scales"], d["rotations"], 1.0,
                                          d["e"], d["viewmatrix"], d["projmatrix"], d["tanfovx"], d["tanfovy"], grad,
                                          d["shs"], 3, d["campos"], gb, nr, bb, ib, False)


def make_step(d, dev, seed, C, dist):
    from gs4d_train import _C as TC
    gt = torch.tensor(np.random.default_rng(seed + 1).uniform(0, 1, (3, d["H"], d["W"])).astype(np.float32),
                      device=dev)

    def step():
        nr, color, depth, radii, gb, bb, ib = _fwd(C, d)
        # train.py:244 L1 loss and its gradient sign(color - gt) / N for loss.backward()'s dloss = 1: value and
        # gradient in one pass (gs4d_l1_loss_grad, csrc/train_tail.hip; bitwise the two-pass form)
        loss, grad = TC.l1_loss_grad(color, gt, 1.0)
        _bwd(C, d, radii, grad, gb, nr, bb, ib)
        if dist:
            import torch.distributed as tdist
            tdist.all_reduce(loss)                    # the harness's loss all-reduce over RCCL
        return nr
    return step


def timed_steps(step, steps, warmup, dist, sync=True):
    """W untimed steps, then K steps bracketed by barrier + synchronize on both sides."""
    import torch.distributed as tdist
    cuda = sync and torch.cuda.is_available()
    nr = 0
    for _ in range(warmup):
        nr = step()
    if cuda:
        torch.cuda.synchronize()
    if dist:
        tdist.barrier()
    if cuda:
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        nr = step()
    if cuda:
        torch.cuda.synchronize()
    if dist:
        tdist.barrier()
    if cuda:
        torch.cuda.synchronize()
    return time.perf_counter() - t0, nr


def gather_per_rank(row, world, dev, dist):
    """[[num_rendered, ms_per_step] of every rank] (one all-reduce of a world x 2 table)."""
    if not dist:
        return [row]
    import torch.distributed as tdist
    tab = torch.zeros(world, len(row), dtype=torch.float64, device=dev)
    tab[tdist.get_rank()] = torch.tensor(row, dtype=torch.float64)
    tdist.all_reduce(tab)
    return tab.cpu().tolist()


def stage_timings(d, C, steps, repeats=1):
    """Per-kernel hipEvent timings on the launch stream (same workload, a few more steps).  With
    repeats > 1 the two blend kernels run `repeats` times back to back inside their stage and report the
    per-launch average (gs4d_set_profiling(level)): a kernel duration without the event brackets' gaps,
    the quantity rocprofv3's kernel trace reports (the roofline's avg_ms)."""
    C.set_profiling(repeats if repeats > 1 else 1)
    stage_ms = {}
    gt = torch.tensor(np.random.default_rng(1).uniform(0, 1, (3, d["H"], d["W"])).astype(np.float32),
                      device=d["bg"].device)
    for _ in range(max(5, min(steps, 20))):
        nr, color, depth, radii, gb, bb, ib = _fwd(C, d)
        for name, ms in C.last_timings():
            stage_ms.setdefault("fwd." + name, []).append(ms)
        grad = torch.sign(color - gt) / color.numel()
        _bwd(C, d, radii, grad, gb, nr, bb, ib)
        for name, ms in C.last_timings():
            stage_ms.setdefault("bwd." + name, []).append(ms)
    C.set_profiling(0)
    out = {k: float(np.mean(v)) for k, v in stage_ms.items()}
    if repeats > 1:   # only the blend kernels are repeated; the other entries include the repeats' gaps
        out = {k: v for k, v in out.items() if k in ("fwd.render", "bwd.render_backward")}
    return out


def forward_timing(d, C, steps, warmup):
    """Forward only (the inference path render.py times: rasterizer forward of one view), ms and FPS."""
    el, nr = timed_steps(lambda: _fwd(C, d)[0], steps, warmup, False)
    ms = el / steps * 1e3
    return {"ms": round(ms, 4), "fps": round(1e3 / ms, 1), "num_rendered": int(nr)}


def config_timings(dev, steps, warmup, C, names=("c2_800", "c4_per_view", "c5_broom"), fwd_only=("c2_800",)):
    """BASELINE configs C2 (100k, 800x800), C4 (300k, 1352x1014: one view of the 8-GPU run) and C5 (1M,
    960x536): the headline step (fwd + L1 + bwd) per config, MGaussians/s and L; forward-only at C2."""
    from gs4d_train.synthetic import CONFIGS, make_scene
    res = {}
    for name in names:
        P, W, H = CONFIGS[name]
        d = upload_scene(make_scene(P, W, H, seed=0), dev)
        el, nr = timed_steps(make_step(d, dev, 0, C, False), steps, warmup, False)
        ms = el / steps * 1e3
        res[name] = {"P": P, "image": f"{W}x{H}", "ms_per_step": round(ms, 4),
                     "MGaussians_s": round(P / (ms * 1e-3) / 1e6, 3), "num_rendered": int(nr)}
        if name in fwd_only:
            res[name]["forward_only"] = forward_timing(d, C, steps, warmup)
        del d
        torch.cuda.empty_cache()
    return res


def autograd_timing(d, dgr, steps, warmup, P):
    """The same fwd+bwd through the Python API (GaussianRasterizer + torch.autograd), as
    gaussian_renderer/__init__.py drives it (report it with and without the wrapper)."""
    settings = dgr.GaussianRasterizationSettings(
        image_height=d["H"], image_width=d["W"], tanfovx=d["tanfovx"], tanfovy=d["tanfovy"], bg=d["bg"],
        scale_modifier=1.0, viewmatrix=d["viewmatrix"], projmatrix=d["projmatrix"], sh_degree=3,
        campos=d["campos"], prefiltered=False, debug=False)
    rast = dgr.GaussianRasterizer(settings)
    leaves = {k: d[k].clone().requires_grad_(True) for k in ("means3D", "shs", "opacities", "scales", "rotations")}
    means2D = torch.zeros_like(leaves["means3D"], requires_grad=True)
    gt = torch.tensor(np.random.default_rng(1).uniform(0, 1, (3, d["H"], d["W"])).astype(np.float32),
                      device=d["bg"].device)

    def step():
        for v in list(leaves.values()) + [means2D]:
            v.grad = None
        color, radii, depth = rast(means3D=leaves["means3D"], means2D=means2D, shs=leaves["shs"],
                                   opacities=leaves["opacities"], scales=leaves["scales"],
                                   rotations=leaves["rotations"])
        loss = torch.abs(color - gt).mean()          # train.py:244 l1_loss
        loss.backward()
        return 0
    el, _ = timed_steps(step, steps, warmup, False)
    ms = el / steps * 1e3
    return {"ms_per_step": round(ms, 4), "MGaussians_s": round(P / (ms * 1e-3) / 1e6, 3),
            "note": "GaussianRasterizer + torch L1 + loss.backward() (torch's own L1 kernels, not the fused "
                    "ones of the headline step)"}


def train_like_timing(P, W, H, dev, steps, warmup, C, seed):
    """A second named workload: the metric-size rasterizer fwd+bwd on the scene a training run starts
    from (gs4d_train.synthetic.make_train_like_scene: k-NN scales, larger splats, ~1,200 instances per
    touched tile), where the blend kernels weigh more than in the metric scene."""
    from gs4d_train.synthetic import make_train_like_scene
    s = make_train_like_scene(P, W, H, seed=0)
    d = upload_scene(s, dev)
    step = make_step(d, dev, seed, C, False)
    el, nr = timed_steps(step, steps, warmup, False)
    ms = el / steps * 1e3
    stages = stage_timings(d, C, steps)
    T = ((W + 15) // 16) * ((H + 15) // 16)
    return {"workload": f"train_like: P={P}, {W}x{H}, k-NN-initialised point cloud (create_from_pcd), view 0",
            "ms_per_step": round(ms, 4), "MGaussians_s": round(P / (ms * 1e-3) / 1e6, 3),
            "num_rendered": int(nr), "tiles": T,
            "stage_ms": {k: round(v, 4) for k, v in sorted(stages.items(), key=lambda kv: -kv[1])[:6]}}


def load_profile_summary(kernel):
    """The rocprofv3 PMC evidence for the dominant kernel, committed under profiles/ by
    tools/profile.sh + tools/pmc_summary.py (bytes per launch; VALU busy from SQ counters)."""
    out = {}
    for key, name in (("traffic", "pmc_traffic.json"), ("traffic_raw", "pmc_traffic_raw.json"),
                      ("valu", "pmc_valu.json")):
        try:
            with open(os.path.join(ROOT, "profiles", name)) as f:
                out[key] = json.load(f).get(kernel)
        except (OSError, ValueError):
            out[key] = None
    return out


def dry_run(args, world, rank):
    """The launcher path without the GPU: gloo rendezvous, a CPU stand-in step, the same per-rank
    gather and max-over-ranks timing, and a JSON line marked as not a measurement."""
    import torch.distributed as tdist
    dist = world > 1
    if dist:
        tdist.init_process_group("gloo")
        assert tdist.get_world_size() == args.gpus, (tdist.get_world_size(), args.gpus)
    x = torch.randn(256, 256, generator=torch.Generator().manual_seed(rank))

    def step():
        y = x @ x
        if dist:
            v = y.sum().reshape(1)
            tdist.all_reduce(v)
        return 1000 + rank
    el, nr = timed_steps(step, args.steps, args.warmup, dist, sync=False)
    per_rank = gather_per_rank([float(nr), el / args.steps * 1e3], world, torch.device("cpu"), dist)
    if rank == 0:
        ms = max(r[1] for r in per_rank)
        print(json.dumps({"metric": BASELINE_METRIC, "value": None, "unit": "MGaussians/s", "n_gpus": world,
                          "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 4),
                          "dry_run": True, "per_rank": [{"rank": i, "num_rendered": int(r[0]),
                                                         "ms_per_step": round(r[1], 4)}
                                                        for i, r in enumerate(per_rank)]}), flush=True)
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

    def run(fused, n_steps, n_warm, mlp_dtype="fp32"):
        hyper, opt = config.dynerf()
        hyper.mlp_dtype = mlp_dtype
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
        state = {"i": it0}

        def one():
            loss = train_step(g, views, opt, hyper, state["i"], bg, data_parallel=dist)
            state["i"] += 1
            return loss
        el, loss = timed_steps(one, n_steps, n_warm, dist)
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
    # BASELINE C3's "bf16/fp32": the same step with the deformation heads on bf16 operands (opt-in,
    # deformation.py _DeformHeadsBF16: the heads block forward on the bf16 MFMA, the second-layer backward on
    # bf16 a / da, the two W x 5W GEMMs of the backward as hand-written bf16-MFMA passes (dW1 with fp32 sums,
    # dh); the rasterizer, feature_out, parameters, gradients and the heads' outputs stay fp32)
    bms, bloss = run(True, steps, warmup, mlp_dtype="bf16")
    res["bf16_mlp"] = {"ms": round(bms, 3), "loss": round(bloss, 6),
                       "config": "as above, hyper.mlp_dtype = 'bf16' (gs4d_heads_block_forward_bf16, "
                                 "gs4d_heads_backward_bf16, gs4d_mlp_dw_bf16 / gs4d_mlp_dx_bf16)"}
    if unfused and world == 1:
        ums, _ = run(False, max(3, steps // 4), 2)
        res["reference_torch_tail_ms"] = round(ums, 3)
    return res


def _cpu_sample(s, threads, budget_s, max_samples):
    from oracle import oracle as O
    from gs4d_train.synthetic import make_upstream_grad
    O.set_threads(threads)
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
        if time.perf_counter() - t_start > budget_s or len(times) >= max_samples:
            break
    return float(np.median(times)), len(times)


def cpu_baseline(s, budget_s):
    """The oracle (C restatement, OpenMP) on the host cores: same scene, full fwd+bwd per sample, with
    the box's CPU share (<= 16 threads) and with one thread."""
    try:
        affinity = len(os.sched_getaffinity(0))
    except Exception:
        affinity = os.cpu_count() or 1
    # threads: OMP_NUM_THREADS when set (the GPU box sets it to this job's CPU share), else the affinity
    env_threads = os.environ.get("OMP_NUM_THREADS", "")
    cores = int(env_threads) if env_threads.isdigit() and int(env_threads) > 0 else affinity
    cores = min(cores, affinity)
    P, W, H = s["means3D"].shape[0], s["W"], s["H"]
    med, n = _cpu_sample(s, cores, budget_s, 20)
    med1, n1 = _cpu_sample(s, 1, 0.0, 1)     # one sample: a full view takes seconds on one thread
    return {"value": round(P / med / 1e6, 4), "unit": "MGaussians/s", "cores": cores, "kind": "port",
            "affinity_cpus": affinity, "threads_used": cores,
            "threads_source": "OMP_NUM_THREADS" if env_threads.isdigit() else "sched_getaffinity",
            "sample": f"{n} full fwd+bwd of the same metric view (P={P}, {W}x{H}) by the OpenMP C oracle, "
                      f"median {med * 1e3:.1f} ms",
            "one_thread": {"value": round(P / med1 / 1e6, 5), "cores": 1,
                           "sample": f"{n1} full fwd+bwd of the same view, {med1 * 1e3:.0f} ms"}}


if __name__ == "__main__":
    main()
