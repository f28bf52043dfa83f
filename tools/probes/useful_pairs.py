"""Useful-pair fraction of the blend kernels (CPU, from the oracle's forward state).

For every tile the reverse walk (render.hip render_backward_kernel) evaluates, per emitted instance
below the tile's largest n_contrib, the 128 pixels of each half tile the splat reaches.  A pair
(pixel, splat) is USEFUL when the reference's backward does work for it (backward.cu:486-497):
the pixel is inside the image, the splat is at or before the pixel's last contributor, and
alpha = min(0.99, o G) >= 1/255 with power <= 0.  The forward (render_forward_kernel) evaluates, per
half tile, the splats reaching that half until every pixel of the half terminated.

The script reports evaluated vs useful pairs for both kernels at the current work unit (16x8 half
tiles) and what finer reach units (8x8, 8x4, 4x4 sub-tiles) would evaluate, so the choice between a
finer work unit and fewer instructions per pair rests on a measurement.

  python tools/probes/useful_pairs.py [metric|train_like|c2_800|...] [--json out.json]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "4dgaussians-fast-train_amd")]
from gs4d_train.synthetic import CONFIGS, make_scene, make_train_like_scene  # noqa: E402
from oracle import oracle as O  # noqa: E402

UNITS = {"half16x8": (16, 8), "quarter8x8": (8, 8), "8x4": (8, 4), "4x4": (4, 4), "16x4": (16, 4)}


def analyse(s):
    W, H = s["W"], s["H"]
    nr, color, depth, radii, st = O.rasterize_forward(
        s["bg"], s["means3D"], None, s["opacities"], s["scales"], s["rotations"], 1.0, None, s["viewmatrix"],
        s["projmatrix"], s["tanfovx"], s["tanfovy"], H, W, s["shs"], 3, s["campos"])
    ex = st.export()
    gx, gy = (W + 15) // 16, (H + 15) // 16
    xy, co, plist, ranges, nc = ex["means2D"], ex["conic_opacity"], ex["point_list"], ex["ranges"], ex["n_contrib"]
    ly, lx = np.mgrid[0:16, 0:16]
    lx = lx.reshape(-1).astype(np.float32)
    ly = ly.reshape(-1).astype(np.float32)
    tot = dict(L=int(nr), emitted=0, bwd_eval=0, fwd_eval=0, useful=0, alpha_pass=0, bwd_walked_inst=0,
               unit_eval={k: 0 for k in UNITS}, unit_eval_walk={k: 0 for k in UNITS})
    ncpad = np.zeros((gy * 16, gx * 16), np.int64)
    ncpad[:H, :W] = nc
    for t in range(gx * gy):
        rs, re = int(ranges[t, 0]), int(ranges[t, 1])
        if re <= rs:
            continue
        tx, ty = t % gx, t // gx
        g = plist[rs:re]
        px = tx * 16 + lx
        py = ty * 16 + ly
        inside = (px < W) & (py < H)
        dx = xy[g, 0][:, None] - px[None, :]
        dy = xy[g, 1][:, None] - py[None, :]
        c = co[g]
        power = -0.5 * (c[:, 0:1] * dx * dx + c[:, 2:3] * dy * dy) - c[:, 1:2] * dx * dy
        alpha = np.minimum(0.99, c[:, 3:4] * np.exp(power))
        ok = (alpha >= 1.0 / 255.0) & (power <= 0) & inside[None, :]          # (n, 256)
        pos = np.arange(1, re - rs + 1)[:, None]
        last = ncpad[ty * 16:(ty + 1) * 16, tx * 16:(tx + 1) * 16].reshape(-1)
        useful = ok & (pos <= last[None, :])
        # reach per half (exact; the emission's closed form adds a 0.1 % margin)
        okr = ok.reshape(-1, 2, 8, 16)
        half = okr.any(axis=(2, 3))                                           # (n, 2)
        # full halves: every inside pixel of the half passes the alpha test (the walk could skip it)
        insr = inside.reshape(2, 8, 16)
        full = np.array([(okr[:, h] | ~insr[h][None]).all(axis=(1, 2)) for h in range(2)]).T & half
        emit = half.any(1)
        n_em = int(emit.sum())
        tot["emitted"] += n_em
        tot["alpha_pass"] += int(ok.sum())
        tot["useful"] += int(useful.sum())
        # backward: emitted instances at emitted positions < max over pixels of the emitted-list n_contrib
        epos = np.cumsum(emit)                                                # 1-based emitted position
        lmax = int(last.max())
        walk_lim = int(epos[lmax - 1]) if lmax > 0 else 0
        walked = emit & (epos <= walk_lim)
        tot["bwd_walked_inst"] += int(walked.sum())
        tot["bwd_eval"] += 128 * int(half[walked].sum())
        tot["bwd_half_steps"] = tot.get("bwd_half_steps", 0) + int(half[walked].sum())
        tot["bwd_full_half_steps"] = tot.get("bwd_full_half_steps", 0) + int(full[walked].sum())
        # the same walk with each half skipped past the largest n_contrib of ITS pixels
        for h in range(2):
            lh = int(last.reshape(2, 128)[h].max())
            lim_h = int(epos[lh - 1]) if lh > 0 else 0
            tot["bwd_half_steps_perhalf"] = tot.get("bwd_half_steps_perhalf", 0) + int(
                half[emit & (epos <= lim_h), h].sum())
        # forward: per half, splats reaching it until every live pixel of the half terminated (or the end)
        for h in range(2):
            lh = last.reshape(2, 128)[h]
            ins = inside.reshape(2, 128)[h]
            # a pixel that never terminated walks the whole list; terminated pixels stop at n_contrib + 1
            term = (final_T_tile(ex, tx, ty, W, H).reshape(2, 128)[h])
            stop = np.where(term, lh + 1, re - rs)
            lim = int(stop[ins].max()) if ins.any() else 0
            tot["fwd_eval"] += 128 * int(half[:lim, h].sum())
        for k, (ux, uy) in UNITS.items():
            sub = ok.reshape(-1, 16 // uy, uy, 16 // ux, ux).any(axis=(2, 4))  # (n, units_y, units_x)
            tot["unit_eval"][k] += ux * uy * int(sub.sum())
            tot["unit_eval_walk"][k] += ux * uy * int(sub[walked].sum())
    return tot


def final_T_tile(ex, tx, ty, W, H):
    """Pixels of the tile that terminated (final T fell to its last value before 1e-4 ended the walk):
    the forward's early exit; approximated by final_T < 1e-3 (T only stops near 1e-4)."""
    ft = np.ones((16, 16), np.float32)
    y1, x1 = min(16, H - ty * 16), min(16, W - tx * 16)
    ft[:y1, :x1] = ex["final_T"][ty * 16:ty * 16 + y1, tx * 16:tx * 16 + x1]
    return (ft < 1e-3).reshape(-1)


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("-") else "metric"
    out = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    O.set_threads(os.cpu_count() or 1)
    if cfg == "train_like":
        P, W, H = CONFIGS["metric"]
        s = make_train_like_scene(P, W, H, seed=0)
    else:
        P, W, H = CONFIGS[cfg]
        s = make_scene(P, W, H, seed=0)
    r = analyse(s)
    r["scene"] = cfg
    r["useful_frac_bwd"] = r["useful"] / max(r["bwd_eval"], 1)
    r["alpha_frac_bwd"] = r["alpha_pass"] / max(r["bwd_eval"], 1)
    r["full_half_frac"] = r.get("bwd_full_half_steps", 0) / max(r.get("bwd_half_steps", 1), 1)
    r["useful_per_inst"] = r["useful"] / max(r["bwd_walked_inst"], 1)
    r["bwd_eval_per_inst"] = r["bwd_eval"] / max(r["bwd_walked_inst"], 1)
    r["unit_frac_of_half"] = {k: v / max(r["unit_eval_walk"]["half16x8"], 1) for k, v in r["unit_eval_walk"].items()}
    print(json.dumps(r, indent=1))
    if out:
        with open(out, "w") as f:
            json.dump(r, f, indent=1)


if __name__ == "__main__":
    main()
