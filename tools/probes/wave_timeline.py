"""Wave timeline of the blend kernels (GPU diagnostic, needs a libgs4d built with the temporary
s_memrealtime instrumentation that exports gs4d_debug_timeline): per wave start, first-blend and end
times (10 ns ticks), so the kernel's span splits into start latency, blend and tail.
python tools/probes/wave_timeline.py [synthetic|train_like]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "4dgaussians-fast-train_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import diff_gaussian_rasterization as dgr  # noqa: E402
from gs4d_train.synthetic import CONFIGS, make_scene, make_train_like_scene  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "synthetic"
P, W, H = CONFIGS["metric"]
dev = torch.device("cuda:0")
s = make_train_like_scene(P, W, H, seed=0) if scene == "train_like" else make_scene(P, W, H, seed=0)
d = bench.upload_scene(s, dev)
step = bench.make_step(d, dev, 0, dgr._C, None)
for _ in range(5):
    step()
torch.cuda.synchronize()
lib = ctypes.CDLL(os.path.join(ROOT, "4dgaussians-fast-train_amd/diff_gaussian_rasterization/libgs4d.so"))
lib.gs4d_debug_timeline_clear()
torch.cuda.synchronize()
step()
torch.cuda.synchronize()
for which, name in ((0, "forward"), (1, "backward")):
    buf = np.zeros(32768 * 4, np.uint64)
    assert lib.gs4d_debug_timeline(buf.ctypes.data_as(ctypes.c_void_p), which) == 0
    r = buf.reshape(-1, 4)
    r = r[r[:, 0] != 0]
    t0, t1, t2 = (r[:, i].astype(np.int64) for i in range(3))
    info = (r[:, 3] >> np.uint64(40)).astype(np.int64)
    hw = (r[:, 3] & np.uint64((1 << 40) - 1))
    base = t0.min()
    t0, t1, t2 = t0 - base, t1 - base, t2 - base
    span = t2.max()
    print(f"{name}: waves {len(r)} span {span / 100:.1f} us; start: median {np.median(t0) / 100:.1f} "
          f"p90 {np.percentile(t0, 90) / 100:.1f} max {t0.max() / 100:.1f} us; setup (t1-t0): median "
          f"{np.median(t1 - t0) / 100:.1f} p90 {np.percentile(t1 - t0, 90) / 100:.1f} us; duration median "
          f"{np.median(t2 - t0) / 100:.1f} p99 {np.percentile(t2 - t0, 99) / 100:.1f} max {(t2 - t0).max() / 100:.1f} us")
    # resident waves over time (20 bins)
    edges = np.linspace(0, span, 21)
    act = [int(((t0 < e1) & (t2 > e0)).sum()) for e0, e1 in zip(edges[:-1], edges[1:])]
    ends = np.histogram(t2, edges)[0]
    print("  resident per 5% bin:", act)
    print("  finishing per bin  :", list(ends))
    last = np.argsort(t2)[-8:]
    print("  last waves: end us", [round(t2[i] / 100, 1) for i in last], "start", [round(t0[i] / 100, 1) for i in last],
          "work", [int(info[i]) for i in last])
    # per SIMD (xcc, se, cu, simd) busy span vs kernel span
    hw_id = hw & np.uint64(0xFFFFFFFF)
    xcc = (hw >> np.uint64(32)) & np.uint64(0xF)
    simd = (hw_id >> np.uint64(4)) & np.uint64(3)
    cu = (hw_id >> np.uint64(8)) & np.uint64(0xF)
    se = (hw_id >> np.uint64(13)) & np.uint64(0x7)
    key = ((xcc * np.uint64(8) + se) * np.uint64(16) + cu) * np.uint64(4) + simd
    uk, inv = np.unique(key, return_inverse=True)
    last_end = np.zeros(len(uk), np.int64)
    np.maximum.at(last_end, inv, t2)
    print(f"  SIMDs used {len(uk)}; SIMD last-end: median {np.median(last_end) / 100:.1f} p10 "
          f"{np.percentile(last_end, 10) / 100:.1f} us of span {span / 100:.1f}")
