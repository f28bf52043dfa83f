"""The short-horizon training pair of tests/test_training_quality_gpu.py over many seeds, with the unfused (reference
torch formulation) arm run twice per seed: measures the unfused arm's own run-to-run spread (torch's grid_sample
backward sums with float atomics) and the fused-vs-unfused gaps, to set the test's bars from measurements.
Prints one JSON line per seed and a summary.  Usage: python tools/probes/conv_spread.py [n_seeds] [first_seed]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path[:0] = [os.path.join(ROOT, "4dgaussians-fast-train_amd"), ROOT, os.path.join(ROOT, "tests")]
from test_training_quality_gpu import _train, make_dataset  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 12
s0 = int(sys.argv[2]) if len(sys.argv) > 2 else 0
ds = make_dataset()
rows = []
for seed in range(s0, s0 + n):
    f = _train(ds, True, seed=seed, k_coarse=200, k_fine=200, densify=False)[1]
    u1 = _train(ds, False, seed=seed, k_coarse=200, k_fine=200, densify=False)[1]
    u2 = _train(ds, False, seed=seed, k_coarse=200, k_fine=200, densify=False)[1]
    rows.append((seed, f, u1, u2))
    print(json.dumps({"seed": seed, "fused": round(f, 4), "unfused": round(u1, 4), "unfused_rerun": round(u2, 4)}),
          flush=True)
a = np.array([r[1:] for r in rows])
print(json.dumps({"n": n, "self_spread_sd": float(np.std(a[:, 1] - a[:, 2], ddof=1)),
                  "gap_sd": float(np.std(a[:, 0] - a[:, 1], ddof=1)), "gap_mean": float(np.mean(a[:, 0] - a[:, 1])),
                  "max_abs_gap": float(np.abs(a[:, 0] - a[:, 1]).max()),
                  "max_abs_self": float(np.abs(a[:, 1] - a[:, 2]).max())}), flush=True)
