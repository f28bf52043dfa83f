"""simple_knn distCUDA2 timing (GPU) on the point clouds the tests and the train step use."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "4dgaussians-fast-train_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from simple_knn._C import distCUDA2  # noqa: E402

rng = np.random.default_rng(0)
clouds = {
    "uniform cube 100k (make_point_cloud)": rng.uniform(-1.2, 1.2, (100_000, 3)),
    "uniform cube 1M": rng.uniform(-1.2, 1.2, (1_000_000, 3)),
    "clustered 200k": np.concatenate([rng.normal(c, 0.05, (20_000, 3)) for c in rng.uniform(-1, 1, (10, 3))]),
    "sphere shells 3k": np.concatenate([rng.normal(size=(1000, 3)) for _ in range(3)]),
}
for name, pts in clouds.items():
    x = torch.tensor(pts.astype(np.float32), device="cuda")
    for _ in range(2):
        distCUDA2(x)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 5
    for _ in range(n):
        distCUDA2(x)
    torch.cuda.synchronize()
    print(f"{name}: {(time.perf_counter() - t0) / n * 1e3:.3f} ms", flush=True)
