"""Convergence diagnostics (GPU): fused vs unfused training of the bouncing-balls scene over seeds and
lengths (tests/test_training_quality_gpu.py), to separate trajectory noise from a systematic gap."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "4dgaussians-fast-train_amd"), os.path.join(ROOT, "tests")]
import test_training_quality_gpu as T  # noqa: E402

ds = T.make_dataset()
kc, kf = int(sys.argv[1]), int(sys.argv[2])
for seed in range(int(sys.argv[3])):
    for fused in (True, False):
        i, t, tr, n = T._train(ds, fused, seed=seed, k_coarse=kc, k_fine=kf)
        print(f"seed {seed} fused={fused}: init {i:.2f} test {t:.2f} train {tr:.2f} n={n}", flush=True)
