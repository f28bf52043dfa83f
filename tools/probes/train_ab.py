"""fp32 vs bf16-MLP train step, alternated (diagnostic, GPU): bench.train_step_timing run ROUNDS times so
that host-speed drift on a shared box shows up in both legs alike."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "4dgaussians-fast-train_amd")]
import bench  # noqa: E402
from gs4d_train.synthetic import CONFIGS  # noqa: E402


def main(rounds=3, steps=30):
    P, W, H = CONFIGS["metric"]
    dev = torch.device("cuda:0")
    for r in range(rounds):
        res = bench.train_step_timing(P, W, H, dev, 1, 0, steps, 5, False, unfused=False)
        print(f"round {r}: fp32 {res['ms']:.3f} ms  bf16 {res['bf16_mlp']['ms']:.3f} ms  "
              f"loss {res['loss']:.5f} / {res['bf16_mlp']['loss']:.5f}", flush=True)


if __name__ == "__main__":
    main()
