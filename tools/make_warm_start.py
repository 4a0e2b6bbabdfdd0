"""Synthesise configs[1]'s `warm_start.pt` (the reference's blob is not in the repo):
a seeded pre-training run of the same simulation on the GPU (n = 10, d = 50, --throttle) on the
same data as the runs it warm-starts (the seed-0 pool and test split), with seed 1 for the k-draws,
sample indices and dropout masks so the pre-training batches differ from theirs, saved as a plain
models.py state_dict with the reference's keys -- the file main.py:98-100 / `--model_file` loads.

    python tools/make_warm_start.py --epochs 500 --out gpurun_out/warm_start.pt
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "fl-distributed-delay_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=500)
    ap.add_argument("--n_workers", type=int, default=10)
    ap.add_argument("--delay", type=int, default=50)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--model", default="PerformantNet1")
    ap.add_argument("--out", default="gpurun_out/warm_start.pt")
    args = ap.parse_args()
    from flsim.data import make_pool, make_test_pool
    from flsim.sim import FLSimulation
    sim = FLSimulation(args.n_workers, delay=args.delay, throttle=True, seed=args.seed,
                       device="cuda:0", model=args.model, chunk_workers=8,
                       pool=make_pool(0), test_pool=make_test_pool(0))
    for t in range(args.epochs):
        loss = sim.epoch()
        if t % 50 == 0 or t == args.epochs - 1:
            print(f"epoch {t} Avg. Loss {loss:.5f}", flush=True)
    acc, per = sim.evaluate()
    print(f"test accuracy {acc:.2f} %  per class {[round(a, 1) for a in per]}", flush=True)
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    torch.save(sim.model_state_dict(), args.out)
    print("wrote", args.out)


if __name__ == "__main__":
    main()
