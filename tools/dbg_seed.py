"""Debug helper: n = 10, d = 50, --throttle loss curves of the GPU engine for a few (seed, chunk)
settings on the seed-0 pool, and the CPU oracle's curve for the first epochs of one seed."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "fl-distributed-delay_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from flsim.data import make_pool
    from flsim.sim import FLSimulation
    from oracle import model_ref as MR
    pool = make_pool(0)
    E = int(os.environ.get("EPOCHS", "120"))
    for seed, chunk in [(0, 32), (0, 8), (1, 32), (1, 8), (2, 32)]:
        sim = FLSimulation(10, delay=50, throttle=True, seed=seed, device="cuda:0",
                           chunk_workers=chunk, pool=pool)
        ls = [sim.epoch() for _ in range(E)]
        print(f"seed {seed} chunk {chunk}:", " ".join(f"{x:.3f}" for x in ls[::10]),
              "min", round(min(ls), 4), flush=True)
    EO = int(os.environ.get("ORACLE_EPOCHS", "30"))
    torch.set_num_threads(16)
    for seed in (1,):
        osim = MR.OracleSim(10, delay=50, throttle=True, seed=seed, pool=pool)
        gsim = FLSimulation(10, delay=50, throttle=True, seed=seed, device="cuda:0",
                            chunk_workers=32, pool=pool)
        t0 = time.time()
        for t in range(EO):
            lo, lg = osim.epoch(), gsim.epoch()
            print(f"oracle seed {seed} epoch {t}: cpu {lo:.5f} gpu {lg:.5f}", flush=True)
        print("oracle time", round(time.time() - t0, 1))


if __name__ == "__main__":
    main()
