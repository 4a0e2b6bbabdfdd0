"""Fixture generator (run in the build container, CPU): the oracle's fp32 and fp64 trajectories
of configs[1] -- n = 10 workers, delay 50, --throttle, --model_file warm_start.pt (the warm start
of tests/golden/warm_n10.npz, made by make_warm_start_n10.py: a short fp64 oracle pre-training,
sha-pinned in meta.json), 52 epochs (through the first tick at t = 50 and the 9-worker epoch after
it), seed 1, pool seed 0.  Stores the per-epoch mean losses of both and JL sketches
(oracle.theta_sketch) of theta after epochs SKETCH_AT, so tests/test_gpu_configs.py can bound the
GPU's drift from fp64 by the CPU fp32 port's own drift without shipping parameter vectors.

The "fp64" oracle runs the forward/backward in fp64 and the rule() + Adam in fp32 (OracleSim).
Usage:  python tests/golden/make_trajectory.py   (about 5 minutes on 8 threads)
"""
import json
import os
import platform
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [REPO, os.path.join(REPO, "fl-distributed-delay_amd"), HERE]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import model_ref as MR  # noqa: E402
from oracle import oracle as O  # noqa: E402

N, DELAY, SEED, EPOCHS = 10, 50, 1, 52
SKETCH_AT = (10, 20, 30, 40, 51)


def warm_theta():
    """configs[1]'s warm start: tests/golden/warm_n10.npz dequantised (fp32, sha-pinned)."""
    from make_warm_start_n10 import dequantise
    f = np.load(os.path.join(HERE, "warm_n10.npz"))
    return dequantise(f["codes"], f["scales"])


def run(dtype):
    pool = O.make_pool(0)
    sim = MR.OracleSim(N, delay=DELAY, throttle=True, seed=SEED, pool=pool, dtype=dtype,
                       theta0=warm_theta())
    losses, sk = [], []
    for t in range(EPOCHS):
        losses.append(sim.epoch())
        if t in SKETCH_AT:
            sk.append(O.theta_sketch(sim.theta))
        print(dtype, t, losses[-1], flush=True)
    return np.asarray(losses, np.float64), np.stack(sk)


def main():
    t0 = time.time()
    l32, s32 = run(torch.float32)
    l64, s64 = run(torch.float64)
    np.savez(os.path.join(HERE, "traj_n10.npz"), loss32=l32, loss64=l64, sketch32=s32,
             sketch64=s64, sketch_at=np.asarray(SKETCH_AT), config=np.asarray([N, DELAY, SEED, EPOCHS]))
    meta_path = os.path.join(HERE, "meta.json")
    meta = json.load(open(meta_path))
    meta["traj_n10"] = dict(threads=torch.get_num_threads(), torch=torch.__version__,
                            cpu=platform.processor() or platform.machine(),
                            seconds=round(time.time() - t0, 1),
                            config="n=10 delay=50 throttle seed=1 pool seed 0, 52 epochs, "
                                   "warm start warm_n10 (sha in warm_n10)")
    json.dump(meta, open(meta_path, "w"), indent=1)


if __name__ == "__main__":
    main()
