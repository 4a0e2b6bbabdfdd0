"""Fixture generator (build container, CPU): configs[1]'s warm start (`--model_file
warm_start.pt`, main.py:49-50,98-100).  The reference's blob is not available, so the
warm start is synthesised by a short pre-training with the CPU oracle: the same loop (n = 10,
delay 50, --throttle) in fp64 from the seed-2 default init, on the seed-0 pool, seed 2 for the
k-draws / samples / dropout (the warm-started runs use seed 1: different batches), PRE_EPOCHS
epochs.  The result is stored as per-tensor int8 codes with an fp32 scale (theta = code * scale,
exact in fp32): 5.6 MB instead of 22 MB, and every test that loads it (GPU or oracle) starts from
bit-identical parameters.  The sha256 of the dequantised fp32 vector is pinned in
tests/golden/meta.json and checked by tests/test_oracle_golden.py.

Usage:  python tests/golden/make_warm_start_n10.py      (about 2 minutes on 8 threads)
"""
import hashlib
import json
import os
import platform
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [REPO, os.path.join(REPO, "fl-distributed-delay_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import model_ref as MR  # noqa: E402
from oracle import oracle as O  # noqa: E402

N, DELAY, SEED, PRE_EPOCHS = 10, 50, 2, 30


def quantise(theta):
    """Per parameter tensor: int8 codes q and an fp32 scale s = max|theta| / 127 (exact powers
    are not needed: the fixture's value IS q * s in fp32)."""
    codes, scales = [], []
    off = 0
    for _, shp in MR.param_shapes():
        n = int(np.prod(shp))
        a = theta[off:off + n].astype(np.float64)
        s = np.float32(max(np.abs(a).max(), 1e-30) / 127.0)
        codes.append(np.clip(np.rint(a / np.float64(s)), -127, 127).astype(np.int8))
        scales.append(s)
        off += n
    return np.concatenate(codes), np.asarray(scales, np.float32)


def dequantise(codes, scales):
    out = np.empty(codes.shape[0], np.float32)
    off = 0
    for (_, shp), s in zip(MR.param_shapes(), scales):
        n = int(np.prod(shp))
        out[off:off + n] = codes[off:off + n].astype(np.float32) * np.float32(s)
        off += n
    return out


def sha(theta):
    return hashlib.sha256(np.ascontiguousarray(theta, np.float32).tobytes()).hexdigest()


def main():
    t0 = time.time()
    pool = O.make_pool(0)
    sim = MR.OracleSim(N, delay=DELAY, throttle=True, seed=SEED, pool=pool, dtype=torch.float64,
                       theta0=MR.init_params(SEED))
    for t in range(PRE_EPOCHS):
        print("pre-training epoch", t, sim.epoch(), flush=True)
    codes, scales = quantise(sim.theta)
    theta = dequantise(codes, scales)
    np.savez_compressed(os.path.join(HERE, "warm_n10.npz"), codes=codes, scales=scales)
    meta_path = os.path.join(HERE, "meta.json")
    meta = json.load(open(meta_path))
    meta["warm_n10"] = dict(sha256=sha(theta), threads=torch.get_num_threads(),
                            torch=torch.__version__, cpu=platform.processor() or platform.machine(),
                            seconds=round(time.time() - t0, 1),
                            config=f"oracle fp64 pre-training n={N} delay={DELAY} throttle "
                                   f"seed={SEED} pool seed 0, {PRE_EPOCHS} epochs, int8 per-tensor")
    json.dump(meta, open(meta_path, "w"), indent=1)
    print("sha256", meta["warm_n10"]["sha256"])


if __name__ == "__main__":
    main()
