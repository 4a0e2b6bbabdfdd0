"""GPU parity at the sizes of BASELINE.json's configs (the reference loop main.py:126-188).

  * configs[2] / the bench line's shape: n = 1024, delay 50, --throttle, through the first tick
    (t = 50) and the 1023-worker epoch after it: staleness trace bit-exact against the reference's
    own loop (tests/golden/schedule.npz, traced by tests/golden/make_golden.py), finite losses,
    and S_t of the 1023-worker epoch independent of the chunking (128- vs 32-worker launches);
  * configs[1]'s shape: n = 10, delay 50, --throttle, 52 epochs against the CPU oracle's fp32 and
    fp64 trajectories (tests/golden/traj_n10.npz): Adam turns last-bit gradient differences into
    O(lr) parameter moves, so the GPU's distance from fp64 is bounded by a stated
    multiple of the CPU fp32 port's own distance from fp64, in loss and in parameters (JL sketch);
  * configs[4]'s launch size for vgg11: a 128-worker chunk (16,384 samples) against 32-worker
    chunks.
"""
import numpy as np
import pytest
import torch

from conftest import has_gpu

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not has_gpu(), reason="needs an MI355X")]

DEV = "cuda:0"


@pytest.fixture(scope="module")
def pool():
    from oracle import oracle as O
    return O.make_pool(0)


def _rel_l2(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def test_n1024_d50_through_first_tick(pool, golden):
    from flsim.engine import PN1_SHAPES, PN1_SIZES
    from flsim.sim import FLSimulation
    key = "n1024_d50_thr1_e600"
    g = golden.schedule
    E = 52
    ref_comp = np.unpackbits(g[key + "_computes"], axis=1)[:E, :1024]
    ref_c = g[key + "_c_t"][:E]
    ref_stale = g[key + "_stale"][:E]
    a = FLSimulation(1024, delay=50, throttle=True, device=DEV, pool=pool)
    for t in range(E - 1):
        a.epoch(sync_loss=False)
    ck = a.checkpoint()
    b = FLSimulation(1024, delay=50, throttle=True, device=DEV, pool=pool, chunk_workers=32,
                     keep_S=True)
    b.restore(ck)
    a.keep_S = True                             # epoch 51: S_t into comm[:P] on both
    a.epoch(sync_loss=False)
    b.epoch(sync_loss=False)
    for t, plan in enumerate(a.trace):
        assert np.array_equal(plan.computes, ref_comp[t]), t
        assert plan.c_t == ref_c[t], t
        assert [s for (_, s) in plan.stale] == ([int(ref_stale[t])] if ref_stale[t] >= 0 else []), t
    assert int(a.trace[50].computes.sum()) == 513 and int(a.trace[51].computes.sum()) == 1023
    losses = a.losses()
    assert len(losses) == E and np.all(np.isfinite(losses))
    # the 1023 worker losses of epoch 51 do not depend on the chunking; S_t only through the
    # split-K slab order
    wa = a.comm[a.Ppad:a.Ppad + 1023].cpu().numpy()
    wb = b.comm[b.Ppad:b.Ppad + 1023].cpu().numpy()
    assert np.array_equal(wa.view(np.uint32), wb.view(np.uint32))
    sa = a.comm[:a.P].cpu().numpy().astype(np.float64)
    sb = b.comm[:b.P].cpu().numpy().astype(np.float64)
    off = 0
    for (name, _), n in zip(PN1_SHAPES, PN1_SIZES):
        r = _rel_l2(sb[off:off + n], sa[off:off + n])
        assert r <= 1e-5, (name, r)
        off += n
    assert b.losses()[-1] == losses[-1]


# Stated bound of the configs[1] trajectory test: the GPU's distance from the fp64 oracle is at
# most DRIFT_C times the CPU fp32 port's own distance from it (+ a floor for the first epochs,
# where both are at the fp32 noise level), in the running-max loss gap and in parameters.
DRIFT_C = 4.0


def test_n10_d50_trajectory_drift_vs_oracle(pool, golden):
    from flsim.sim import FLSimulation
    from oracle import oracle as O
    f = golden.traj_n10
    n, d, seed, E = (int(x) for x in f["config"])
    sim = FLSimulation(n, delay=d, throttle=True, seed=seed, device=DEV, pool=pool)
    l64, l32 = f["loss64"], f["loss32"]
    at = [int(x) for x in f["sketch_at"]]
    lg, sk = [], []
    for t in range(E):
        lg.append(sim.epoch())
        if t in at:
            sk.append(O.theta_sketch(sim.theta[:sim.P].cpu().numpy()))
    lg = np.asarray(lg)
    assert abs(lg[0] - l32[0]) <= 1e-4
    gap_gpu = np.maximum.accumulate(np.abs(lg - l64))
    gap_cpu = np.maximum.accumulate(np.abs(l32 - l64))
    d_gpu = [O.sketch_distance(s, s64) for s, s64 in zip(sk, f["sketch64"])]
    d_cpu = [O.sketch_distance(s32, s64) for s32, s64 in zip(f["sketch32"], f["sketch64"])]
    print("loss gap gpu/cpu:", [(int(t), float(a), float(b)) for t, a, b in
                                zip(range(0, E, 5), gap_gpu[::5], gap_cpu[::5])])
    print("param drift gpu/cpu:", list(zip(at, d_gpu, d_cpu)))
    assert np.all(gap_gpu <= DRIFT_C * gap_cpu + 2e-4), (gap_gpu, gap_cpu)
    for t, dg, dc in zip(at, d_gpu, d_cpu):
        assert dg <= DRIFT_C * dc + 1e-6, (t, dg, dc)


def test_vgg11_max_chunk_matches_small_chunks(pool):
    """configs[4]'s launch size: one 128-worker vgg11 launch (16,384 samples) against four
    32-worker launches from the same theta and batches."""
    from flsim.engine import VGG11_SHAPES, VGG11_SIZES
    from flsim.sim import FLSimulation
    n = 129
    kw = dict(delay=50, throttle=False, device=DEV, pool=pool, model="vgg11", keep_S=True)
    a = FLSimulation(n, chunk_workers=32, **kw)
    b = FLSimulation(n, chunk_workers=128, **kw)
    a.epoch()
    b.epoch()
    for x, y in ((b.theta, a.theta), (b.m, a.m), (b.v, a.v)):
        x.copy_(y)
    la, lb = a.epoch(), b.epoch()
    assert int(a.trace[-1].computes.sum()) == 128 and b.chunks(0, 128) == [(0, 128)]
    assert la == lb
    wa = a.comm[a.Ppad:a.Ppad + 128].cpu().numpy()
    wb = b.comm[b.Ppad:b.Ppad + 128].cpu().numpy()
    assert np.array_equal(wa.view(np.uint32), wb.view(np.uint32))
    sa = a.comm[:a.P].cpu().numpy().astype(np.float64)
    sb = b.comm[:b.P].cpu().numpy().astype(np.float64)
    off = 0
    for (name, _), size in zip(VGG11_SHAPES, VGG11_SIZES):
        r = _rel_l2(sb[off:off + size], sa[off:off + size])
        assert r <= 1e-5, (name, r)
        off += size
