"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle on the same seeded inputs.

Tolerances (calibrated on the reference's own fp32-vs-fp64 spread):
  * aggregation + Adam kernel: bit-exact with the oracle (same correctly rounded sqrt);
  * one worker-step gradient: per-tensor rel-L2 vs fp64 <= 5e-3 and
    ||g_gpu - g64|| <= 2 ||g_cpu32 - g64|| + 1e-6 ||g64||;
  * losses: |dloss| <= 1e-4 on the first step, <= 1e-3 over the first epochs;
  * staleness trace: bit-exact.
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


def _sizes():
    from flsim.engine import PN1_SIZES
    return PN1_SIZES


def _oracle_agg_adam(S, c, stale, p, m, v, step, semantics_zero=False):
    from oracle import oracle as O
    g = np.empty_like(S)
    off = 0
    for n in _sizes():
        ents = [S[off:off + n]] * c + [s[off:off + n] for s in stale]
        g[off:off + n] = O.cascade_mean(ents)
        off += n
    O.adam_step(p, m, v, g, step)
    return p, m, v


@pytest.mark.parametrize("c,ns", [(1, 0), (3, 1), (9, 0), (512, 1), (1023, 1), (40, 2)])
def test_aggregate_adam_bit_exact(c, ns):
    from flsim.engine import PN1Engine
    eng = PN1Engine(DEV, chunk_workers=1)
    P = eng.P
    rs = np.random.RandomState(c * 7 + ns)
    S = (rs.standard_normal(P) * 1e-2).astype(np.float32)
    stale = [(rs.standard_normal(P) * 1e-2).astype(np.float32) for _ in range(ns)]
    p = rs.standard_normal(P).astype(np.float32)
    m = (rs.standard_normal(P) * 1e-3).astype(np.float32)
    v = (rs.rand(P) * 1e-5).astype(np.float32)
    step = 3
    dS = torch.from_numpy(S).to(DEV)
    dst = [torch.from_numpy(s).to(DEV) for s in stale]
    dp, dm, dv = (torch.from_numpy(a.copy()).to(DEV) for a in (p, m, v))
    eng.aggregate_adam(dS, c, dst, dp, dm, dv, step)
    torch.cuda.synchronize()
    _oracle_agg_adam(S, c, stale, p, m, v, step)
    for name, a, b in (("p", dp, p), ("m", dm, m), ("v", dv, v)):
        got = a.cpu().numpy()
        nbad = int((got.view(np.uint32) != b.view(np.uint32)).sum())
        assert nbad == 0, (name, nbad)


def test_aggregate_adam_torch1_zero_stale():
    from flsim.engine import PN1Engine
    eng = PN1Engine(DEV, chunk_workers=1)
    P = eng.P
    rs = np.random.RandomState(5)
    S = (rs.standard_normal(P) * 1e-2).astype(np.float32)
    p = rs.standard_normal(P).astype(np.float32)
    m = np.zeros(P, np.float32)
    v = np.zeros(P, np.float32)
    dS = torch.from_numpy(S).to(DEV)
    dp, dm, dv = (torch.from_numpy(a.copy()).to(DEV) for a in (p, m, v))
    eng.aggregate_adam(dS, 9, [None], dp, dm, dv, 1)
    _oracle_agg_adam(S, 9, [np.zeros(P, np.float32)], p, m, v, 1)
    assert np.array_equal(dp.cpu().numpy().view(np.uint32), p.view(np.uint32))


def _rel_l2(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def _grad_checks(g_gpu, g32, g64):
    off = 0
    from flsim.engine import PN1_SHAPES
    for (name, _), n in zip(PN1_SHAPES, _sizes()):
        a, b32, b64 = g_gpu[off:off + n], g32[off:off + n], g64[off:off + n]
        off += n
        r = _rel_l2(a, b64)
        e_gpu = np.linalg.norm(a - b64)
        e_cpu = np.linalg.norm(b32 - b64)
        assert r <= 5e-3, (name, r)
        assert e_gpu <= 2 * e_cpu + 1e-6 * np.linalg.norm(b64) + 1e-12, (name, e_gpu, e_cpu)


@pytest.mark.parametrize("dropout", [False, True])
def test_single_worker_step_gradient(pool, dropout):
    import torch as T
    from flsim.data import DevicePool
    from flsim.engine import PN1Engine, worker_table
    from oracle import model_ref as MR
    sim = MR.OracleSim(4, delay=2, pool=pool, dropout=dropout)
    items = [(0, 0, 0)]
    g32, l32 = sim.grad_of(sim.theta, items)
    g64, l64 = sim.grad_of(sim.theta, items, dtype=T.float64)
    eng = PN1Engine(DEV, chunk_workers=1)
    dpool = DevicePool(DEV, 0, pool)
    theta = T.from_numpy(sim.theta.copy()).to(DEV)
    eng.begin_epoch(theta)
    loss = T.zeros(1, device=DEV)
    eng.run_chunk(theta, dpool, worker_table(items, DEV), 1, 4, 0, dropout, loss)
    S = T.zeros(eng.P, device=DEV)
    eng.end_epoch(S)
    T.cuda.synchronize()
    assert abs(float(loss.item()) - l64[0]) <= 1e-4
    _grad_checks(S.cpu().numpy().astype(np.float64), g32.astype(np.float64), g64)


def test_chunk_of_workers_sums_gradients(pool):
    """A chunk of 3 worker-steps (different (t,i,k), incl. the {1,9} dataset) == the sum of the
    per-worker gradients (agents.py:35 accumulation) -- oracle runs them sequentially."""
    import torch as T
    from flsim.data import DevicePool
    from flsim.engine import PN1Engine, worker_table
    from oracle import model_ref as MR
    sim = MR.OracleSim(4, delay=2, pool=pool)
    items = [(2, 0, 1), (2, 1, 3), (2, 3, 0)]
    g32, l32 = sim.grad_of(sim.theta, items)
    g64, l64 = sim.grad_of(sim.theta, items, dtype=T.float64)
    eng = PN1Engine(DEV, chunk_workers=2)
    dpool = DevicePool(DEV, 0, pool)
    theta = T.from_numpy(sim.theta.copy()).to(DEV)
    eng.begin_epoch(theta)
    loss = T.zeros(3, device=DEV)
    eng.run_chunk(theta, dpool, worker_table(items[:2], DEV), 2, 4, 0, True, loss[:2])
    eng.run_chunk(theta, dpool, worker_table(items[2:], DEV), 1, 4, 0, True, loss[2:])
    S = T.zeros(eng.P, device=DEV)
    eng.end_epoch(S)
    T.cuda.synchronize()
    np.testing.assert_allclose(loss.cpu().numpy(), l64, atol=1e-4)
    _grad_checks(S.cpu().numpy().astype(np.float64), g32.astype(np.float64), g64)


@pytest.mark.parametrize("thr", [False, True])
def test_simulation_matches_oracle_trajectory(pool, thr):
    from flsim.sim import FLSimulation
    from oracle import model_ref as MR
    n, d, ep = 4, 2, 5
    osim = MR.OracleSim(n, delay=d, throttle=thr, pool=pool)
    gsim = FLSimulation(n, delay=d, throttle=thr, device=DEV, chunk_workers=2, pool=pool)
    assert np.array_equal(gsim.theta.cpu().numpy(), osim.theta)
    for t in range(ep):
        lo = osim.epoch()
        lg = gsim.epoch()
        tr_o = osim.trace[-1]
        plan = gsim.trace[-1]
        assert [i for (_, i, _) in tr_o["items"]] == list(np.nonzero(plan.computes)[0])
        assert [s for (k, s) in tr_o["appended"] if k == "stale"] == [s for (_, s) in plan.stale]
        assert abs(lg - lo) <= (1e-4 if t == 0 else 1e-3), (t, lg, lo)
    th = gsim.theta.cpu().numpy()
    assert _rel_l2(th.astype(np.float64), osim.theta.astype(np.float64)) < 1e-3


def test_reference_api_facade_loop(pool):
    """The reference's own loop structure (main.py:126-188) written against the drop-in FL.agents
    API (Worker.fwd_bkwd / Agg(rule) / Central.update_model), fed the spec's batches, against
    the oracle: same losses (tolerance), same aliasing (every fast entry is the same buffer)."""
    import torch.nn as nn
    from FL.agents import Agg, Central, Worker, rule
    from FL.models import PerformantNet1
    from oracle import model_ref as MR
    from oracle import oracle as O
    n, d, ep = 4, 2, 4
    osim = MR.OracleSim(n, delay=d, throttle=True, pool=pool)
    torch.manual_seed(0)
    model = PerformantNet1().to(DEV)
    optimizer = torch.optim.Adam(model.parameters(), lr=0.001)
    central = Central(model, optimizer)
    workers = [Worker(nn.CrossEntropyLoss()) for _ in range(n)]
    for i, w in enumerate(workers):
        w.index = i
    agg = Agg(rule)
    rs = np.random.RandomState(0)
    lists = O.class_lists(pool[1])
    lut = O.normalize_lut()
    pesky, window, gone = [], 0, False
    for t in range(ep):
        weight_ups, losses = [], []
        model.train()
        for i in range(n):
            k = rs.randint(0, n)
            idx = O.batch_indices(0, t, i, k, n, lists)
            x = torch.from_numpy(lut[pool[0][idx]]).to(DEV)
            y = torch.from_numpy(pool[1][idx]).to(DEV)
            if i == n - 1:
                gone = False
                ups = None
                if t == 0:
                    workers[i].model = central.model
                    ups, _ = workers[i].fwd_bkwd(x, y)
                    pesky.append(ups)
                    ups = None
                elif t % d == 0:
                    workers[i].model = central.model
                    ups, _ = workers[i].fwd_bkwd(x, y)
                    pesky.append(ups)
                    ups = pesky.pop(0)
                if ups is not None:
                    weight_ups.append(ups)
                    gone = True
            elif window <= 0:
                workers[i].model = central.model
                ups, lv = workers[i].fwd_bkwd(x, y)
                weight_ups.append(ups)
                losses.append(lv)
                window = 1 if gone else 2
            if window > 0:
                window -= 1
        fin = agg.rule(weight_ups)
        central.update_model(fin)
        lo = osim.epoch()
        assert abs(float(np.mean(losses)) - lo) <= (1e-4 if t == 0 else 1e-3), (t, lo)
        assert len({u[0].data_ptr() for u in weight_ups[:len(losses)]}) == 1
    th = torch.cat([p.detach().reshape(-1) for p in model.parameters()]).cpu().numpy()
    assert _rel_l2(th.astype(np.float64), osim.theta.astype(np.float64)) < 1e-3
