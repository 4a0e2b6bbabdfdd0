"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle on the same seeded inputs.

Tolerances:
  * aggregation + Adam kernel: bit-exact with the oracle (same correctly rounded sqrt);
  * one worker-step gradient (tests/_flips.py): the arithmetic within 2e-6 (rel-L2) of an fp64
    oracle that takes the GPU's own forward decisions, and the decisions (ReLU signs, pool
    argmax) that differ from the fp64 oracle's own at most 3x the CPU fp32 port's count + 6 --
    a single knife-edge flip moves the gradient by up to ~5e-3 (profiles/r02a/flip_census.txt),
    so a flat tolerance against fp64 is either loose or flaky;
  * losses: |dloss| <= 1e-4 on the first step, <= 1e-3 over the first epochs;
  * staleness trace: bit-exact.
"""
import json

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
    bad = {}
    for name, a, b in (("p", dp, p), ("m", dm, m), ("v", dv, v)):
        got = a.cpu().numpy()
        bad[name] = int((got.view(np.uint32) != b.view(np.uint32)).sum())
    assert bad == {"p": 0, "m": 0, "v": 0}, bad


@pytest.mark.parametrize("c,ns,sizes", [
    (4095, 0, [1000, 4096, 33, 7]),                       # k = 4095: three level-1 groups
    (16383, 1, [2048, 31, 4000]),                         # 16k workers (configs[3])
    (6, 3, [5, 37, 64, 1, 96, 100, 33, 2, 3, 70, 9, 11]), # > 8 tails: split launches
])
def test_aggregate_adam_layouts_and_edges(c, ns, sizes):
    """Large k, odd tensor layouts (many row_sum tails, unaligned tensor starts) and the value
    edge cases of the division paths: +-0, subnormal and huge gradients."""
    from flsim.engine import aggregate_adam
    from oracle import oracle as O
    P = sum(sizes)
    rs = np.random.RandomState(c + ns)
    S = (rs.standard_normal(P) * 1e-2).astype(np.float32)
    S[::17] = 0.0
    S[1::17] = -0.0
    S[2::17] = np.float32(3e-39) * rs.choice([-1, 1], len(S[2::17]))
    S[3::17] = np.float32(1e30)
    stale = [(rs.standard_normal(P) * 1e-2).astype(np.float32) for _ in range(ns)]
    p = rs.standard_normal(P).astype(np.float32)
    m = (rs.standard_normal(P) * 1e-3).astype(np.float32)
    v = (rs.rand(P) * 1e-5).astype(np.float32)
    dS = torch.from_numpy(S).to(DEV)
    dst = [torch.from_numpy(s).to(DEV) for s in stale]
    dp, dm, dv = (torch.from_numpy(a.copy()).to(DEV) for a in (p, m, v))
    aggregate_adam(dS, c, dst, dp, dm, dv, 2, sizes)
    torch.cuda.synchronize()
    g = np.empty_like(S)
    off = 0
    for n in sizes:
        g[off:off + n] = O.cascade_mean([S[off:off + n]] * c + [s[off:off + n] for s in stale])
        off += n
    O.adam_step(p, m, v, g, 2)
    bad = {}
    for name, a, b in (("p", dp, p), ("m", dm, m), ("v", dv, v)):
        got = a.cpu().numpy()
        bad[name] = int((got.view(np.uint32) != b.view(np.uint32)).sum())
    assert bad == {"p": 0, "m": 0, "v": 0}, bad


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


def _items_batch(sim, items, dropout=True):
    """The chunk's inputs as one batch: x, y and the dropout noise of each worker-step's
    128-sample group (key (t, i))."""
    import _flips
    xs, ys = zip(*[sim.batch(*it, dtype=torch.float64) for it in items])
    x, y = torch.cat(xs), torch.cat(ys)
    return x, y, _flips.noise_groups([(t, i) for (t, i, _) in items], x.shape[0], dropout)


@pytest.mark.parametrize("dropout", [False, True])
def test_single_worker_step_gradient(pool, dropout):
    import torch as T
    from flsim.data import DevicePool
    from flsim.engine import PN1Engine, worker_table
    from oracle import model_ref as MR
    import _flips
    sim = MR.OracleSim(4, delay=2, pool=pool, dropout=dropout)
    items = [(0, 0, 0)]
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
    x, y, noise = _items_batch(sim, items, dropout)
    _flips.check_worker_step(S.cpu().numpy().astype(np.float64), eng, sim.theta, x, y, noise,
                             1.0 / 128)


def test_chunk_of_workers_sums_gradients(pool):
    """A chunk of 3 worker-steps (different (t,i,k), incl. the {1,9} dataset) == the sum of the
    per-worker gradients (agents.py:35 accumulation) -- oracle runs them sequentially."""
    import torch as T
    from flsim.data import DevicePool
    from flsim.engine import PN1Engine, worker_table
    from oracle import model_ref as MR
    import _flips
    sim = MR.OracleSim(4, delay=2, pool=pool)
    items = [(2, 0, 1), (2, 1, 3), (2, 3, 0)]
    g64, l64 = sim.grad_of(sim.theta, items, dtype=T.float64)
    eng = PN1Engine(DEV, chunk_workers=2)
    dpool = DevicePool(DEV, 0, pool)
    theta = T.from_numpy(sim.theta.copy()).to(DEV)
    eng.begin_epoch(theta)
    loss = T.zeros(3, device=DEV)
    eng.run_chunk(theta, dpool, worker_table(items[:2], DEV), 2, 4, 0, True, loss[:2])
    S1 = T.zeros(eng.P, device=DEV)
    eng.end_epoch(S1)
    x, y, noise = _items_batch(sim, items[:2])
    _flips.check_worker_step(S1.cpu().numpy().astype(np.float64), eng, sim.theta, x, y, noise,
                             1.0 / 128)
    eng.run_chunk(theta, dpool, worker_table(items[2:], DEV), 1, 4, 0, True, loss[2:])
    S = T.zeros(eng.P, device=DEV)
    eng.end_epoch(S)                  # the slabs kept chunk 1: S = both chunks (agents.py:35)
    T.cuda.synchronize()
    np.testing.assert_allclose(loss.cpu().numpy(), l64, atol=1e-4)
    x, y, noise = _items_batch(sim, items[2:])
    d2 = S.cpu().numpy().astype(np.float64) - S1.cpu().numpy().astype(np.float64)
    _flips.check_worker_step(d2, eng, sim.theta, x, y, noise, 1.0 / 128)
    assert _rel_l2(S.cpu().numpy().astype(np.float64), g64) <= 1e-2


def test_small_chunk_tiles_bit_identical(pool):
    """Chunks of at most small_chunk_samples() (256) samples run the GEMMs on half-height tiles
    (net_kernels.h): the k order per output is the large tiles', so the forward -- and
    with it every worker's loss -- must be bit-identical.  One worker (128 samples: the facade's
    one-call forward, flsim_pn1_fwd_rows) and two workers (256 samples), both on the small tiles,
    against the same workers inside a three-worker chunk (384 samples, large tiles).  Only the
    forward is compared bit for bit: the weight gradients' split of the pixel range follows the
    chunk size (wsplit), so a chunk's gradient bits depend on its size by design; its accuracy
    is checked per tensor at every chunk size by the worker-step and chunk tests
    (test_gpu_survey_chunk.py)."""
    import torch as T
    from flsim.data import DevicePool
    from flsim.engine import PN1Engine, worker_table
    from oracle import model_ref as MR
    sim = MR.OracleSim(4, delay=2, pool=pool)
    items = [(3, 0, 1), (3, 2, 3), (3, 3, 0)]
    eng = PN1Engine(DEV, chunk_workers=3)
    dpool = DevicePool(DEV, 0, pool)
    theta = T.from_numpy(sim.theta.copy()).to(DEV)
    eng.begin_epoch(theta)
    tiny = T.zeros(1, device=DEV)
    small = T.zeros(2, device=DEV)
    large = T.zeros(3, device=DEV)
    eng.run_chunk(theta, dpool, worker_table(items[:1], DEV), 1, 4, 0, True, tiny)
    eng.run_chunk(theta, dpool, worker_table(items[:2], DEV), 2, 4, 0, True, small)
    eng.run_chunk(theta, dpool, worker_table(items, DEV), 3, 4, 0, True, large)
    S = T.zeros(eng.P, device=DEV)
    eng.end_epoch(S)
    T.cuda.synchronize()
    a = small.cpu().numpy()
    b = large[:2].cpu().numpy()
    c = tiny.cpu().numpy()
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), (a, b)
    assert np.array_equal(c.view(np.uint32), b[:1].view(np.uint32)), (c, b)
    assert np.all(np.isfinite(S.cpu().numpy()))


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
    # Adam turns last-bit gradient differences into O(lr) parameter moves: compare
    # the drift from the fp64 oracle with the CPU's own fp32-vs-fp64 drift (4.7e-3 / 2.2e-3 after
    # 5 epochs without / with throttle, measured in the build container).
    o64 = MR.OracleSim(n, delay=d, throttle=thr, pool=pool, dtype=torch.float64)
    for t in range(ep):
        o64.epoch()
    th = gsim.theta.cpu().numpy().astype(np.float64)
    drift_gpu = _rel_l2(th, o64.theta.astype(np.float64))
    drift_cpu = _rel_l2(osim.theta.astype(np.float64), o64.theta.astype(np.float64))
    print("MEASURED", json.dumps(dict(test=f"n4_d2_trajectory_thr{int(thr)}",
                                      drift_gpu=drift_gpu, drift_cpu=drift_cpu,
                                      ratio=drift_gpu / drift_cpu)))
    # bound = 1.5 x the ratio the split-bf16 build measured on MI355X (2.39 without throttle,
    # 1.20 with; profiles/r04/prof_r04e/pytest_gpu.txt MEASURED)
    assert drift_gpu <= (3.6 if not thr else 1.8) * drift_cpu, (drift_gpu, drift_cpu)


def test_warm_start_model_file_trajectory(pool, tmp_path):
    """configs[1]'s --model_file warm start: a pre-trained state_dict (written by the engine's
    model_state_dict, as tools/make_warm_start.py does) loaded through load_model_file starts
    the GPU run and the oracle at the same theta; same trace, losses within the trajectory
    tolerance."""
    from flsim.sim import FLSimulation, load_model_file
    from oracle import model_ref as MR
    pre = FLSimulation(4, delay=2, throttle=True, seed=1, device=DEV, chunk_workers=2, pool=pool)
    for _ in range(3):
        pre.epoch()
    path = str(tmp_path / "warm_start.pt")
    torch.save(pre.model_state_dict(), path)
    theta0, _ = load_model_file(path)
    assert torch.equal(theta0, pre.theta.cpu()[:theta0.numel()])
    n, d = 4, 2
    osim = MR.OracleSim(n, delay=d, throttle=True, pool=pool, theta0=theta0.numpy())
    gsim = FLSimulation(n, delay=d, throttle=True, device=DEV, chunk_workers=2, pool=pool,
                        theta0=theta0)
    for t in range(4):
        lo = osim.epoch()
        lg = gsim.epoch()
        assert [i for (_, i, _) in osim.trace[-1]["items"]] == \
            list(np.nonzero(gsim.trace[-1].computes)[0])
        assert abs(lg - lo) <= (1e-4 if t == 0 else 1e-3), (t, lg, lo)


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
    assert _rel_l2(th.astype(np.float64), osim.theta.astype(np.float64)) < 0.03


def _gather_pool(z, idx_nhwc):
    """max-pool with the GPU's argmax decisions: z [N,C,H,W], idx [N,PH,PW,C] (0..3)."""
    idx = torch.from_numpy(idx_nhwc.astype(np.int64)).permute(0, 3, 1, 2)
    N, C, PH, PW = idx.shape
    rows = 2 * torch.arange(PH).view(1, 1, PH, 1) + (idx >> 1)
    cols = 2 * torch.arange(PW).view(1, 1, 1, PW) + (idx & 1)
    n = torch.arange(N).view(N, 1, 1, 1)
    c = torch.arange(C).view(1, C, 1, 1)
    return z[n, c, rows, cols]


@pytest.mark.parametrize("dropout,items", [
    (False, [(0, 1, 2)]), (True, [(0, 1, 2)]), (True, [(1, 0, 3), (1, 2, 0)])])
def test_gradient_teacher_forced_decisions(pool, dropout, items):
    """Backward kernels checked tightly: an fp64 reference that takes the GPU's own forward
    decisions (ReLU signs, max-pool argmax, dropout masks) must give the GPU's gradient to fp32
    accumulation accuracy (per-tensor rel-L2 <= 2e-5).  Decision flips at near-zero
    pre-activations are what the looser rel-L2 <= 5e-3 of test_single_worker_step_gradient covers.
    The two-item case runs both workers as ONE chunk (256 samples): the chunk's gradient must be
    the sum of the per-worker mean-CE gradients (agents.py:35 accumulation)."""
    import torch.nn.functional as F
    from flsim.data import DevicePool
    from flsim.engine import PN1Engine, PN1_SHAPES, worker_table
    from oracle import model_ref as MR
    nw = len(items)
    NS = 128 * nw
    sim = MR.OracleSim(4, delay=2, pool=pool, dropout=dropout)
    eng = PN1Engine(DEV, chunk_workers=nw)
    dpool = DevicePool(DEV, 0, pool)
    theta = torch.from_numpy(sim.theta.copy()).to(DEV)
    eng.begin_epoch(theta)
    loss = torch.zeros(nw, device=DEV)
    eng.run_chunk(theta, dpool, worker_table(items, DEV), nw, 4, 0, dropout, loss)
    S = torch.zeros(eng.P, device=DEV)
    eng.end_epoch(S)
    torch.cuda.synchronize()
    W = lambda i, shp, dt=torch.float32: eng.workspace_view(i, shp, dt).cpu().numpy()
    nchw = lambda a: torch.from_numpy(np.ascontiguousarray(a.transpose(0, 3, 1, 2)))
    A = dict(a1=nchw(W(1, (NS, 34, 34, 48))), d1=nchw(W(3, (NS, 18, 18, 48))),
             a3=nchw(W(4, (NS, 20, 20, 96))), d2=nchw(W(6, (NS, 11, 11, 96))),
             a5=nchw(W(7, (NS, 13, 13, 192))), d3=torch.from_numpy(W(9, (NS, 9408))),
             e1=torch.from_numpy(W(10, (NS, 512))), e2=torch.from_numpy(W(11, (NS, 256))),
             i1=W(19, (NS, 18, 18, 48), torch.uint8), i2=W(20, (NS, 11, 11, 96), torch.uint8),
             i3=W(21, (NS, 7, 7, 192), torch.uint8))
    import _flips

    def forced(dt):
        """the reference forward + backward in dtype dt with the GPU's decisions"""
        np_dt = np.float64 if dt == torch.float64 else np.float32
        P = [torch.tensor(a, requires_grad=True) for a in MR.split_flat(sim.theta.astype(np_dt))]
        (w1, b1, w2, b2, w3, b3, w4, b4, w5, b5, w6, b6, l1w, l1b, l2w, l2b, l3w, l3b) = P
        m = lambda t: (t > 0).to(dt)                                      # noqa: E731
        s50 = 2.0 if dropout else 1.0
        lrefs = []
        for wi, it in enumerate(items):
            sl = slice(128 * wi, 128 * (wi + 1))
            a = {k: v[sl] for k, v in A.items()}
            x, y = sim.batch(*it, dtype=dt)
            noise = MR.dropout_noise(0, it[0], it[1], 128, dt) if dropout else None
            h = F.conv2d(x, w1, b1, padding=2) * m(a["a1"])
            h = _gather_pool(F.conv2d(h, w2, b2, padding=2), a["i1"]) * m(a["d1"])
            h = h * noise[0] if dropout else h
            h = F.conv2d(h, w3, b3, padding=2) * m(a["a3"])
            h = _gather_pool(F.conv2d(h, w4, b4, padding=2), a["i2"]) * m(a["d2"])
            h = h * noise[1] if dropout else h
            h = F.conv2d(h, w5, b5, padding=2) * m(a["a5"])
            h = _gather_pool(F.conv2d(h, w6, b6, padding=2), a["i3"]).reshape(128, -1) * m(a["d3"])
            h = h * noise[2].reshape(128, -1) if dropout else h
            h = F.linear(h, l1w, l1b) * m(a["e1"]) * s50
            h = F.linear(h, l2w, l2b) * m(a["e2"]) * s50
            lref = F.cross_entropy(F.linear(h, l3w, l3b), y)
            lref.backward()
            lrefs.append(lref.item())
        return torch.cat([p.grad.reshape(-1) for p in P]).double().numpy(), lrefs

    g_tf, lrefs = forced(torch.float64)
    g_tf32, _ = forced(torch.float32)
    g = S.cpu().numpy().astype(np.float64)
    off = 0
    worst = {}
    for (name, shp) in PN1_SHAPES:
        n = int(np.prod(shp))
        worst[name] = _rel_l2(g[off:off + n], g_tf[off:off + n])
        off += n
    np.testing.assert_allclose(loss.cpu().numpy(), lrefs, atol=1e-5)
    assert max(worst.values()) <= 2e-5, worst
    # per tensor no farther from fp64 than 2x the CPU fp32 port (same decisions)
    _flips.assert_survey(_flips.survey_ratios(g, g_tf32, g_tf, PN1_SHAPES), "pn1_teacher_forced")


def test_eval_predictions_match_oracle(pool):
    """Device evaluation (util.py:31-45, dropout off) vs the oracle's fp32 CPU forward: chunks of
    256 samples and a ragged last chunk (1000 images), predictions = argmax with first-max ties.
    Predictions may differ only where two logits are within fp32 noise of each other."""
    from flsim.data import DevicePool, make_test_pool
    from flsim.engine import PN1Engine
    from oracle import model_ref as MR
    sim = MR.OracleSim(4, delay=2, pool=pool)
    test = make_test_pool(0, size=1000)
    eng = PN1Engine(DEV, chunk_workers=2)
    dtest = DevicePool(DEV, 0, test)
    theta = torch.from_numpy(sim.theta.copy()).to(DEV)
    pred = eng.evaluate(theta, dtest).cpu().numpy()
    ref = MR.predict(sim.theta, test[0])
    assert pred.shape == (1000,)
    assert (pred == ref).mean() >= 0.995, (pred != ref).sum()
    pred2 = eng.evaluate(theta, dtest, first=100, n_images=37).cpu().numpy()
    assert np.array_equal(pred2, pred[100:137])


def test_simulation_evaluate_and_checkpoint_resume(pool, tmp_path):
    """FLSimulation.evaluate returns the reference's accuracy numbers; a run cut in two by
    save_checkpoint / restore continues bit for bit (theta, Adam state, FIFO'd stale gradient)."""
    from flsim.sim import FLSimulation
    n, d, total, cut = 4, 2, 5, 3
    ref = FLSimulation(n, delay=d, throttle=True, device=DEV, chunk_workers=2, pool=pool)
    for _ in range(total):
        ref.epoch()
    acc, per = ref.evaluate()
    assert 0.0 <= acc <= 100.0 and len(per) == 10
    labels = ref._test.labels.cpu().numpy()
    assert abs(acc - np.mean([per[c] for c in range(10)])) < 1e-6   # balanced classes
    a = FLSimulation(n, delay=d, throttle=True, device=DEV, chunk_workers=2, pool=pool)
    for _ in range(cut):
        a.epoch()
    path = str(tmp_path / "ck.pt")
    a.save_checkpoint(path)
    b = FLSimulation(n, delay=d, throttle=True, device=DEV, chunk_workers=2, pool=pool)
    b.restore(path)
    for _ in range(total - cut):
        b.epoch()
    for x, y in ((b.theta, ref.theta), (b.m, ref.m), (b.v, ref.v)):
        assert torch.equal(x, y)
    assert b.losses() == ref.losses()
    sd = b.model_state_dict()
    from FL.models import PerformantNet1
    m = PerformantNet1()
    m.load_state_dict(sd)                     # the reference's load_state_dict contract
    assert len(labels) == 10000


@pytest.mark.parametrize("k,nev,sizes", [
    (37, 5, [64, 33, 100]),                    # events inside blocks and the row_sum tails
    (700, 40, [1000, 31, 4099]),               # pure level-1 groups between mixed blocks
    (5000, 3, [2048, 7]),                      # pure level-2 groups (k > 4096)
    (12, 12, [40, 10]),                        # every entry a stale one
    (16383, 50, [5000, 4099, 31, 70000]),      # configs[3]'s size: 16k entries, ~50 events
])
def test_aggregate_adam_general_order_bit_exact(k, nev, sizes):
    """Heterogeneous-delay extension: stale entries interleaved with the S_t copies in worker
    order, several entries sharing one stale array, a zero (torch-1.x) entry; bit-exact vs the
    oracle's cascade over the explicit entry list."""
    from flsim.engine import ProgramStager, Rule, aggregate_rule
    from oracle import oracle as O
    P = sum(sizes)
    rs = np.random.RandomState(k + nev)
    S = (rs.standard_normal(P) * 1e-2).astype(np.float32)
    arrays = [(rs.standard_normal(P) * 1e-2).astype(np.float32) for _ in range(3)]
    pos = np.sort(rs.choice(k, nev, replace=False))
    which = rs.randint(0, 4, nev)               # 3 = the zero entry
    p = rs.standard_normal(P).astype(np.float32)
    m = (rs.standard_normal(P) * 1e-3).astype(np.float32)
    v = (rs.rand(P) * 1e-5).astype(np.float32)
    dS = torch.from_numpy(S).to(DEV)
    darr = [torch.from_numpy(a).to(DEV) for a in arrays] + [None]
    dp, dm, dv = (torch.from_numpy(a.copy()).to(DEV) for a in (p, m, v))
    rule = Rule(k, darr, events=list(zip(pos.tolist(), which.tolist())),
                stager=ProgramStager(DEV))
    aggregate_rule(dS, rule, dp, dm, dv, 4, sizes)
    torch.cuda.synchronize()
    zero = np.zeros(P, np.float32)
    ents = [S] * k
    for q, w in zip(pos, which):
        ents[q] = arrays[w] if w < 3 else zero
    g = np.empty_like(S)
    off = 0
    for n in sizes:
        g[off:off + n] = O.cascade_mean([e[off:off + n] for e in ents])
        off += n
    O.adam_step(p, m, v, g, 4)
    bad = {name: int((a.cpu().numpy().view(np.uint32) != b.view(np.uint32)).sum())
           for name, a, b in (("p", dp, p), ("m", dm, m), ("v", dv, v))}
    assert bad == {"p": 0, "m": 0, "v": 0}, bad


def test_general_order_kernel_equals_reference_kernel():
    """On the reference order ([S_t] * c, stale last) both aggregation kernels agree bit for bit."""
    from flsim.engine import PN1Engine, PN1_SIZES, ProgramStager, Rule, aggregate_rule
    eng = PN1Engine(DEV, chunk_workers=1)
    P = eng.P
    g = torch.Generator(device="cpu").manual_seed(5)
    S = (torch.randn(P, generator=g) * 1e-2).to(DEV)
    st = (torch.randn(P, generator=g) * 1e-2).to(DEV)
    base = [torch.randn(P, generator=g).to(DEV), torch.zeros(P, device=DEV),
            torch.zeros(P, device=DEV)]
    a = [t.clone() for t in base]
    b = [t.clone() for t in base]
    eng.aggregate_adam(S, 511, [st], *a, 1)
    aggregate_rule(S, Rule(512, [st], events=[(511, 0)], stager=ProgramStager(DEV)), *b, 1,
                   PN1_SIZES)
    for x, y in zip(a, b):
        assert torch.equal(x, y)


def test_heterogeneous_delays_trajectory(pool):
    """Several slow workers with their own delays and FIFOs (SURVEY 8 a1 extension), stale
    entries interleaved in worker order: staleness trace identical to the oracle's loop, losses
    within the fp32 tolerance."""
    from flsim.sim import FLSimulation
    from oracle import model_ref as MR
    delays = [0, 2, 0, 3, 0, 2]
    n, ep = len(delays), 7
    osim = MR.OracleSim(n, delays=delays, throttle=True, pool=pool)
    gsim = FLSimulation(n, delays=delays, throttle=True, device=DEV, chunk_workers=2, pool=pool)
    for t in range(ep):
        lo = osim.epoch()
        lg = gsim.epoch()
        tr_o = osim.trace[-1]
        plan = gsim.trace[-1]
        assert [i for (_, i, _) in tr_o["items"]] == list(np.nonzero(plan.computes)[0])
        assert [s for (kd, s) in tr_o["appended"] if kd == "stale"] == [s for (_, s) in plan.stale]
        if not np.isnan(lo):
            assert abs(lg - lo) <= (1e-4 if t == 0 else 1e-3), (t, lg, lo)


def test_max_chunk_matches_small_chunks(pool):
    """The largest worker-batched launch (128 workers = 16,384 samples, the 32-bit index budget)
    against 4 launches of 32 from the same theta and batches: the forward does not depend on the
    chunking, so every worker's loss is bit-identical; S_t differs only by the split-K slab
    order (rel-L2 <= 1e-5 per tensor)."""
    from flsim.engine import PN1_SHAPES
    from flsim.sim import FLSimulation
    n = 129                                   # epoch 1: the 128 fast workers, no tick
    a = FLSimulation(n, delay=50, throttle=False, device=DEV, chunk_workers=32, pool=pool,
                     keep_S=True)
    b = FLSimulation(n, delay=50, throttle=False, device=DEV, chunk_workers=128, pool=pool,
                     keep_S=True)
    a.epoch()
    b.epoch()
    for x, y in ((b.theta, a.theta), (b.m, a.m), (b.v, a.v)):
        x.copy_(y)
    assert b.chunks(0, 128) == [(0, 128)]
    la, lb = a.epoch(), b.epoch()
    assert int(a.trace[-1].computes.sum()) == 128
    assert la == lb
    wa = a.comm[a.Ppad:a.Ppad + 128].cpu().numpy()
    wb = b.comm[b.Ppad:b.Ppad + 128].cpu().numpy()
    assert np.array_equal(wa.view(np.uint32), wb.view(np.uint32))
    sa = a.comm[:a.P].cpu().numpy().astype(np.float64)
    sb = b.comm[:b.P].cpu().numpy().astype(np.float64)
    off = 0
    for (name, _), size in zip(PN1_SHAPES, _sizes()):
        r = _rel_l2(sb[off:off + size], sa[off:off + size])
        assert r <= 1e-5, (name, r)
        off += size


@pytest.mark.parametrize("thr", [False, True])
def test_independent_entries_trajectory(pool, thr):
    """Independent-entry semantics (distinct per-worker weight_ups entries; the slow worker's
    FIFO holds its own gradient) against the oracle's per-worker restatement: same trace, losses
    within the trajectory tolerance, parameter drift bounded by the CPU's own fp32 drift."""
    from flsim.sim import FLSimulation
    from oracle import model_ref as MR
    n, d, ep = 4, 2, 5
    osim = MR.OracleSim(n, delay=d, throttle=thr, pool=pool, semantics="independent")
    gsim = FLSimulation(n, delay=d, throttle=thr, device=DEV, chunk_workers=2, pool=pool,
                        semantics="independent")
    for t in range(ep):
        lo = osim.epoch()
        lg = gsim.epoch()
        assert [i for (_, i, _) in osim.trace[-1]["items"]] == \
            list(np.nonzero(gsim.trace[-1].computes)[0])
        assert abs(lg - lo) <= (1e-4 if t == 0 else 1e-3), (t, lg, lo)
    o64 = MR.OracleSim(n, delay=d, throttle=thr, pool=pool, dtype=torch.float64,
                       semantics="independent")
    for t in range(ep):
        o64.epoch()
    th = gsim.theta.cpu().numpy().astype(np.float64)
    drift_gpu = _rel_l2(th, o64.theta.astype(np.float64))
    drift_cpu = _rel_l2(osim.theta.astype(np.float64), o64.theta.astype(np.float64))
    print("MEASURED", json.dumps(dict(test=f"n4_d2_independent_thr{int(thr)}",
                                      drift_gpu=drift_gpu, drift_cpu=drift_cpu,
                                      ratio=drift_gpu / drift_cpu)))
    # bound = 1.5 x the ratio the split-bf16 build measured on MI355X (3.04 without throttle,
    # 2.45 with; profiles/r04/prof_r04e/pytest_gpu.txt MEASURED; the GPU sums the fast
    # workers' gradients in GEMM order, the oracle per worker)
    assert drift_gpu <= (4.6 if not thr else 3.7) * drift_cpu, (drift_gpu, drift_cpu)
