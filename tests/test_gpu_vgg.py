"""GPU parity of the VGG-11 engine (configs[4]; models.py:50-103, flsim_vgg11_* in
csrc/vgg_net.hip) through the C-ABI, against the oracle's torch-CPU restatement (oracle/model_ref.py
VGG11Ref, itself pinned to the reference's own vgg11() by tests/golden/vgg.npz).

Tolerances (as tests/test_gpu_parity.py):
  * one worker-step gradient: per-tensor rel-L2 vs fp64 <= 5e-3; whole gradient within
    2.5e-4 of |g64| (or 4x the CPU's own fp32 error), or else at most 8 knife-edge decisions
    that fp64 takes the other way, with the teacher-forced gradient exact to TF_TOL;
  * teacher-forced (the GPU's own ReLU / argmax / dropout decisions in an fp64 reference):
    per-tensor rel-L2 <= TF_TOL, losses to 1e-5;
  * losses |dloss| <= 1e-4 on the first step, <= 1e-3 over the first epochs; trace bit-exact.
"""
import numpy as np
import pytest
import torch

from conftest import has_gpu

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not has_gpu(), reason="needs an MI355X")]


# per-tensor rel-L2 of the GPU gradient against the fp64 reference with the GPU's own decisions.
# The bound is 1.5 x the shipped build's measured worst: features.18.weight at 1.35e-6 (dropout,
# items1; 8.3e-7 and 1.10e-6 for the other cases; profiles/r05/tol_r05j.jsonl).  Round
# 4's build, with the data gradients on the split-bf16 MFMA, measured 3.14e-5: the MFMA's
# truncating sums biased them.  A wrong kernel misses by orders of magnitude.
TF_TOL = 2.1e-6

def _tol_log(worst):
    """Per-tensor error census across builds (measurement only: FLSIM_TOL_LOG=<file>)."""
    import json
    import os
    path = os.environ.get("FLSIM_TOL_LOG")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps(dict(test=os.environ.get("PYTEST_CURRENT_TEST", ""),
                                    worst={k: float(v) for k, v in worst.items()})) + "\n")

DEV = "cuda:0"
M = "vgg11"


@pytest.fixture(scope="module")
def pool():
    from oracle import oracle as O
    return O.make_pool(0)


def _rel_l2(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def _run(theta_np, items, dropout, pool, n_total=4):
    """One chunk of len(items) worker-steps through flsim_vgg11_fwd_bwd_chunk -> S, losses."""
    from flsim.data import DevicePool
    from flsim.engine import VGG11Engine, worker_table
    nw = len(items)
    eng = VGG11Engine(DEV, chunk_workers=nw)
    dpool = DevicePool(DEV, 0, pool)
    theta = torch.from_numpy(theta_np.copy()).to(DEV)
    eng.begin_epoch(theta)
    loss = torch.zeros(nw, device=DEV)
    eng.run_chunk(theta, dpool, worker_table(items, DEV), nw, n_total, 0, dropout, loss)
    S = torch.zeros(eng.P, device=DEV)
    eng.end_epoch(S)
    torch.cuda.synchronize()
    return eng, S.cpu().numpy().astype(np.float64), loss.cpu().numpy()


def _teacher_forced(sim, eng, items, dropout, dt=torch.float64):
    """fp64 VGG-11 forward + backward that takes the GPU's own forward decisions (ReLU signs, max-
    pool argmax, dropout masks, read back from the workspace).  Returns the per-tensor gradient,
    the per-worker losses, and the number of GPU decisions that the fp64 pre-activations computed
    on the way disagree with (a ReLU sign, a pool argmax among live windows, a kept unit whose
    fp64 pre-activation is <= 0): knife-edge decisions any fp32 order can take either way.
    dt = torch.float32: the CPU fp32 port given the same decisions (SURVEY 8(c)'s comparison)."""
    import torch.nn.functional as F
    import _flips
    from flsim.engine import VGG11Engine
    from oracle import model_ref as MR
    from test_gpu_parity import _gather_pool
    NS = 128 * len(items)
    ids = {name: j for j, name in enumerate(VGG11Engine.WORKSPACE)}

    def W(name, shp, dt=torch.float32):
        return eng.workspace_view(ids[name], shp, dt).cpu().numpy()

    def nchw(a):
        return torch.from_numpy(np.ascontiguousarray(a.transpose(0, 3, 1, 2))).to(dt)

    A = dict(d1=nchw(W("d1", (NS, 16, 16, 64))), d2=nchw(W("d2", (NS, 8, 8, 128))),
             a3=nchw(W("a3", (NS, 8, 8, 256))), d4=nchw(W("d4", (NS, 4, 4, 256))),
             a5=nchw(W("a5", (NS, 4, 4, 512))), d6=nchw(W("d6", (NS, 2, 2, 512))),
             a7=nchw(W("a7", (NS, 2, 2, 512))), f0=torch.from_numpy(W("f0", (NS, 512))).to(dt),
             e1=torch.from_numpy(W("e1", (NS, 512))).to(dt),
             e2=torch.from_numpy(W("e2", (NS, 512))).to(dt),
             i1=W("i1", (NS, 16, 16, 64), torch.uint8), i2=W("i2", (NS, 8, 8, 128), torch.uint8),
             i4=W("i4", (NS, 4, 4, 256), torch.uint8), i6=W("i6", (NS, 2, 2, 512), torch.uint8),
             i8=W("i8", (NS, 1, 1, 512), torch.uint8))
    np_dt = np.float64 if dt == torch.float64 else np.float32
    P = [torch.tensor(a, requires_grad=True)
         for a in MR.split_flat(sim.theta.astype(np_dt), M)]
    cw, cb = P[0:16:2], P[1:16:2]
    l1w, l1b, l2w, l2b, l3w, l3b = P[16:]
    flips = [0]

    def m(t):
        return (t > 0).to(dt)

    def conv(h, j):
        return F.conv2d(h, cw[j], cb[j], padding=1)

    def pool(z, idx, mask, kept_only=False):
        zd = z.detach()
        own = _flips.pool_idx(F.relu(zd))
        gidx = torch.from_numpy(idx.astype(np.int64)).permute(0, 3, 1, 2)
        pz = _gather_pool(zd, idx)
        live = (pz > 0) | (mask > 0)
        flips[0] += int(((own != gidx) & live).sum())
        flips[0] += int(((mask > 0) & (pz <= 0)).sum()) if kept_only else int(((pz > 0) != (mask > 0)).sum())
        return _gather_pool(z, idx) * m(mask)

    def relu(z, mask, kept_only=False):
        zd = z.detach()
        flips[0] += int(((mask > 0) & (zd <= 0)).sum()) if kept_only else int(((zd > 0) != (mask > 0)).sum())
        return z * m(mask)

    s50 = 2.0 if dropout else 1.0
    lrefs = []
    for wi, it in enumerate(items):
        sl = slice(128 * wi, 128 * (wi + 1))
        a = {k: v[sl] for k, v in A.items()}
        x, y = sim.batch(*it, dtype=dt)
        h = pool(conv(x, 0), a["i1"], a["d1"])
        h = pool(conv(h, 1), a["i2"], a["d2"])
        h = relu(conv(h, 2), a["a3"])
        h = pool(conv(h, 3), a["i4"], a["d4"])
        h = relu(conv(h, 4), a["a5"])
        h = pool(conv(h, 5), a["i6"], a["d6"])
        h = relu(conv(h, 6), a["a7"])
        h = pool(conv(h, 7), a["i8"], a["f0"].reshape(128, 512, 1, 1), kept_only=dropout)
        h = h.reshape(128, 512) * s50
        h = relu(F.linear(h, l1w, l1b), a["e1"], kept_only=dropout) * s50
        h = relu(F.linear(h, l2w, l2b), a["e2"])
        lref = F.cross_entropy(F.linear(h, l3w, l3b), y)
        lref.backward()
        lrefs.append(lref.item())
    g = np.concatenate([p.grad.reshape(-1).double().numpy() for p in P])
    return g, lrefs, flips[0]


@pytest.mark.parametrize("dropout", [False, True])
def test_vgg_single_worker_step_gradient(pool, dropout):
    """The GPU gradient of one worker-step against the fp64 oracle with its OWN decisions.  A
    knife-edge decision (ReLU sign / argmax within rounding) taken the other way moves a gradient
    by ~1e-4 of |g|; so beyond the flat bound the excess must come with a handful of such
    decisions (counted against the fp64 pre-activations, at most FLIPS of ~2e6) while the
    teacher-forced gradient (same decisions) stays at fp32 accuracy."""
    from flsim.engine import VGG11_SHAPES
    from oracle import model_ref as MR
    FLIPS = 8
    sim = MR.OracleSim(4, delay=2, pool=pool, dropout=dropout, model=M)
    items = [(0, 0, 0)]
    g32, l32 = sim.grad_of(sim.theta, items)
    g64, l64 = sim.grad_of(sim.theta, items, dtype=torch.float64)
    eng, g, loss = _run(sim.theta, items, dropout, pool)
    assert abs(float(loss[0]) - l64[0]) <= 1e-4, (loss[0], l64[0])
    off = 0
    for (name, shp) in VGG11_SHAPES:
        n = int(np.prod(shp))
        r = _rel_l2(g[off:off + n], g64[off:off + n])
        off += n
        assert r <= 5e-3, (name, r)
    e_gpu = np.linalg.norm(g - g64)
    e_cpu = np.linalg.norm(g32.astype(np.float64) - g64)
    if e_gpu > max(2.5e-4 * np.linalg.norm(g64), 4 * e_cpu):
        g_tf, _, flips = _teacher_forced(sim, eng, items, dropout)
        assert 1 <= flips <= FLIPS, (e_gpu, e_cpu, flips)
        assert _rel_l2(g, g_tf) <= TF_TOL, (e_gpu, flips, _rel_l2(g, g_tf))


@pytest.mark.parametrize("dropout,items", [
    (False, [(0, 1, 2)]), (True, [(0, 1, 2)]), (True, [(1, 0, 3), (1, 2, 0)])])
def test_vgg_gradient_teacher_forced_decisions(pool, dropout, items):
    """Every backward kernel checked tightly: an fp64 reference that takes the GPU's own forward
    decisions (ReLU signs, max-pool argmax, dropout masks, read back from the workspace) must give
    the GPU's gradient to fp32 accumulation accuracy.  The two-item case is ONE chunk of 256
    samples whose gradient must be the sum of the per-worker mean-CE gradients (agents.py:35)."""
    from flsim.engine import VGG11_SHAPES
    from oracle import model_ref as MR
    sim = MR.OracleSim(4, delay=2, pool=pool, dropout=dropout, model=M)
    eng, g, loss = _run(sim.theta, items, dropout, pool)
    g_tf, lrefs, flips = _teacher_forced(sim, eng, items, dropout)
    off = 0
    worst = {}
    for (name, shp) in VGG11_SHAPES:
        n = int(np.prod(shp))
        worst[name] = _rel_l2(g[off:off + n], g_tf[off:off + n])
        off += n
    _tol_log(worst)
    np.testing.assert_allclose(loss, lrefs, atol=1e-5)
    assert max(worst.values()) <= TF_TOL, worst
    assert flips <= 8 * len(items), flips
    # per tensor no farther from fp64 than 2x the CPU fp32 port (same decisions)
    import _flips
    g_tf32, _, _ = _teacher_forced(sim, eng, items, dropout, torch.float32)
    _flips.assert_survey(_flips.survey_ratios(g, g_tf32, g_tf, VGG11_SHAPES), "vgg11_teacher_forced")


def test_vgg_simulation_matches_oracle_trajectory(pool):
    """The batched server loop with vgg11 (FLSimulation(model='vgg11')) against the oracle loop:
    bit-exact staleness trace, each epoch's loss within the fp32 forward tolerance.  The oracle
    starts every epoch from the GPU's theta / Adam moments: Adam's first steps turn any fp32
    difference in a near-zero gradient (a knife-edge decision taken the other way, see
    test_vgg_single_worker_step_gradient) into a parameter change of ~lr, so free-running
    trajectories part by more than the forward tolerance within a few epochs.  The update itself
    (rule() + Adam) is bit-exact with the oracle in tests/test_gpu_server_step.py."""
    from flsim.sim import FLSimulation
    from oracle import model_ref as MR
    n, d, ep = 3, 2, 4
    osim = MR.OracleSim(n, delay=d, throttle=True, pool=pool, model=M)
    gsim = FLSimulation(n, delay=d, throttle=True, device=DEV, chunk_workers=2, pool=pool, model=M)
    assert np.array_equal(gsim.theta.cpu().numpy(), osim.theta)
    P = osim.theta.size
    for t in range(ep):
        osim.theta = gsim.theta[:P].cpu().numpy().copy()
        osim.m = gsim.m[:P].cpu().numpy().copy()
        osim.v = gsim.v[:P].cpu().numpy().copy()
        lo = osim.epoch()
        lg = gsim.epoch()
        tr_o = osim.trace[-1]
        plan = gsim.trace[-1]
        assert [i for (_, i, _) in tr_o["items"]] == list(np.nonzero(plan.computes)[0])
        assert [s for (k, s) in tr_o["appended"] if k == "stale"] == [s for (_, s) in plan.stale]
        assert abs(lg - lo) <= 1e-4, (t, lg, lo)


def test_vgg_eval_predictions_match_oracle(pool):
    """Device evaluation (util.py:31-45, dropout off) of vgg11 vs the oracle's fp32 forward over a
    ragged 600-image range (chunks of 256); differences only at fp32 near-ties."""
    from flsim.data import DevicePool, make_test_pool
    from flsim.engine import VGG11Engine
    from oracle import model_ref as MR
    theta = MR.init_params(0, M)
    test = make_test_pool(0, size=600)
    eng = VGG11Engine(DEV, chunk_workers=2)
    pred = eng.evaluate(torch.from_numpy(theta).to(DEV), DevicePool(DEV, 0, test)).cpu().numpy()
    ref = MR.predict(theta, test[0], model=M)
    assert (pred == ref).mean() >= 0.99, (pred != ref).sum()


def test_vgg_reference_api_facade(pool):
    """FL.agents drop-in with the reference's vgg11 module: Worker.fwd_bkwd per worker (one
    aliased gradient buffer), Agg(rule), Central.update_model -- one epoch against the oracle."""
    import torch.nn as nn
    from FL.agents import Agg, Central, Worker, rule
    from FL.models import vgg11
    from oracle import model_ref as MR
    from oracle import oracle as O
    n = 3
    osim = MR.OracleSim(n, delay=2, throttle=False, pool=pool, model=M)
    torch.manual_seed(0)
    model = vgg11().to(DEV)
    central = Central(model, torch.optim.Adam(model.parameters(), lr=0.001))
    workers = [Worker(nn.CrossEntropyLoss()) for _ in range(n)]
    for i, w in enumerate(workers):
        w.index = i
    rs = np.random.RandomState(0)
    lists = O.class_lists(pool[1])
    lut = O.normalize_lut()
    model.train()
    ups, losses = [], []
    for i in range(n):
        k = rs.randint(0, n)
        idx = O.batch_indices(0, 0, i, k, n, lists)
        workers[i].model = central.model
        g, lv = workers[i].fwd_bkwd(torch.from_numpy(lut[pool[0][idx]]).to(DEV),
                                    torch.from_numpy(pool[1][idx]).to(DEV))
        if i < n - 1:               # the slow worker's t == 0 entry goes to its FIFO
            ups.append(g)
            losses.append(lv)
    central.update_model(Agg(rule).rule(ups))
    lo = osim.epoch()
    assert abs(float(np.mean(losses)) - lo) <= 1e-4, (np.mean(losses), lo)
    th = torch.cat([p.detach().reshape(-1) for p in model.parameters()]).cpu().numpy()
    # Adam's first step is ~lr * sign(g): near-zero gradients flip, so theta is
    # compared loosely, as in test_gpu_parity.test_reference_api_facade_loop
    assert _rel_l2(th.astype(np.float64), osim.theta.astype(np.float64)) < 0.03


def _vgg_facade_loop(pool, monkeypatch, lazy, n=6):
    """One epoch of main.py:126-188's worker loop through FL.agents with vgg11: losses kept as
    returned (np.mean at the end, main.py:181), chunks of 4 staged calls, the epoch's .grad read
    before update_model."""
    import torch.nn as nn
    from FL.agents import Agg, Central, Worker, rule
    from FL.models import vgg11
    from oracle import oracle as O
    monkeypatch.setenv("FLSIM_FACADE_CHUNK", "4")
    monkeypatch.setenv("FLSIM_FACADE_LAZY_LOSS", "1" if lazy else "0")
    torch.manual_seed(0)
    model = vgg11().to(DEV)
    central = Central(model, torch.optim.Adam(model.parameters(), lr=0.001))
    workers = [Worker(nn.CrossEntropyLoss()) for _ in range(n)]
    rs = np.random.RandomState(7)
    lut = O.normalize_lut()
    model.train()
    ups, losses = [], []
    for i in range(n):
        idx = rs.randint(0, pool[0].shape[0], 128)
        workers[i].model = central.model
        g, lv = workers[i].fwd_bkwd(torch.from_numpy(lut[pool[0][idx]]).to(DEV),
                                    torch.from_numpy(pool[1][idx]).to(DEV))
        ups.append(g)
        losses.append(lv)
    grad = torch.cat([t.reshape(-1) for t in ups[0]]).double().cpu()
    central.update_model(Agg(rule).rule(ups))
    mean = np.mean(losses)
    th = central.ctx.theta[:central.ctx.P].double().cpu()
    return np.asarray([float(v) for v in losses], np.float32), mean, grad, th


def test_vgg_facade_lazy_loss_matches_eager(pool, monkeypatch):
    """vgg11 through the facade with the deferred fwd_bkwd (staged 128-sample calls, one batched
    forward + backward per chunk of 4, flsim_vgg11_load_rows / fwd_bwd_loaded_rows) against a
    forward and backward per call: per-call losses and their float32 mean bit for bit (the
    forward's sums per output do not depend on the row count); the epoch's gradient differs only
    in the order the calls' partial sums are added (rel-L2 <= 1e-6), theta after the Adam step by
    at most the ~2 lr a near-zero gradient component can move."""
    la, ma, ga, ta = _vgg_facade_loop(pool, monkeypatch, lazy=False)
    lb, mb, gb, tb = _vgg_facade_loop(pool, monkeypatch, lazy=True)
    assert np.array_equal(la.view(np.uint32), lb.view(np.uint32)), (la, lb)
    assert ma.dtype == mb.dtype == np.float32 and ma == mb
    assert float((ga - gb).norm() / ga.norm()) <= 1e-6
    assert float((ta - tb).abs().max()) <= 2.1e-3
