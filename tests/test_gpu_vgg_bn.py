"""GPU parity of the vgg11_bn engine (models.py:106-108; flsim_vgg11_bn_* in csrc/vgg_net.hip +
csrc/bn_kernels.h) through the C-ABI, against the oracle's torch-CPU restatement
(oracle/model_ref.py VGG11BNRef / vgg_bn_forward, pinned to the reference's own vgg11_bn() by
tests/golden/vgg_bn.npz).

BatchNorm2d in train mode normalises every fwd_bkwd call (= one simulated worker's 128 samples)
with that call's batch statistics and advances the running buffers once per call, in worker
order.  Tolerances:
  * one worker-step gradient vs fp64: the classifier and the last BatchNorm (upstream of every
    max-pool decision in the backward) per-tensor rel-L2 <= 5e-3; the feature layers <= 5e-2.
    A max-pool near-tie that fp32 resolves differently from fp64 (measured on MI355X with
    tools/dbg_bn.py: 1 of 65,536 pooled conv8 values for worker (0, 0, 0)) moves one
    (sample, channel) gradient to another window position, and the BatchNorm backward spreads
    that over the whole channel: 0.1-1.5 % in every feature tensor.  The exactness of every
    backward kernel is the teacher-forced test's job (the GPU's own decisions, 7e-6);
  * conv biases: a bias in front of a BatchNorm cancels, so its gradient is rounding noise of a
    zero sum -- checked as an absolute error against the whole gradient's norm (<= 1e-6 |g64|,
    or 10x the CPU's);
  * teacher-forced (the GPU's ReLU / argmax / dropout decisions in an fp64 reference with fp64
    batch statistics): per-tensor rel-L2 <= 7e-6 (conv biases absolute as above), losses 1e-5;
  * running buffers: running_var rel 1e-5, running_mean abs 1e-6 after one call (the trajectory
    test: abs 2e-4, see tests/test_oracle_golden._check_running);
  * losses |dloss| <= 1e-4 / 2e-3 / 5e-3 / 1e-2 over epochs 0-3: the near-tie flips above, then
    Adam's sign sensitivity on near-zero gradients.  Calibration: the oracle's own fp32 run
    drifts from its fp64-gradient run by 0 / 4e-5 / 4.7e-4 / 6.6e-4 / 3.1e-3 over epochs 0-4
    (n = 3, d = 2, throttle); the GPU measured 1.4e-5 / <1e-3 / 2.1e-3 / 6.6e-3.  Trace
    bit-exact.
"""
import numpy as np
import pytest
import torch

from conftest import has_gpu

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not has_gpu(), reason="needs an MI355X")]


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
M = "vgg11_bn"


@pytest.fixture(scope="module")
def pool():
    from oracle import oracle as O
    return O.make_pool(0)


def _rel_l2(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def _run(theta_np, items, dropout, pool, n_total=4):
    """One chunk of len(items) worker-steps through flsim_vgg11_bn_fwd_bwd_chunk -> engine, S,
    losses, per-worker BatchNorm statistics."""
    from flsim.data import DevicePool
    from flsim.engine import VGG11BNEngine, worker_table
    nw = len(items)
    eng = VGG11BNEngine(DEV, chunk_workers=nw)
    dpool = DevicePool(DEV, 0, pool)
    theta = torch.from_numpy(theta_np.copy()).to(DEV)
    eng.begin_epoch(theta)
    loss = torch.zeros(nw, device=DEV)
    stats = torch.zeros(nw, eng.STATS_PER_WORKER, device=DEV)
    eng.run_chunk(theta, dpool, worker_table(items, DEV), nw, n_total, 0, dropout, loss,
                  stats_out=stats)
    S = torch.zeros(eng.P, device=DEV)
    eng.end_epoch(S)
    torch.cuda.synchronize()
    return eng, S.cpu().numpy().astype(np.float64), loss.cpu().numpy(), stats


def _is_conv_bias(name):
    """conv biases of vgg11_bn: features.{0,4,8,11,15,18,22,25}.bias (before a BatchNorm)."""
    from flsim.engine import VGG11_BN_SHAPES
    return name.endswith(".bias") and name.startswith("features.") and \
        len(dict(VGG11_BN_SHAPES)[name.replace(".bias", ".weight")]) == 4


def _check_grad(g, ref, g_cpu=None, rtol=5e-3, rtol_features=None):
    """per-tensor rel-L2 <= rtol (feature layers before the last BatchNorm: rtol_features);
    conv biases absolute (module docstring)."""
    from flsim.engine import VGG11_BN_SHAPES
    rtol_features = rtol if rtol_features is None else rtol_features
    off, worst = 0, {}
    nb_gpu = nb_cpu = 0.0
    for (name, shp) in VGG11_BN_SHAPES:
        n = int(np.prod(shp))
        a, b = g[off:off + n], ref[off:off + n]
        if _is_conv_bias(name):
            nb_gpu += float(np.sum((a - b) ** 2))
            if g_cpu is not None:
                nb_cpu += float(np.sum((g_cpu[off:off + n] - b) ** 2))
        else:
            late = name.startswith("classifier.") or name.startswith("features.26.")
            worst[name] = _rel_l2(a, b) / (rtol if late else rtol_features)
        off += n
    _tol_log(worst)
    assert max(worst.values()) <= 1.0, worst
    assert np.sqrt(nb_gpu) <= max(1e-6 * np.linalg.norm(ref), 10 * np.sqrt(nb_cpu)), \
        (np.sqrt(nb_gpu), np.sqrt(nb_cpu), np.linalg.norm(ref))


@pytest.mark.parametrize("dropout", [False, True])
def test_vgg_bn_single_worker_step_gradient_and_running(pool, dropout):
    """One worker-step: gradient vs the fp64 oracle, and the running buffers after that call
    (flsim_vgg11_bn_update_running on the call's statistics) vs nn.BatchNorm2d's."""
    from oracle import model_ref as MR
    sim = MR.OracleSim(4, delay=2, pool=pool, dropout=dropout, model=M)
    items = [(0, 0, 0)]
    g32, l32 = sim.grad_of(sim.theta, items)               # advances sim.bn by one call
    g64, l64 = sim.grad_of(sim.theta, items, dtype=torch.float64, bn=False)
    eng, g, loss, stats = _run(sim.theta, items, dropout, pool)
    assert abs(float(loss[0]) - l64[0]) <= 1e-4, (loss[0], l64[0])
    _check_grad(g, g64, g32.astype(np.float64), rtol_features=5e-2)
    eng.update_running(stats, 1)
    assert eng.num_batches_tracked == sim.bn.num_batches_tracked == 1
    got, ref = eng.running.double().cpu().numpy(), sim.bn.flat()
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("dropout,items", [
    (False, [(0, 1, 2)]), (True, [(0, 1, 2)]), (True, [(1, 0, 3), (1, 2, 0)])])
def test_vgg_bn_gradient_teacher_forced_decisions(pool, dropout, items):
    """Every backward kernel checked tightly: an fp64 reference that takes the GPU's forward
    decisions (ReLU signs, max-pool argmax, dropout masks from the workspace) and computes each
    worker's BatchNorm with fp64 batch statistics must give the GPU's gradient to fp32
    accumulation accuracy.  Two items = ONE chunk of 256 samples: each worker keeps its own
    batch statistics, and S is the sum of the per-worker gradients (agents.py:35)."""
    import torch.nn.functional as F
    from flsim.engine import VGG11_BN_SHAPES, VGG11BNEngine
    from oracle import model_ref as MR
    from test_gpu_parity import _gather_pool
    NS = 128 * len(items)
    sim = MR.OracleSim(4, delay=2, pool=pool, dropout=dropout, model=M)
    eng, g, loss, stats = _run(sim.theta, items, dropout, pool)
    ids = {name: j for j, name in enumerate(VGG11BNEngine.WORKSPACE)}

    def W(name, shp, dt=torch.float32):
        return eng.workspace_view(ids[name], shp, dt).cpu().numpy()

    def nchw(a):
        return torch.from_numpy(np.ascontiguousarray(a.transpose(0, 3, 1, 2))).double()

    A = dict(d1=nchw(W("d1", (NS, 16, 16, 64))), d2=nchw(W("d2", (NS, 8, 8, 128))),
             a3=nchw(W("a3", (NS, 8, 8, 256))), d4=nchw(W("d4", (NS, 4, 4, 256))),
             a5=nchw(W("a5", (NS, 4, 4, 512))), d6=nchw(W("d6", (NS, 2, 2, 512))),
             a7=nchw(W("a7", (NS, 2, 2, 512))), f0=torch.from_numpy(W("f0", (NS, 512))).double(),
             e1=torch.from_numpy(W("e1", (NS, 512))).double(),
             e2=torch.from_numpy(W("e2", (NS, 512))).double(),
             i1=W("i1", (NS, 16, 16, 64), torch.uint8), i2=W("i2", (NS, 8, 8, 128), torch.uint8),
             i4=W("i4", (NS, 4, 4, 256), torch.uint8), i6=W("i6", (NS, 2, 2, 512), torch.uint8),
             i8=W("i8", (NS, 1, 1, 512), torch.uint8))
    def forced(dt):
        """fp64 (or, for SURVEY 8(c), the CPU fp32 port's) forward + backward with the GPU's
        decisions and each worker's own batch statistics"""
        np_dt = np.float64 if dt == torch.float64 else np.float32
        P = [torch.tensor(a, requires_grad=True)
             for a in MR.split_flat(sim.theta.astype(np_dt), M)]
        cw, cb, gw, gb = P[0:32:4], P[1:32:4], P[2:32:4], P[3:32:4]
        l1w, l1b, l2w, l2b, l3w, l3b = P[32:]
        Ad = {k: (v.to(dt) if torch.is_tensor(v) else v) for k, v in A.items()}

        def m(t):
            return (t > 0).to(dt)

        def conv(h, j):
            z = F.conv2d(h, cw[j], cb[j], padding=1)
            return F.batch_norm(z, None, None, gw[j], gb[j], True, 0.1, 1e-5)

        s50 = 2.0 if dropout else 1.0
        lrefs = []
        for wi, it in enumerate(items):
            sl = slice(128 * wi, 128 * (wi + 1))
            a = {k: v[sl] for k, v in Ad.items()}
            x, y = sim.batch(*it, dtype=dt)
            h = _gather_pool(conv(x, 0), a["i1"]) * m(a["d1"])
            h = _gather_pool(conv(h, 1), a["i2"]) * m(a["d2"])
            h = conv(h, 2) * m(a["a3"])
            h = _gather_pool(conv(h, 3), a["i4"]) * m(a["d4"])
            h = conv(h, 4) * m(a["a5"])
            h = _gather_pool(conv(h, 5), a["i6"]) * m(a["d6"])
            h = conv(h, 6) * m(a["a7"])
            h = _gather_pool(conv(h, 7), a["i8"]).reshape(128, 512) * m(a["f0"]) * s50
            h = F.linear(h, l1w, l1b) * m(a["e1"]) * s50
            h = F.linear(h, l2w, l2b) * m(a["e2"])
            lref = F.cross_entropy(F.linear(h, l3w, l3b), y)
            lref.backward()
            lrefs.append(lref.item())
        return P, torch.cat([p.grad.reshape(-1) for p in P]).double().numpy(), lrefs

    P, ref, lrefs = forced(torch.float64)
    np.testing.assert_allclose(loss, lrefs, atol=1e-5)
    # 1.5 x the shipped build's measured worst, 4.57e-6 (features.23.weight, dropout items2;
    # profiles/r05/tol_r05j.jsonl stores it as 0.0703 of the former 6.5e-5 bound; round 4's build,
    # data gradients on the split-bf16 MFMA: 4.31e-5)
    _check_grad(g, ref, rtol=7.0e-6)
    # per tensor no farther from fp64 than 2x the CPU fp32 port (same decisions);
    # the conv biases ahead of a BatchNorm have an exact gradient of 0 (floor: the whole gradient)
    import _flips
    _, ref32, _ = forced(torch.float32)
    _flips.assert_survey(_flips.survey_ratios(
        g, ref32, ref, VGG11_BN_SHAPES,
        whole_floor={n for n, _ in VGG11_BN_SHAPES if _is_conv_bias(n)}), "vgg11_bn_teacher_forced")
    # per-worker statistics of the chunk vs each worker's own BatchNorm batch (oracle, fp64)
    st = stats.double().cpu().numpy()
    for wi, it in enumerate(items):
        bn = MR.BNState(torch.float64)
        bn.bufs = [(torch.zeros(c, dtype=torch.float64), torch.zeros(c, dtype=torch.float64))
                   for c in MR.VGG_BN_CHANNELS]
        x, _ = sim.batch(*it, dtype=torch.float64)
        noise = MR.dropout_noise(0, it[0], it[1], 128, torch.float64, M) if dropout else None
        with torch.no_grad():
            MR.vgg_bn_forward([p.detach() for p in P], x, noise, bn)
        # momentum 0.1 from zero buffers: running = 0.1 * stat
        np.testing.assert_allclose(st[wi], bn.flat() / 0.1, rtol=2e-4, atol=2e-5)


def test_vgg_bn_simulation_matches_oracle_trajectory(pool):
    """The batched server loop with vgg11_bn against the oracle loop: bit-exact staleness trace,
    losses within the fp32 tolerance, running buffers advanced over every computing worker."""
    from flsim.sim import FLSimulation
    from oracle import model_ref as MR
    n, d, ep = 3, 2, 4
    osim = MR.OracleSim(n, delay=d, throttle=True, pool=pool, model=M)
    gsim = FLSimulation(n, delay=d, throttle=True, device=DEV, chunk_workers=2, pool=pool, model=M)
    assert np.array_equal(gsim.theta.cpu().numpy(), osim.theta)
    for t in range(ep):
        lo = osim.epoch()
        lg = gsim.epoch()
        tr_o = osim.trace[-1]
        plan = gsim.trace[-1]
        assert [i for (_, i, _) in tr_o["items"]] == list(np.nonzero(plan.computes)[0])
        assert [s for (k, s) in tr_o["appended"] if k == "stale"] == [s for (_, s) in plan.stale]
        assert abs(lg - lo) <= (1e-4, 2e-3, 5e-3, 1e-2)[t], (t, lg, lo)
        if t == 0:      # every call of epoch 0 ran on theta_0: the buffers agree tightly
            np.testing.assert_allclose(gsim.engine.running.double().cpu().numpy(),
                                       osim.bn.flat(), rtol=1e-5, atol=1e-6)
    assert gsim.engine.num_batches_tracked == osim.bn.num_batches_tracked
    # after several epochs the buffers follow two (legitimately) different trajectories --
    # statistical agreement only (Adam's first steps move every weight by ~lr whatever the
    # gradient's size, i.e. ~5 % of a VGG conv weight's init std, in the direction of sign(g)): the
    # conv biases (noise-driven, +-lr per Adam step, see _check_running) enter running_mean
    # directly, and the weights differ at the trajectory tolerance.  The per-call update itself
    # is checked at 1e-5 (single-step and facade tests, tests/test_oracle_golden).
    # calibration: the oracle's own fp32 vs fp64-gradient runs differ by rel-L2 5e-8 / 8e-5 /
    # 4.4e-3 / 1.0e-2 in the buffers after epochs 0-3 (theta: 4e-4 ... 5.3e-3); GPU: 2.2e-2
    assert _rel_l2(gsim.engine.running.double().cpu().numpy(), osim.bn.flat()) < 5e-2
    # the state dict loads into the models.py module (main.py:98-100 / 192-194 round trip)
    from FL.models import vgg11_bn
    sd = gsim.model_state_dict()
    mod = vgg11_bn()
    mod.load_state_dict(sd)
    assert list(sd.keys()) == list(mod.state_dict().keys())
    assert int(mod.features[1].num_batches_tracked) == osim.bn.num_batches_tracked


def test_vgg_bn_eval_predictions_match_oracle(pool):
    """Device evaluation in eval mode (util.py:31-45: BatchNorm with the running buffers, dropout
    off) vs the oracle's fp32 forward over a ragged 600-image range; near-ties only."""
    from flsim.data import DevicePool, make_test_pool
    from flsim.engine import VGG11BNEngine
    from oracle import model_ref as MR
    theta = MR.init_params(0, M)
    rs = np.random.RandomState(3)
    run = np.concatenate([np.concatenate([rs.normal(0, 0.3, c), rs.uniform(0.5, 2.0, c)])
                          for c in MR.VGG_BN_CHANNELS]).astype(np.float32)
    test = make_test_pool(0, size=600)
    eng = VGG11BNEngine(DEV, chunk_workers=2)
    eng.running.copy_(torch.from_numpy(run))
    pred = eng.evaluate(torch.from_numpy(theta).to(DEV), DevicePool(DEV, 0, test)).cpu().numpy()
    ref = MR.predict(theta, test[0], model=M, bn=run)
    assert (pred == ref).mean() >= 0.99, (pred != ref).sum()


def test_vgg_bn_reference_api_facade(pool):
    """FL.agents drop-in with the reference's vgg11_bn module: Worker.fwd_bkwd per worker, the
    module's running buffers advanced per call, Agg(rule), Central.update_model -- one epoch."""
    import torch.nn as nn
    from FL.agents import Agg, Central, Worker, rule
    from FL.models import vgg11_bn
    from oracle import model_ref as MR
    from oracle import oracle as O
    n = 3
    osim = MR.OracleSim(n, delay=2, throttle=False, pool=pool, model=M)
    torch.manual_seed(0)
    model = vgg11_bn().to(DEV)
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
        if i < n - 1:
            ups.append(g)
            losses.append(lv)
    central.update_model(Agg(rule).rule(ups))
    lo = osim.epoch()
    assert abs(float(np.mean(losses)) - lo) <= 1e-4, (np.mean(losses), lo)
    assert int(model.features[1].num_batches_tracked) == n
    run = torch.cat([torch.cat([mod.running_mean, mod.running_var]) for mod in model.modules()
                     if isinstance(mod, nn.BatchNorm2d)]).double().cpu().numpy()
    np.testing.assert_allclose(run, osim.bn.flat(), rtol=1e-5, atol=1e-6)


def _bn_facade_loop(pool, monkeypatch, lazy, n=6):
    """One epoch of the reference worker loop through FL.agents with vgg11_bn: chunks of 4 staged
    calls, the running buffers read after call 3 (mid-chunk) and at the epoch's end."""
    import torch.nn as nn
    from FL.agents import Agg, Central, Worker, rule
    from FL.models import vgg11_bn
    from oracle import oracle as O
    monkeypatch.setenv("FLSIM_FACADE_CHUNK", "4")
    monkeypatch.setenv("FLSIM_FACADE_LAZY_LOSS", "1" if lazy else "0")
    torch.manual_seed(0)
    model = vgg11_bn().to(DEV)
    central = Central(model, torch.optim.Adam(model.parameters(), lr=0.001))
    workers = [Worker(nn.CrossEntropyLoss()) for _ in range(n)]
    rs = np.random.RandomState(11)
    lut = O.normalize_lut()
    model.train()
    ups, losses, mids = [], [], None
    bn = [m for m in model.modules() if isinstance(m, torch.nn.BatchNorm2d)]
    for i in range(n):
        idx = rs.randint(0, pool[0].shape[0], 128)
        workers[i].model = central.model
        g, lv = workers[i].fwd_bkwd(torch.from_numpy(lut[pool[0][idx]]).to(DEV),
                                    torch.from_numpy(pool[1][idx]).to(DEV))
        ups.append(g)
        losses.append(lv)
        if i == 2:
            mids = (torch.cat([bn[0].running_mean.cpu(), bn[-1].running_var.cpu()]),
                    int(bn[3].num_batches_tracked))
    grad = torch.cat([t.reshape(-1) for t in ups[0]]).double().cpu()
    central.update_model(Agg(rule).rule(ups))
    mean = np.mean(losses)
    sd = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()
          if "running" in k or "num_batches" in k}
    return np.asarray([float(v) for v in losses], np.float32), mean, grad, sd, mids


def test_vgg_bn_facade_lazy_matches_per_call(pool, monkeypatch):
    """vgg11_bn through the facade with staged calls (one batched forward + backward per chunk of
    4, each call its own BatchNorm batch, the running updates folded in call order at the flush;
    the module's buffers are lazy views that run the staged calls when read) against a forward and
    backward per call: losses, running buffers read mid-chunk and after the epoch, and
    num_batches_tracked agree, the gradient within the order of the calls' partial sums."""
    la, ma, ga, sa, mida = _bn_facade_loop(pool, monkeypatch, lazy=False)
    lb, mb, gb, sb, midb = _bn_facade_loop(pool, monkeypatch, lazy=True)
    np.testing.assert_allclose(lb, la, rtol=2e-6)
    assert mb.dtype == np.float32 and abs(float(mb) - float(ma)) <= 2e-6 * abs(float(ma))
    assert midb[1] == mida[1] == 3
    torch.testing.assert_close(midb[0], mida[0], rtol=2e-6, atol=1e-7)
    assert sa.keys() == sb.keys()
    for k in sa:
        if "num_batches" in k:
            assert int(sa[k]) == int(sb[k]) == 6, k
        else:
            torch.testing.assert_close(sb[k], sa[k], rtol=2e-6, atol=1e-7)
    assert float((ga - gb).norm() / ga.norm()) <= 1e-5
