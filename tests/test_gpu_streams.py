"""GPU: the stream-level scheduling of round 3 changes no result.

  * FLSimulation with pipelined chunks (flsim_pn1_fwd_bwd_chunk_async: chunk i's forward beside
    chunk i-1's backward, two workspaces) against the synchronous chunks: losses, theta, m and v
    bit for bit, for small chunks (weight gradients also on the side stream) and 32-worker ones;
  * the FL.agents facade with the pipelined fwd_bkwd (flsim_pn1_fwd_bwd_input_async) against the
    synchronous one: the same per-call losses, the same .grad values read between calls (the lazy
    views join the backward stream), the same parameters after update_model (main.py:126-188);
  * the facade's deferred backward (flsim_pn1_fwd_rows / bwd_rows: each call's forward alone,
    one batched backward per chunk of calls) against the per-call backward -- the same per-call
    losses bit for bit, parameters within fp32 tolerance -- and against FLSimulation running the
    same epochs: bit for bit when an epoch's calls form one chunk in both.
"""
import numpy as np
import pytest
import torch
import torch.nn as nn

from conftest import has_gpu

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not has_gpu(), reason="needs an MI355X")]

DEV = "cuda:0"


@pytest.fixture(scope="module")
def pool():
    from oracle import oracle as O
    return O.make_pool(0)


@pytest.mark.parametrize("n,chunk", [(8, 2), (96, 32)])
def test_pipelined_chunks_match_sync(pool, n, chunk):
    from flsim.sim import FLSimulation
    kw = dict(delay=2, throttle=False, device=DEV, pool=pool, chunk_workers=chunk)
    a = FLSimulation(n, **kw)
    a.pipeline = False
    b = FLSimulation(n, **kw)
    b.pipeline = True
    assert len(b.chunks(0, n)) > 1
    for t in range(3):
        la, lb = a.epoch(), b.epoch()
        assert la == lb, (t, la, lb)
    for name in ("theta", "m", "v"):
        assert torch.equal(getattr(a, name), getattr(b, name)), name
    wa = a.comm[a.Ppad:a.Ppad + n].cpu()
    wb = b.comm[b.Ppad:b.Ppad + n].cpu()
    assert torch.equal(wa, wb)


def _loop(pool, pipeline, epochs=2, n=4, read_grads=False, defer="0"):
    """The reference's loop (main.py:126-188 without the slow worker) through FL.agents.
    defer: FLSIM_FACADE_CHUNK ("0": a backward per call, pipelined or not)."""
    import os
    from FL.agents import Agg, Central, Worker, rule
    from FL.models import PerformantNet1
    from oracle import oracle as O
    torch.manual_seed(0)
    model = PerformantNet1().to(DEV)
    old = os.environ.get("FLSIM_FACADE_CHUNK")
    os.environ["FLSIM_FACADE_CHUNK"] = defer
    try:
        central = Central(model, torch.optim.Adam(model.parameters(), lr=0.001))
    finally:
        if old is None:
            del os.environ["FLSIM_FACADE_CHUNK"]
        else:
            os.environ["FLSIM_FACADE_CHUNK"] = old
    central.ctx.pipeline = pipeline
    workers = [Worker(nn.CrossEntropyLoss()) for _ in range(n)]
    agg = Agg(rule)
    rs = np.random.RandomState(5)
    losses, grads = [], []
    for t in range(epochs):
        ups_all = []
        model.train()
        for i in range(n):
            idx = rs.randint(0, pool[0].shape[0], 128)
            x = torch.from_numpy(O.normalize_lut()[pool[0][idx]]).to(DEV)
            y = torch.from_numpy(pool[1][idx]).to(DEV)
            workers[i].model = central.model
            ups, lv = workers[i].fwd_bkwd(x, y)
            losses.append(float(lv))
            if read_grads and i == 1:        # a read between calls: the accumulated .grad
                grads.append(torch.cat([g.reshape(-1) for g in ups]).cpu())
            ups_all.append(ups)
        central.update_model(agg.rule(ups_all))
    return central.ctx, losses, grads


@pytest.mark.parametrize("read_grads", [False, True])
def test_facade_pipelined_matches_sync(pool, read_grads):
    ca, la, ga = _loop(pool, False, read_grads=read_grads)
    cb, lb, gb = _loop(pool, True, read_grads=read_grads)
    assert la == lb
    for x, y in zip(ga, gb):
        assert torch.equal(x, y)
    for name in ("theta", "m", "v"):
        assert torch.equal(getattr(ca, name), getattr(cb, name)), name


@pytest.mark.parametrize("read_grads", [False, True])
def test_facade_deferred_backward(pool, read_grads):
    """Deferred chunk backward vs a backward per call: the forwards are the same kernels on the
    same rows (losses bit-identical); the gradient differs only in summation order."""
    ca, la, ga = _loop(pool, True, read_grads=read_grads, defer="0")
    cb, lb, gb = _loop(pool, True, read_grads=read_grads, defer="128")
    assert la == lb
    for t, (x, y) in enumerate(zip(ga, gb)):
        x, y = x.double(), y.double()
        # epoch 0: the same theta, only the summation order differs (arithmetic, ~1e-7);
        # epoch 1: theta after one Adam step can differ by +-2 lr where a gradient component is
        # ~0 (its sign decides), which moves the next gradient further
        assert float((x - y).norm() / y.norm()) < (1e-6 if t == 0 else 1e-3), t
    a, b = ca.theta[:ca.P].double(), cb.theta[:cb.P].double()
    # two Adam steps: a near-zero gradient component can move by ~2 lr either way
    assert float((a - b).abs().max()) <= 4.1e-3
    assert float((a - b).norm() / b.norm()) < 1e-2


def test_deferred_facade_equals_simulation(pool, monkeypatch):
    """main.py:126-188 through FL.agents (deferred backward) and FLSimulation on the same data,
    dropout keys and schedule (n = 6, d = 3, throttle, 5 epochs): every epoch's calls form one
    deferred chunk and one FLSimulation chunk, so per-worker losses and theta / m / v after every
    epoch agree bit for bit -- the drop-in API runs the batched engine's own arithmetic."""
    from FL.agents import Agg, Central, Worker, rule
    from FL.models import PerformantNet1
    from flsim.sim import FLSimulation
    from oracle import oracle as O
    monkeypatch.setenv("FLSIM_FACADE_CHUNK", "8")
    n, d, ep = 6, 3, 5
    sim = FLSimulation(n, delay=d, throttle=True, device=DEV, pool=pool, chunk_workers=8)
    torch.manual_seed(0)
    model = PerformantNet1().to(DEV)
    central = Central(model, torch.optim.Adam(model.parameters(), lr=0.001))
    ctx = central.ctx
    assert torch.equal(ctx.theta[:ctx.P], sim.theta[:sim.P])
    workers = [Worker(nn.CrossEntropyLoss()) for _ in range(n)]
    agg = Agg(rule)
    rs = np.random.RandomState(0)
    lists = O.class_lists(pool[1])
    lut = O.normalize_lut()
    pesky, window, gone = [], 0, False
    for t in range(ep):
        sim.epoch()
        ks = rs.randint(0, n, size=n)
        weight_ups, call_losses = [], []
        model.train()
        for i in range(n):
            idx = O.batch_indices(0, t, i, int(ks[i]), n, lists)
            x = torch.from_numpy(lut[pool[0][idx]]).to(DEV)
            y = torch.from_numpy(pool[1][idx]).to(DEV)
            if i == n - 1:
                gone = False
                ups = None
                if t == 0 or t % d == 0:
                    workers[i].model = central.model
                    ups, lv = workers[i].fwd_bkwd(x, y)
                    call_losses.append(lv)
                    pesky.append(ups)
                    ups = pesky.pop(0) if t > 0 else None
                if ups is not None:
                    weight_ups.append(ups)
                    gone = True
            elif window <= 0:
                workers[i].model = central.model
                ups, lv = workers[i].fwd_bkwd(x, y)
                call_losses.append(lv)
                weight_ups.append(ups)
                window = 1 if gone else 2
            if window > 0:
                window -= 1
        central.update_model(agg.rule(weight_ups))
        got = np.asarray([float(v) for v in call_losses], np.float32)
        ref = sim.comm[sim.Ppad:sim.Ppad + len(got)].cpu().numpy()
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), (t, got, ref)
        for name in ("theta", "m", "v"):
            a = getattr(ctx, name)[:ctx.P]
            b = getattr(sim, name)[:sim.P]
            assert torch.equal(a, b), (t, name, int((a != b).sum()))


def _lazy_loop(pool, monkeypatch, lazy, n=20, epochs=2):
    """main.py:126-188's worker loop through FL.agents with losses kept as returned and read
    only by np.mean at the epoch's end (main.py:181); deferred chunks of 8 calls, one call of 64
    samples (worker 5: a one-call forward between staged blocks) and one .grad read mid-epoch
    (worker 11 of epoch 1: the staged forwards and the pending backward run there)."""
    from FL.agents import Agg, Central, Worker, rule
    from FL.models import PerformantNet1
    from oracle import oracle as O
    monkeypatch.setenv("FLSIM_FACADE_CHUNK", "8")
    monkeypatch.setenv("FLSIM_FACADE_LAZY_LOSS", "1" if lazy else "0")
    torch.manual_seed(0)
    model = PerformantNet1().to(DEV)
    central = Central(model, torch.optim.Adam(model.parameters(), lr=0.001))
    workers = [Worker(nn.CrossEntropyLoss()) for _ in range(n)]
    agg = Agg(rule)
    rs = np.random.RandomState(3)
    lut = O.normalize_lut()
    means, all_losses, reads = [], [], []
    for t in range(epochs):
        ups_all, losses = [], []
        model.train()
        for i in range(n):
            b = 64 if i == 5 else 128
            idx = rs.randint(0, pool[0].shape[0], b)
            x = torch.from_numpy(lut[pool[0][idx]]).to(DEV)
            y = torch.from_numpy(pool[1][idx]).to(DEV)
            workers[i].model = central.model
            ups, lv = workers[i].fwd_bkwd(x, y)
            losses.append(lv)
            ups_all.append(ups)
            if t == 1 and i == 11:
                reads.append(torch.cat([g.reshape(-1) for g in ups]).cpu())
        central.update_model(agg.rule(ups_all))
        means.append(np.mean(losses))
        all_losses.append(np.asarray([float(v) for v in losses], np.float32))
    return central.ctx, means, all_losses, reads


def test_facade_lazy_loss_matches_eager(pool, monkeypatch):
    """The deferred forward (128-sample calls staged, one batched forward per block of calls,
    _LazyLoss returned) against every call running its forward at once: per-call losses, the
    epoch's np.mean (float32, as the reference's), a .grad read mid-epoch and theta / m / v after
    each update bit for bit -- the batched forward's sums per output are the one-call forward's."""
    ca, ma, la, ra = _lazy_loop(pool, monkeypatch, lazy=False)
    cb, mb, lb, rb = _lazy_loop(pool, monkeypatch, lazy=True)
    for t, (x, y) in enumerate(zip(la, lb)):
        assert np.array_equal(x.view(np.uint32), y.view(np.uint32)), (t, x, y)
    for x, y in zip(ma, mb):
        assert isinstance(y, np.floating) and y.dtype == np.float32 and x.dtype == y.dtype
        assert x == y
    for x, y in zip(ra, rb):
        assert torch.equal(x, y)
    for name in ("theta", "m", "v"):
        assert torch.equal(getattr(ca, name), getattr(cb, name)), name
