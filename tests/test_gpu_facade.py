"""GPU: the drop-in Python API (FL/agents.py, FL/util.py) against the CPU oracle.

  * Worker.fwd_bkwd with --batch_size other than 128 (main.py:43-44): CrossEntropyLoss's mean
    over the n samples, padding groups that add nothing, per-group dropout keys;
  * batches of different sizes in one epoch (the engine grows mid-epoch and keeps the gradient);
  * Central.update_model with stale entries interleaved among the fresh ones (several slow
    workers): bit-exact with the oracle's cascade + Adam;
  * the reference's loop (main.py:126-188) written against FL.agents with `from FL.util import *`
    and print_test_accuracy (util.py:31-45) on the device;
  * a CIFAR-10-binary-format pool (main.py:65-91 from a local copy) through the HIP path.
"""
import numpy as np
import pytest
import torch
import torch.nn as nn

from conftest import has_gpu

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not has_gpu(), reason="needs an MI355X")]

DEV = "cuda:0"
GROUP = 1 << 20


@pytest.fixture(scope="module")
def pool():
    from oracle import oracle as O
    return O.make_pool(0)


def _rel_l2(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def _fresh_central(seed=0):
    from FL.agents import Central
    from FL.models import PerformantNet1
    torch.manual_seed(seed)
    model = PerformantNet1().to(DEV)
    opt = torch.optim.Adam(model.parameters(), lr=0.001)
    return model, Central(model, opt)


def _batch(pool, n, seed):
    from oracle import oracle as O
    rs = np.random.RandomState(seed)
    idx = rs.randint(0, pool[0].shape[0], n)
    x = O.normalize_lut()[pool[0][idx]]
    return torch.from_numpy(x), torch.from_numpy(pool[1][idx])


def _oracle_grad(theta, batches, dtype):
    """Sum over batches [(x, y, worker index, epoch)] of the mean-CE gradient (agents.py:35),
    dropout masks by the facade's key rule (group b of worker i: i + b * 2^20)."""
    from oracle import model_ref as MR
    params = [torch.tensor(a, dtype=dtype, requires_grad=True)
              for a in MR.split_flat(theta.astype(np.float64 if dtype == torch.float64
                                                  else np.float32))]
    losses = []
    for x, y, i, t in batches:
        n = x.shape[0]
        groups = -(-n // 128)
        per = [MR.dropout_noise(0, t, i + b * GROUP, 128, dtype) for b in range(groups)]
        noise = [torch.cat([p[s] for p in per])[:n] for s in range(len(per[0]))]
        losses.append(float(MR.fwd_bkwd(params, x.to(dtype), y, noise)))
    return torch.cat([p.grad.reshape(-1) for p in params]).numpy().astype(np.float64), losses


def _check_facade_step(g_gpu, model, x, y, keys, theta, n):
    """Arithmetic (teacher forced) and decision checks of one fwd_bkwd call (tests/_flips.py)."""
    import _flips
    from FL.agents import _context
    eng = _context(model).engine
    noise = _flips.noise_groups(keys, n)
    return _flips.check_worker_step(g_gpu, eng, theta, x, y, noise, 1.0 / n)


@pytest.mark.parametrize("n", [100, 256])
def test_worker_batch_sizes_match_oracle(pool, n):
    from FL.agents import Worker
    from oracle import model_ref as MR
    model, central = _fresh_central()
    w = Worker(nn.CrossEntropyLoss())
    assert w.index == 0
    model.train()
    w.model = model
    x, y = _batch(pool, n, n)
    grads, loss = w.fwd_bkwd(x.to(DEV), y.to(DEV))
    theta = MR.init_params(0)
    g64, l64 = _oracle_grad(theta, [(x, y, 0, 0)], torch.float64)
    g = torch.cat([t.reshape(-1) for t in grads]).cpu().numpy().astype(np.float64)
    assert abs(float(loss) - l64[0]) <= 1e-4, (float(loss), l64[0])
    keys = [(0, 0 + b * GROUP) for b in range(-(-n // 128))]
    _check_facade_step(g, model, x, y, keys, theta, n)


def test_mixed_batch_sizes_in_one_epoch(pool, monkeypatch):
    """A 128-sample then a 256-sample batch in the same epoch: the engine (a deferred chunk of one
    128-sample group, FLSIM_FACADE_CHUNK=1) grows between the calls and the epoch's gradient
    keeps both (agents.py:35 keeps accumulating into .grad)."""
    from FL.agents import Worker
    from oracle import model_ref as MR
    monkeypatch.setenv("FLSIM_FACADE_CHUNK", "1")
    model, central = _fresh_central()
    ws = [Worker(nn.CrossEntropyLoss()) for _ in range(2)]
    model.train()
    theta = MR.init_params(0)
    xa, ya = _batch(pool, 128, 1)
    xb, yb = _batch(pool, 256, 2)
    ws[0].model = model
    grads, _ = ws[0].fwd_bkwd(xa.to(DEV), ya.to(DEV))
    ga = torch.cat([t.reshape(-1) for t in grads]).cpu().numpy().astype(np.float64)
    _check_facade_step(ga, model, xa, ya, [(0, 0)], theta, 128)
    ws[1].model = model
    grads, _ = ws[1].fwd_bkwd(xb.to(DEV), yb.to(DEV))
    gab = torch.cat([t.reshape(-1) for t in grads]).cpu().numpy().astype(np.float64)
    _check_facade_step(gab - ga, model, xb, yb, [(0, 1), (0, 1 + GROUP)], theta, 256)
    g64, _ = _oracle_grad(theta, [(xa, ya, 0, 0), (xb, yb, 1, 0)], torch.float64)
    assert _rel_l2(gab, g64) <= 1e-2
    assert all(p.grad.data_ptr() == t.data_ptr() for p, t in zip(model.parameters(), grads))


def test_mixed_batch_sizes_untouched_grads(pool, monkeypatch):
    """The same two calls with no .grad read in between: the engine grows while the
    128-sample call is still a deferred forward (its backward not run).  The epoch's gradient
    read after the second call equals the one read with a flush between the calls, bit for bit."""
    from FL.agents import Worker
    monkeypatch.setenv("FLSIM_FACADE_CHUNK", "1")

    def run(read_between):
        model, central = _fresh_central()
        ws = [Worker(nn.CrossEntropyLoss()) for _ in range(2)]
        model.train()
        xa, ya = _batch(pool, 128, 1)
        xb, yb = _batch(pool, 256, 2)
        ws[0].model = model
        grads, _ = ws[0].fwd_bkwd(xa.to(DEV), ya.to(DEV))
        if read_between:
            float(grads[0].sum())
        ws[1].model = model
        grads, _ = ws[1].fwd_bkwd(xb.to(DEV), yb.to(DEV))
        return torch.cat([t.reshape(-1) for t in grads]).cpu().numpy()

    g_read, g_untouched = run(True), run(False)
    assert np.abs(g_read).max() > 0
    assert np.array_equal(g_read.view(np.uint32), g_untouched.view(np.uint32))


def test_interleaved_stale_entries_update_model(pool):
    """weight_ups = [fresh, stale(t=0), fresh, stale(t=0), fresh] in worker order (two slow
    workers popping the same epoch): Central.update_model == the oracle's cascade + Adam, bit
    for bit (main.py:23-25 over the entries in append order, agents.py:9-21)."""
    from FL.agents import Agg, Worker, rule
    from flsim.engine import PN1_SIZES
    from oracle import oracle as O
    model, central = _fresh_central()
    ws = [Worker(nn.CrossEntropyLoss()) for _ in range(3)]
    agg = Agg(rule)
    model.train()
    ups0 = None
    for i, w in enumerate(ws):                     # epoch 0
        w.model = model
        x, y = _batch(pool, 128, 10 + i)
        ups0, _ = w.fwd_bkwd(x.to(DEV), y.to(DEV))
    central.update_model(agg.rule([ups0, ups0]))
    S0 = torch.cat([t.reshape(-1) for t in ups0]).cpu().numpy()
    ups1 = None
    for i, w in enumerate(ws):                     # epoch 1
        x, y = _batch(pool, 128, 20 + i)
        ups1, _ = w.fwd_bkwd(x.to(DEV), y.to(DEV))
    S1 = torch.cat([t.reshape(-1) for t in ups1]).cpu().numpy()
    ctx = central.ctx
    p = ctx.theta[:ctx.P].cpu().numpy().copy()
    m = ctx.m[:ctx.P].cpu().numpy().copy()
    v = ctx.v[:ctx.P].cpu().numpy().copy()
    entries = [ups1, ups0, ups1, ups0, ups1]
    central.update_model(agg.rule(entries))
    g = np.empty_like(S1)
    off = 0
    for n in PN1_SIZES:
        g[off:off + n] = O.cascade_mean([e[off:off + n] for e in (S1, S0, S1, S0, S1)])
        off += n
    O.adam_step(p, m, v, g, 2)
    for name, a, b in (("p", ctx.theta, p), ("m", ctx.m, m), ("v", ctx.v, v)):
        got = a[:ctx.P].cpu().numpy()
        assert np.array_equal(got.view(np.uint32), b.view(np.uint32)), name


def test_reference_loop_with_fl_util(pool):
    """main.py:126-188's loop structure (one slow worker, throttle, the stale FIFO) written
    against FL.agents, then main.py:196-203's evaluation through `from FL.util import *`:
    losses track the oracle, print_test_accuracy returns the accuracy of the oracle's
    predictions on the same test batches (util.py:45 returns a scalar)."""
    from FL.agents import Agg, Worker, rule
    from oracle import model_ref as MR
    from oracle import oracle as O
    ns = {}
    exec("from FL.util import *", ns)
    print_test_accuracy = ns["print_test_accuracy"]
    n, d, ep = 4, 2, 4
    osim = MR.OracleSim(n, delay=d, throttle=True, pool=pool)
    model, central = _fresh_central()
    workers = [Worker(nn.CrossEntropyLoss()) for _ in range(n)]
    assert [w.index for w in workers] == list(range(n))
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
                if t == 0 or t % d == 0:
                    workers[i].model = central.model
                    ups, _ = workers[i].fwd_bkwd(x, y)
                    pesky.append(ups)
                    ups = pesky.pop(0) if t > 0 else None
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
        central.update_model(agg.rule(weight_ups))
        lo = osim.epoch()
        assert abs(float(np.mean(losses)) - lo) <= (1e-4 if t == 0 else 1e-3), (t, lo)
    model.eval()
    test_x, test_y = O.make_test_pool(0, size=1000)
    xs = torch.from_numpy(lut[test_x])
    loader = [(xs[j:j + 128], torch.from_numpy(test_y[j:j + 128])) for j in range(0, 1000, 128)]
    acc = print_test_accuracy(model, loader)
    assert isinstance(acc, float)
    th = torch.cat([p.detach().reshape(-1) for p in model.parameters()]).cpu().numpy()
    ref = MR.predict(th, test_x)
    assert abs(acc - 100.0 * float((ref == test_y).mean())) <= 0.5


def test_cifar10_binary_pool_through_hip_path(pool, tmp_path):
    """A pool read from CIFAR-10 binary batches (load_cifar10_bin, main.py:70-73 from a local
    copy) goes through the device draw + HIP fwd/bwd and an FL epoch like the synthetic pool."""
    from flsim.data import DevicePool, load_cifar10_bin
    from flsim.engine import PN1Engine, worker_table
    from flsim.sim import FLSimulation
    from oracle import model_ref as MR
    rs = np.random.RandomState(5)
    for name, nrec in [(f"data_batch_{i}.bin", 400) for i in range(1, 6)] + [("test_batch.bin", 200)]:
        lab = rs.randint(0, 10, nrec).astype(np.uint8)
        proto = pool[0][lab.astype(np.int64) * 7]            # image-like pixels
        img = np.clip(proto.reshape(nrec, -1).astype(np.int16) +
                      rs.randint(-20, 21, (nrec, 3072)), 0, 255).astype(np.uint8)
        (tmp_path / name).write_bytes(np.concatenate([lab[:, None], img], 1).tobytes())
    (tr_x, tr_y), (te_x, te_y) = load_cifar10_bin(str(tmp_path))
    cpool = (tr_x, tr_y)
    osim = MR.OracleSim(4, delay=2, pool=cpool)
    items = [(0, 0, 1), (0, 3, 3)]
    g64, l64 = osim.grad_of(osim.theta, items, dtype=torch.float64)
    eng = PN1Engine(DEV, chunk_workers=2)
    dpool = DevicePool(DEV, 0, cpool)
    theta = torch.from_numpy(osim.theta.copy()).to(DEV)
    eng.begin_epoch(theta)
    loss = torch.zeros(2, device=DEV)
    eng.run_chunk(theta, dpool, worker_table(items, DEV), 2, 4, 0, True, loss)
    S = torch.zeros(eng.P, device=DEV)
    eng.end_epoch(S)
    np.testing.assert_allclose(loss.cpu().numpy(), l64, atol=1e-4)
    import _flips
    xs, ys = zip(*[osim.batch(*it, dtype=torch.float64) for it in items])
    _flips.check_worker_step(S.cpu().numpy().astype(np.float64), eng, osim.theta,
                             torch.cat(xs), torch.cat(ys),
                             _flips.noise_groups([(0, 0), (0, 3)], 256), 1.0 / 128)
    sim = FLSimulation(4, delay=2, throttle=True, device=DEV, chunk_workers=2, pool=cpool,
                       test_pool=(te_x, te_y))
    o2 = MR.OracleSim(4, delay=2, throttle=True, pool=cpool)
    for t in range(3):
        assert abs(sim.epoch() - o2.epoch()) <= (1e-4 if t == 0 else 1e-3)
    acc, per = sim.evaluate()
    assert 0.0 <= acc <= 100.0 and len(per) == 10


@pytest.mark.parametrize("defer", ["0", "128"])
def test_two_calls_teacher_forced(pool, monkeypatch, defer):
    """Two 128-sample fwd_bkwd calls, then a .grad read (agents.py:35 accumulation of both): with
    the deferred backward (FLSIM_FACADE_CHUNK=128: one 256-row backward pass) and with a backward
    per call (0), the epoch's gradient meets the teacher-forced fp64 checks and SURVEY 8(c) per
    tensor (tests/_flips.py) on the two calls' own forward decisions."""
    import _flips
    from FL.agents import Worker
    from oracle import model_ref as MR
    monkeypatch.setenv("FLSIM_FACADE_CHUNK", defer)
    model, central = _fresh_central()
    ws = [Worker(nn.CrossEntropyLoss()) for _ in range(2)]
    model.train()
    theta = MR.init_params(0)
    xs, ys, dec = [], [], []
    grads = None
    for i, w in enumerate(ws):
        x, y = _batch(pool, 128, 40 + i)
        w.model = model
        grads, _ = w.fwd_bkwd(x.to(DEV), y.to(DEV))
        xs.append(x)
        ys.append(y)
        if defer == "0":      # per call: each call's forward decisions are in its own workspace
            dec.append(_flips.gpu_decisions(central.ctx.engine, 128))
    g = torch.cat([t.reshape(-1) for t in grads]).cpu().numpy().astype(np.float64)
    x, y = torch.cat(xs), torch.cat(ys)
    noise = _flips.noise_groups([(0, 0), (0, 1)], 256)
    if defer == "0":
        forced = {k: torch.cat([dec[0][k], dec[1][k]]) for k in dec[0]}
        monkeypatch.setattr(_flips, "gpu_decisions", lambda eng, n, rows=None: forced)
    _flips.check_worker_step(g, central.ctx.engine, theta, x, y, noise, 1.0 / 128)
