"""GPU: the stream-level scheduling of round 3 changes no result.

  * FLSimulation with pipelined chunks (flsim_pn1_fwd_bwd_chunk_async: chunk i's forward beside
    chunk i-1's backward, two workspaces) against the synchronous chunks: losses, theta, m and v
    bit for bit, for small chunks (weight gradients also on the side stream) and 32-worker ones;
  * the FL.agents facade with the pipelined fwd_bkwd (flsim_pn1_fwd_bwd_input_async) against the
    synchronous one: the same per-call losses, the same .grad values read between calls (the lazy
    views join the backward stream), the same parameters after update_model (main.py:126-188).
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


def _loop(pool, pipeline, epochs=2, n=4, read_grads=False):
    """The reference's loop (main.py:126-188 without the slow worker) through FL.agents."""
    from FL.agents import Agg, Central, Worker, rule
    from FL.models import PerformantNet1
    from oracle import oracle as O
    torch.manual_seed(0)
    model = PerformantNet1().to(DEV)
    central = Central(model, torch.optim.Adam(model.parameters(), lr=0.001))
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
