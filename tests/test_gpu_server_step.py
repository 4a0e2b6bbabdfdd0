"""GPU: the server step kernels (csrc/server.hip).

  k_slab_step   world = 1: the epoch's weight-gradient slabs -> S_t [-> the FIFO slot] -> rule()
                + Adam in one launch (flsim_<net>_server_step)
  k_agg_stream  rule() + Adam from S_t in a buffer (after the all-reduce at world > 1; facade)

Both follow the same host-built cascade program (csrc/cascade.h, checked bit for bit against the
oracle on the CPU by tests/test_cascade_program.py).  Here: the fused kernel equals end_epoch +
the streaming kernel bit for bit (every rule form, all three networks), the streaming kernel
equals the oracle bit for bit, and a fused simulation equals an unfused one bit for bit.
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


def _filled_engine(cls, pool, items, n_total=8):
    from flsim.data import DevicePool
    from flsim.sim import default_theta
    from flsim.engine import worker_table
    eng = cls(DEV, chunk_workers=len(items))
    theta = default_theta(0, eng.MODEL).to(DEV)
    dpool = DevicePool(DEV, 0, pool)
    eng.begin_epoch(theta)
    loss = torch.zeros(len(items), device=DEV)
    kw = {"stats_out": torch.zeros(len(items), eng.STATS_PER_WORKER, device=DEV)} \
        if eng.STATS_PER_WORKER else {}
    eng.run_chunk(theta, dpool, worker_table(items, DEV), len(items), n_total, 0, True, loss, **kw)
    return eng, theta


def _rules(P, stager):
    from flsim.engine import Rule
    g = torch.Generator(device="cpu").manual_seed(3)
    arrs = [(torch.randn(P + 64, generator=g) * 1e-3).to(DEV) for _ in range(3)]
    return {
        "reference_tick": Rule(6, [arrs[0]], c=5),
        "reference_plain": Rule(9, [], c=9),
        "torch1_zero_stale": Rule(4, [None], c=3),
        "independent_sum": Rule(7, [], c=1),
        "general_order": Rule(40, [arrs[0], arrs[1], None, arrs[2]],
                              events=[(0, 1), (7, 0), (8, 0), (21, 2), (33, 3), (39, 1)],
                              stager=stager),
    }


@pytest.mark.parametrize("model", ["PerformantNet1", "vgg11", "vgg11_bn"])
def test_fused_step_equals_reduce_then_stream(pool, model):
    from flsim.engine import ProgramStager, engine_class
    cls = engine_class(model)
    eng, theta = _filled_engine(cls, pool, [(0, 0, 1), (0, 3, 7)])
    P = eng.P
    S = torch.zeros(P + 64, device=DEV)
    eng.end_epoch(S)
    S2 = torch.zeros_like(S)
    eng.end_epoch(S2)                          # repeated reduction (counters reset in-launch)
    assert torch.equal(S, S2)
    g = torch.Generator(device="cpu").manual_seed(11)
    base = [theta.clone(), (torch.randn(P, generator=g) * 1e-4).to(DEV),
            (torch.rand(P, generator=g) * 1e-6).to(DEV)]
    for name, rule in _rules(P, ProgramStager(DEV)).items():
        a = [t.clone() for t in base]
        b = [t.clone() for t in base]
        eng.aggregate_rule(S, rule, *a, 3)
        out = torch.full_like(S, float("nan"))
        eng.server_step(out, rule, *b, 3)
        torch.cuda.synchronize()
        assert torch.equal(out[:P], S[:P]), name
        for x, y, what in zip(a, b, "pmv"):
            bad = int((x.view(torch.int32) != y.view(torch.int32)).sum())
            assert bad == 0, (model, name, what, bad)


@pytest.mark.parametrize("delays", [None, [0, 2, 0, 3, 0, 2]])
def test_fused_simulation_equals_unfused(pool, delays):
    """FLSimulation at world = 1 ends every epoch with k_slab_step; fused=False runs end_epoch +
    k_agg_stream.  Same slab reduction order -> identical theta / m / v, ticks included (the FIFO
    slot is written by the fused kernel)."""
    from flsim.sim import FLSimulation
    kw = dict(delay=2, throttle=True, device=DEV, chunk_workers=2, pool=pool)
    n = 6
    a = FLSimulation(n, delays=delays, **kw)
    b = FLSimulation(n, delays=delays, fused=False, **kw)
    for t in range(7):
        la, lb = a.epoch(), b.epoch()
        assert la == lb or (np.isnan(la) and np.isnan(lb))
    for x, y in ((a.theta, b.theta), (a.m, b.m), (a.v, b.v)):
        assert torch.equal(x, y)


def test_stream_rule_reference_tick_bit_exact_vs_oracle():
    """k_agg_stream with the reference's tick entry list at n = 1024 (c_t = 512 fresh + the stale
    S_{t-d}) against the oracle's cascade + Adam, bit for bit."""
    from flsim.engine import PN1_SIZES, Rule, aggregate_rule
    from oracle import oracle as O
    P = sum(PN1_SIZES)
    rs = np.random.RandomState(21)
    S = (rs.standard_normal(P) * 1e-2).astype(np.float32)
    st = (rs.standard_normal(P) * 1e-2).astype(np.float32)
    p = rs.standard_normal(P).astype(np.float32)
    m = (rs.standard_normal(P) * 1e-3).astype(np.float32)
    v = (rs.rand(P) * 1e-5).astype(np.float32)
    dp, dm, dv = (torch.from_numpy(x.copy()).to(DEV) for x in (p, m, v))
    aggregate_rule(torch.from_numpy(S).to(DEV), Rule(513, [torch.from_numpy(st).to(DEV)], c=512),
                   dp, dm, dv, 51, PN1_SIZES)
    g = np.empty_like(S)
    off = 0
    for n in PN1_SIZES:
        g[off:off + n] = O.cascade_mean([S[off:off + n]] * 512 + [st[off:off + n]])
        off += n
    O.adam_step(p, m, v, g, 51)
    for name, x, y in (("p", dp, p), ("m", dm, m), ("v", dv, v)):
        assert np.array_equal(x.cpu().numpy().view(np.uint32), y.view(np.uint32)), name


@pytest.mark.parametrize("narr", [0, 1, 2])
def test_stream_variants_and_fifo_write_agree(narr, monkeypatch):
    """The register-array stream (k_agg_stream_reg, 1 and 2 float4 groups per thread) and the
    LDS-staged k_agg_stream (FLSIM_AGG_G=0) give the same bits for the reference order with 0, 1
    and 2 stale arrays, on every tensor edge and tail; S_out (the FIFO slot written in the same
    pass, world > 1 at a tick) equals S_t."""
    from flsim.engine import PN1_SIZES, Rule, aggregate_rule
    P = sum(PN1_SIZES)
    g = torch.Generator(device="cpu").manual_seed(5 + narr)
    S = (torch.randn(P + 64, generator=g) * 1e-2).to(DEV)
    arrs = [(torch.randn(P + 64, generator=g) * 1e-2).to(DEV) for _ in range(narr)]
    base = [torch.randn(P + 64, generator=g).to(DEV), (torch.randn(P + 64, generator=g) * 1e-3).to(DEV),
            (torch.rand(P + 64, generator=g) * 1e-5).to(DEV)]
    outs = {}
    for G in ("0", "1", "2"):
        monkeypatch.setenv("FLSIM_AGG_G", G)
        a = [t.clone() for t in base]
        slot = torch.full_like(S, float("nan"))
        aggregate_rule(S, Rule(512 + narr, arrs, c=512), *a, 7, PN1_SIZES, S_out=slot)
        torch.cuda.synchronize()
        assert torch.equal(slot[:P], S[:P]), G
        outs[G] = a
    for G in ("1", "2"):
        for x, y, what in zip(outs[G], outs["0"], "pmv"):
            bad = int((x[:P].view(torch.int32) != y[:P].view(torch.int32)).sum())
            assert bad == 0, (G, what, bad)
