"""world_size-2 gloo test of the worker sharding + one all-reduce per server step (CPU).

The HIP engine is replaced by a deterministic CPU stand-in (each worker-step contributes a
vector that depends on (t, i, k, theta)); the test checks that 2 ranks, each computing only its
contiguous block of the epoch's computing workers, end every epoch with the same parameters,
staleness trace and per-worker losses as a single-process run.
"""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

P = 5596090


class StandInEngine:
    """CPU stand-in with PN1Engine's interface (not a model: a fixed function of the inputs)."""

    def __init__(self):
        self.P = P
        self.chunk_workers = 3
        self.acc = torch.zeros(P, dtype=torch.float64)

    def begin_epoch(self, theta):
        self.acc.zero_()
        self.theta_sum = float(theta[:1000].double().sum())

    def run_chunk(self, theta, pool, workers_dev, n_chunk, n_total, seed, dropout, loss_out,
                  backward=True):
        for j, (t, i, k, _) in enumerate(workers_dev.tolist()):
            g = torch.arange(P, dtype=torch.float64).mul_(1e-7 * (i + 1)).sin_()
            self.acc += g * (1 + 0.01 * k) + 1e-3 * self.theta_sum
            loss_out[j] = float(t + 0.001 * i + 0.0001 * k)

    def end_epoch(self, S):
        S.copy_(self.acc.float())

    def aggregate_adam_sum(self, S, k, theta, m, v, step, lr=1e-3, betas=(0.9, 0.999), eps=1e-8):
        theta -= lr * S / k

    def aggregate_rule(self, S, rule, theta, m, v, step, lr=1e-3, betas=(0.9, 0.999), eps=1e-8,
                       S_out=None):
        """rule.arrays in order after c copies of S (reference order) or at the event
        positions (general order); a plain weighted mean, enough to check the sharding.  S_out:
        the FIFO slot of a tick, written with S_t (the product stream does it in its pass)."""
        if S_out is not None:
            S_out[:P].copy_(S)
        if rule.events is None:
            n_s, extra = rule.c, rule.arrays
        else:
            n_s, extra = rule.k - len(rule.events), [rule.arrays[j] for (_, j) in rule.events]
        tot = S * n_s
        for a in extra:
            if a is not None:
                tot = tot + a[:P]
        theta -= lr * tot / rule.k


def _run(rank, world, n, d, thr, epochs, out, port, delays=None, semantics="reference",
         force=False, collective="torch"):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.dirname(here))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "fl-distributed-delay_amd"))
    if world > 1 or force:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
    from flsim.sim import FLSimulation
    sim = FLSimulation(n, delay=d, delays=delays, throttle=thr, device="cpu", semantics=semantics,
                       engine=StandInEngine(), device_pool=object(), theta0=torch.zeros(P),
                       distributed=True if force else None, collective=collective)
    calls = []
    if force:                    # count the epoch's collectives (events are CUDA-only)
        inner = sim._all_reduce
        sim._all_reduce = lambda buf: (calls.append(buf.numel()), inner(buf))
    abi = []
    if sim._comm is not None:    # ... and the C-ABI's flsim_allreduce_sum calls among them
        inner_c = sim._comm.all_reduce_sum
        sim._comm.all_reduce_sum = lambda buf: (abi.append(buf.numel()), inner_c(buf))
    losses = [sim.epoch() for _ in range(epochs)]
    res = dict(theta=sim.theta.numpy().copy(), losses=losses,
               trace=[(p.t, p.computes.tobytes(), p.stale) for p in sim.trace],
               distributed=sim.distributed, collectives=len(calls), abi_calls=len(abi))
    if world > 1 or force:
        dist.destroy_process_group()
    out[rank] = res


def test_forced_distributed_world1_flsim_collective():
    """The same one-rank N > 1 path with the epoch's all-reduce through the C-ABI
    (collective="flsim-local": flsim_allreduce_sum on the one-rank communicator) instead of
    torch.distributed: one ABI call per epoch, the single-process trace, losses and theta."""
    n, d, epochs = 11, 3, 5
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    single = mgr.dict()
    _run(0, 1, n, d, True, epochs, single, 0)
    out = mgr.dict()
    port = 29500 + (os.getpid() % 1000) + 31
    p = ctx.Process(target=_run, args=(0, 1, n, d, True, epochs, out, port, None, "reference",
                                       True, "flsim-local"))
    p.start()
    p.join(300)
    assert p.exitcode == 0
    assert out[0]["collectives"] == epochs and out[0]["abi_calls"] == epochs
    assert out[0]["trace"] == single[0]["trace"]
    np.testing.assert_array_equal(out[0]["losses"], single[0]["losses"])
    np.testing.assert_array_equal(out[0]["theta"], single[0]["theta"])


@pytest.mark.parametrize("thr,delays", [
    (False, None), (True, None),
    (True, [0, 2, 0, 0, 3, 0, 0, 2, 0, 0, 0]),     # heterogeneous delays: interleaved stale entries
])
def test_two_rank_sharding_matches_single(thr, delays):
    n, d, epochs = 11, 3, 7
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    single = mgr.dict()
    _run(0, 1, n, d, thr, epochs, single, 0, delays)
    out = mgr.dict()
    port = 29500 + (os.getpid() % 1000) + (7 if delays else 0) + (3 if thr else 0)
    procs = [ctx.Process(target=_run, args=(r, 2, n, d, thr, epochs, out, port, delays))
             for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
        assert p.exitcode == 0
    for r in range(2):
        assert out[r]["trace"] == single[0]["trace"]
        np.testing.assert_allclose(out[r]["losses"], single[0]["losses"], rtol=0, atol=1e-6)
        np.testing.assert_allclose(out[r]["theta"], single[0]["theta"], rtol=1e-5, atol=1e-7)
    assert np.array_equal(out[0]["theta"], out[1]["theta"])


@pytest.mark.parametrize("delays", [None, [0, 2, 0, 0, 3, 0, 0, 2, 0, 0, 0]])
def test_two_rank_independent_entries_match_single(delays):
    """Independent-entry semantics: each slow worker's own gradient stays on its owner rank
    (index mod world) and is added to that rank's partial sum before the one all-reduce."""
    n, d, epochs = 11, 3, 8
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    single = mgr.dict()
    _run(0, 1, n, d, True, epochs, single, 0, delays, "independent")
    out = mgr.dict()
    port = 29500 + (os.getpid() % 1000) + 13 + (5 if delays else 0)
    procs = [ctx.Process(target=_run, args=(r, 2, n, d, True, epochs, out, port, delays,
                                            "independent")) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
        assert p.exitcode == 0
    for r in range(2):
        assert out[r]["trace"] == single[0]["trace"]
        np.testing.assert_allclose(out[r]["losses"], single[0]["losses"], rtol=0, atol=1e-6)
        np.testing.assert_allclose(out[r]["theta"], single[0]["theta"], rtol=1e-5, atol=1e-7)
    assert np.array_equal(out[0]["theta"], out[1]["theta"])


def test_forced_distributed_world1_matches_single():
    """bench.py --force-dist at world size 1: the N > 1 code path (sharding, the per-epoch
    all-reduce of [S_t | losses], the streaming server step after it) over a one-rank group must
    give the single-process run's trace, losses and theta, with one collective per epoch."""
    n, d, epochs = 11, 3, 7
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    single = mgr.dict()
    _run(0, 1, n, d, True, epochs, single, 0)
    out = mgr.dict()
    port = 29500 + (os.getpid() % 1000) + 29
    p = ctx.Process(target=_run, args=(0, 1, n, d, True, epochs, out, port, None, "reference",
                                       True))
    p.start()
    p.join(300)
    assert p.exitcode == 0
    assert out[0]["distributed"] and not single[0]["distributed"]
    assert out[0]["collectives"] == epochs
    assert out[0]["trace"] == single[0]["trace"]
    np.testing.assert_array_equal(out[0]["losses"], single[0]["losses"])
    np.testing.assert_array_equal(out[0]["theta"], single[0]["theta"])
