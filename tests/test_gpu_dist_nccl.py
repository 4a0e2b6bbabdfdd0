"""The N > 1 path over RCCL on the one GPU of the test box: a one-rank `nccl` process group.

bench.py --force-dist runs it on the driver's box (RCCL init, the per-epoch all-reduce of
[S_t | losses], the streaming server step after it instead of the fused one); these tests pin it
bit for bit to the fused single-process path through the first tick (main.py:150-166: the slow
worker pushes at t = 0 and t = 50, t = 50 pops S_0, t = 51 runs every fast worker), with

  * collective="torch": torch.distributed.all_reduce (the nccl backend = RCCL);
  * collective="flsim": the C-ABI's flsim_allreduce_sum (include/flsim.h) on an RCCL
    communicator of its own (ncclCommInitRank, unique id shipped over the process group).

The tick epoch builds S_t in the FIFO slot it pushes and all-reduces it there (sim.py in_slot):
the slot must hold the fused path's S_50, and the slot of t = 0 must be released at t = 50.
"""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist

from conftest import has_gpu

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not has_gpu(), reason="needs an MI355X")]

DEV = "cuda:0"
N, D, EPOCHS = 64, 50, 53


@pytest.fixture(scope="module")
def fused():
    from flsim.sim import FLSimulation
    from oracle import oracle as O
    sim = FLSimulation(N, delay=D, throttle=True, device=DEV, pool=O.make_pool(0),
                       chunk_workers=32)
    losses = [sim.epoch() for _ in range(EPOCHS)]
    torch.cuda.synchronize()
    return dict(losses=losses, trace=[(p.t, p.computes.tobytes(), tuple(p.stale))
                                      for p in sim.trace],
                theta=sim.theta.clone(), m=sim.m.clone(), v=sim.v.clone(),
                slot50=sim.stale_store[50][0][:sim.P].clone(), slots=sorted(sim.stale_store))


@pytest.mark.parametrize("collective", ["torch", "flsim"])
def test_one_rank_nccl_group_matches_fused(fused, collective):
    from flsim.sim import FLSimulation
    from oracle import oracle as O
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(29600 + os.getpid() % 1000 + (7 if collective == "flsim"
                                                                   else 0))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device(DEV))
    sim = None
    try:
        sim = FLSimulation(N, delay=D, throttle=True, device=DEV, pool=O.make_pool(0),
                           chunk_workers=32, distributed=True, collective=collective)
        assert sim.distributed and (sim._comm is not None) == (collective == "flsim")
        calls = []
        inner = sim._all_reduce
        sim._all_reduce = lambda buf: (calls.append(buf.numel()), inner(buf))
        losses, slot50 = [], None
        for t in range(EPOCHS):
            losses.append(sim.epoch())
            if t == 50:
                # the tick's all-reduce landed in the FIFO slot it pushed (no second copy)
                slot50 = sim.stale_store[50][0]
                assert 0 not in sim.stale_store            # S_0 popped at t = 50, released
        torch.cuda.synchronize()
    finally:
        if getattr(sim, "_comm", None) is not None:
            sim._comm.close()
        dist.destroy_process_group()
    assert len(calls) == EPOCHS
    assert [(p.t, p.computes.tobytes(), tuple(p.stale)) for p in sim.trace] == fused["trace"]
    assert losses == fused["losses"]
    assert torch.equal(slot50[:sim.P], fused["slot50"])
    assert sorted(sim.stale_store) == fused["slots"]
    for name in ("theta", "m", "v"):
        a, b = getattr(sim, name), fused[name]
        assert torch.equal(a, b), (name, int((a != b).sum()))
    assert np.isfinite(losses).all()
