"""SURVEY 8(c)'s per-tensor accuracy criterion at the headline's own chunk size.

The headline (bench.py: n = 1024, d = 50, throttle) builds S_t from 128-worker chunks, 16,384
samples per launch, and the split-bf16 weight gradients (csrc/gemm_x6.h: conv2-6, linear1) sum
over K = samples x output pixels of one chunk.  The bf16 MFMA drops addend bits toward zero
(DESIGN 6f), a bias that can grow with K, while the other accuracy checks run at <= 256 samples.
Here every weight and bias gradient of nw workers (nw = 2 .. 128 in one chunk; 512 = the bench's
throttled epoch, four chunks into the same slabs) is checked on the GPU's own inputs -- the layer
input and dZ the backward pass left in the workspace -- against

  * fp64: the same contraction in float64 (on the GPU: unfold + a float64 matmul);
  * the CPU fp32 port: torch-CPU's own weight/bias-gradient kernels (the autograd path of
    agents.py:35, `convolution_backward` / `mm`) over each worker's 128 samples, accumulated
    worker by worker in fp32, as AccumulateGrad does across fwd_bkwd calls (agents.py:35,
    main.py:137-170);

and SURVEY 8(c) requires, per tensor T,
    ||g_gpu,T - g64,T|| <= 2 ||g_cpu32,T - g64,T|| + 1e-7 ||g64,T||.

The backward pass is stopped after conv5's / conv3's data gradient (FLSIM_DEBUG_BWD_STOP,
pn1_net.hip) to read dz5 / dz3 before gx is reused; every pass is deterministic, so the three
passes see the same bits.  The ratios per K go to MEASURED lines (and FLSIM_TOL_LOG).
"""
import os

import numpy as np
import pytest
import torch

from conftest import has_gpu

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not has_gpu(), reason="needs an MI355X")]

DEV = "cuda:0"

# workspace ids (PN1Engine.WORKSPACE)
X0, A1, A2, D1, A3, A4, D2, A5, A6, D3, E1, E2, DH1, DH2, GX = range(15)

# layer -> (stop pass, input id, input NHWC shape[1:], dZ id, dZ NHWC shape[1:], param index)
CONV = {
    "conv1": (0, X0, (32, 32, 4), GX, (34, 34, 48), 0),
    "conv2": (0, A1, (34, 34, 48), A2, (36, 36, 48), 2),
    "conv3": (3, D1, (18, 18, 48), GX, (20, 20, 96), 4),
    "conv4": (3, A3, (20, 20, 96), A4, (22, 22, 96), 6),
    "conv5": (5, D2, (11, 11, 96), GX, (13, 13, 192), 8),
    "conv6": (3, A5, (13, 13, 192), A6, (14, 14, 192), 10),   # dz6 compact (row/col 14 = 0)
}
LINEAR = {
    "linear1": (3, D3, 9408, DH1, 512, 12),
    "linear2": (3, E1, 512, DH2, 256, 14),
}
X6 = ("conv2", "conv3", "conv4", "conv5", "conv6", "linear1")   # split-bf16 weight gradients


@pytest.fixture(scope="module")
def setup():
    from flsim.data import DevicePool
    from flsim.engine import PN1Engine
    from oracle import model_ref as MR
    from oracle import oracle as O
    pool = O.make_pool(0)
    sim = MR.OracleSim(1024, delay=50, pool=pool)
    eng = PN1Engine(DEV, chunk_workers=128)
    return sim, eng, DevicePool(DEV, 0, pool)


def _run(eng, dpool, theta, tables, sizes, stop):
    """One epoch of chunk passes ending at `stop` (0: the whole backward); returns S (the
    epoch's sum)."""
    old = os.environ.get("FLSIM_DEBUG_BWD_STOP")
    os.environ["FLSIM_DEBUG_BWD_STOP"] = str(stop)
    try:
        eng.begin_epoch(theta)
        loss = torch.zeros(sum(sizes), device=DEV)
        r = 0
        for table, nw in zip(tables, sizes):
            eng.run_chunk(theta, dpool, table, nw, 1024, 0, True, loss[r:r + nw])
            r += nw
        S = torch.zeros(eng.P, device=DEV)
        eng.end_epoch(S)
        torch.cuda.synchronize()
    finally:
        if old is None:
            del os.environ["FLSIM_DEBUG_BWD_STOP"]
        else:
            os.environ["FLSIM_DEBUG_BWD_STOP"] = old
    assert torch.isfinite(loss).all()
    return S


def _conv_refs(eng, name, n, theta_parts):
    """(fp64 weight, fp64 bias, cpu32 weight, cpu32 bias) of conv `name` over n samples."""
    _, xi, xs, di, ds, j = CONV[name]
    co, ci = theta_parts[j].shape[:2]
    x = eng.workspace_view(xi, (eng.max_samples,) + xs)[:n]
    dz = eng.workspace_view(di, (eng.max_samples,) + ds)[:n]
    oh = xs[0] + 2
    w32 = torch.zeros(co, ci, 3, 3)
    g64 = torch.zeros(co, ci * 9, dtype=torch.float64, device=DEV)
    b64 = torch.zeros(co, dtype=torch.float64, device=DEV)
    gw32 = gb32 = None
    for r in range(0, n, 128):
        xw = x[r:r + 128, :, :, :ci].permute(0, 3, 1, 2).contiguous()        # NCHW
        dzw = torch.zeros(128, co, oh, oh, device=DEV)
        dzw[:, :, :ds[0], :ds[1]] = dz[r:r + 128].permute(0, 3, 1, 2)
        # fp64: unfold + matmul (k order ci, kh, kw = the weight's own)
        col = torch.nn.functional.unfold(xw.double(), 3, padding=2)            # [128, ci*9, L]
        d64 = dzw.double().reshape(128, co, -1)
        g64 += torch.bmm(d64, col.transpose(1, 2)).sum(0)
        b64 += d64.sum((0, 2))
        # the CPU fp32 port: torch-CPU's autograd kernels for this worker, then AccumulateGrad
        _, gw, gb = torch.ops.aten.convolution_backward(
            dzw.cpu(), xw.cpu(), w32, [co], [1, 1], [2, 2], [1, 1], False, [0, 0], 1,
            [False, True, True])
        gw32 = gw if gw32 is None else gw32 + gw
        gb32 = gb if gb32 is None else gb32 + gb
    return (g64.cpu().reshape(-1), b64.cpu(), gw32.double().reshape(-1), gb32.double())


def _linear_refs(eng, name, n):
    _, xi, k, di, co, _ = LINEAR[name]
    x = eng.workspace_view(xi, (eng.max_samples, k))[:n]
    dz = eng.workspace_view(di, (eng.max_samples, co))[:n]
    g64 = (dz.double().t() @ x.double()).cpu().reshape(-1)
    b64 = dz.double().sum(0).cpu()
    gw32 = gb32 = None
    for r in range(0, n, 128):
        xw, dw = x[r:r + 128].cpu(), dz[r:r + 128].cpu()
        gw, gb = dw.t().mm(xw), dw.sum(0)          # torch's linear backward (addmm's grads)
        gw32 = gw if gw32 is None else gw32 + gw
        gb32 = gb if gb32 is None else gb32 + gb
    return g64, b64, gw32.double().reshape(-1), gb32.double()


def _accumulate(dst, refs, key):
    """fp64 parts add; the CPU fp32 port's parts continue its worker-order fp32 accumulation."""
    for i, r in enumerate(refs):
        k = (key, i)
        dst[k] = r if k not in dst else dst[k] + r


@pytest.mark.parametrize("nw", [2, 8, 32, 128, 512])
def test_weight_gradients_survey_8c_at_chunk_size(setup, nw):
    """Every weight/bias gradient of nw workers (chunks of <= 128 workers; nw = 128 is the bench's
    16,384-sample launch, nw = 512 one of its throttled epochs: four launches into the same
    slabs) meets SURVEY 8(c) against fp64 and the CPU fp32 port on the GPU's own inputs."""
    import _flips
    from flsim.engine import PN1_SHAPES, worker_table
    sim, eng, dpool = setup
    rng = np.random.RandomState(nw)
    items = [(7, i, int(rng.randint(0, 1024))) for i in range(0, 2 * nw, 2)]   # (t, i, k)
    items[-1] = (7, items[-1][1], 1023)                      # one {1,9}-dataset worker
    chunks = [items[c:c + 128] for c in range(0, nw, 128)]
    theta = torch.from_numpy(sim.theta.copy()).to(DEV)
    offs = np.concatenate([[0], np.cumsum([int(np.prod(s)) for _, s in PN1_SHAPES])])
    tparts = [torch.from_numpy(sim.theta[offs[j]:offs[j + 1]].copy()).view(s)
              for j, (_, s) in enumerate(PN1_SHAPES)]
    acc = {}
    for ch in chunks:
        table = worker_table(ch, DEV)
        n = 128 * len(ch)
        for stop in (5, 3, 0):
            _run(eng, dpool, theta, [table], [len(ch)], stop)
            for name in list(CONV) + list(LINEAR):
                spec = CONV.get(name) or LINEAR[name]
                if spec[0] == stop:
                    refs = (_conv_refs(eng, name, n, tparts) if name in CONV
                            else _linear_refs(eng, name, n))
                    _accumulate(acc, refs, name)
    # the GPU's S over all chunks (one epoch: the chunks accumulate in the slabs)
    S = _run(eng, dpool, theta, [worker_table(ch, DEV) for ch in chunks],
             [len(ch) for ch in chunks], 0).double().cpu()
    gpu, c32, r64, shapes = [], [], [], []
    for name in list(CONV) + list(LINEAR):
        j = (CONV.get(name) or LINEAR[name])[-1]
        for part in (0, 1):                      # weight, bias
            nm, shp = PN1_SHAPES[j + part]
            gpu.append(S[offs[j + part]:offs[j + part + 1]])
            r64.append(acc[(name, part)])
            c32.append(acc[(name, 2 + part)])
            shapes.append((nm, shp))
    ratios = _flips.survey_ratios(torch.cat(gpu).numpy(), torch.cat(c32).numpy(),
                                  torch.cat(r64).numpy(), shapes)
    rel = {nm: float(np.linalg.norm((a - b).numpy()) / np.linalg.norm(b.numpy()))
           for (nm, _), a, b in zip(shapes, gpu, r64)}
    rel32 = {nm: float(np.linalg.norm((a - b).numpy()) / np.linalg.norm(b.numpy()))
             for (nm, _), a, b in zip(shapes, c32, r64)}
    _flips.log_measured("pn1_chunk_wgrad", workers=nw, samples=128 * nw, rel_gpu=rel,
                        rel_cpu32=rel32, x6=list(X6))
    _flips.assert_survey(ratios, f"pn1_chunk_wgrad_nw{nw}")
