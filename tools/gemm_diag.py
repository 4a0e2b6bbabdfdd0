"""Diagnostic (GPU box): the accuracy of ONE data-gradient GEMM of PerformantNet1 on its own GPU
inputs, against fp64 and against the CPU fp32 port (torch) on the same fp32 inputs.

  FLSIM_DEBUG_BWD_STOP=<6|5|4> python tools/gemm_diag.py [--items t,i,k ...]

The backward pass stops after conv<stop>'s data gradient (pn1_net.hip debug_stop), so that GEMM's
inputs (the dZ it reads, the layer's weights, the forward masks) and its output are still in the
workspace.  Per output: relative L2 error of the GPU and of torch fp32 against fp64, and the
scale coefficient alpha = <err, ref> / <ref, ref> (a systematic shrink or growth of the output
shows as alpha far from 0 with |alpha| close to the relative error).
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (os.path.join(REPO, "tests"), REPO, os.path.join(REPO, "fl-distributed-delay_amd")):
    sys.path.insert(0, _p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--items", nargs="*", default=["0,1,2", "0,2,0"])
    args = ap.parse_args()
    stop = int(os.environ.get("FLSIM_DEBUG_BWD_STOP", "0"))
    assert stop in (4, 5, 6), "set FLSIM_DEBUG_BWD_STOP to 6, 5 or 4"
    import numpy as np
    import torch
    from flsim.data import DevicePool
    from flsim.engine import PN1Engine, worker_table
    from oracle import model_ref as MR
    from oracle import oracle as O

    dev = "cuda:0"
    items = [tuple(int(v) for v in s.split(",")) for s in args.items]
    nw = len(items)
    pool = O.make_pool(0)
    sim = MR.OracleSim(4, delay=2, pool=pool, dropout=True)
    eng = PN1Engine(dev, chunk_workers=nw)
    theta = torch.from_numpy(sim.theta.copy()).to(dev)
    eng.begin_epoch(theta)
    loss = torch.zeros(nw, device=dev)
    eng.run_chunk(theta, DevicePool(dev, 0, pool), worker_table(items, dev), nw, 4, 0, True, loss)
    S = torch.zeros(eng.P, device=dev)
    eng.end_epoch(S)          # the weight gradients that ran before the stop (conv6 .. conv<stop>)
    torch.cuda.synchronize()
    S = S.cpu().double()
    NS = eng.max_samples
    n = 128 * nw

    def W(i, shp, dt=torch.float32):
        return eng.workspace_view(i, shp, dt).cpu()[:n]

    def nchw(t):
        return t.permute(0, 3, 1, 2).contiguous()

    P = MR.split_flat(sim.theta.astype(np.float32))
    cgi = torch.nn.grad.conv2d_input
    s25 = float(np.float32(1.0) / np.float32(0.75))

    def gemm(dt):
        """the GEMM (+ its epilogue) in dtype dt on the GPU's own inputs"""
        w = lambda j: torch.from_numpy(P[j]).to(dt)                 # noqa: E731
        if stop == 6:
            dz6 = nchw(W(8, (NS, 14, 14, 192))).to(dt)
            full = torch.zeros(n, 192, 15, 15, dtype=dt)
            full[:, :, :14, :14] = dz6
            a5 = nchw(W(7, (NS, 13, 13, 192)))
            return cgi((n, 192, 13, 13), w(10), full, padding=2) * (a5 > 0).to(dt)
        if stop == 5:
            dz5 = nchw(W(14, (NS, 13, 13, 192))).to(dt)
            g = cgi((n, 96, 11, 11), w(8), dz5, padding=2)
            d2 = nchw(W(6, (NS, 11, 11, 96)))
            v = g * s25 * (d2 > 0).to(dt)
            idx = nchw(W(20, (NS, 11, 11, 96), torch.uint8)).long()
            out = torch.zeros(n, 96, 22, 22, dtype=dt)
            rows = 2 * torch.arange(11).view(1, 1, 11, 1) + (idx >> 1)
            cols = 2 * torch.arange(11).view(1, 1, 1, 11) + (idx & 1)
            out[torch.arange(n).view(n, 1, 1, 1), torch.arange(96).view(1, 96, 1, 1), rows, cols] = v
            return out
        dz4 = nchw(W(5, (NS, 22, 22, 96))).to(dt)
        a3 = nchw(W(4, (NS, 20, 20, 96)))
        return cgi((n, 96, 20, 20), w(6), dz4, padding=2) * (a3 > 0).to(dt)

    def wgrad(dt):
        """the layer's weight and bias gradient (the slab GEMM + column sum) in dtype dt on the
        GPU's own inputs: conv<stop>'s input activation and its dZ"""
        cgw = torch.nn.grad.conv2d_weight
        if stop == 6:
            x_in = nchw(W(7, (NS, 13, 13, 192))).to(dt)
            dz = torch.zeros(n, 192, 15, 15, dtype=dt)
            dz[:, :, :14, :14] = nchw(W(8, (NS, 14, 14, 192))).to(dt)
            shp = (192, 192, 3, 3)
        elif stop == 5:
            x_in = nchw(W(6, (NS, 11, 11, 96))).to(dt)
            dz = nchw(W(14, (NS, 13, 13, 192))).to(dt)
            shp = (192, 96, 3, 3)
        else:
            x_in = nchw(W(4, (NS, 20, 20, 96))).to(dt)
            dz = nchw(W(5, (NS, 22, 22, 96))).to(dt)
            shp = (96, 96, 3, 3)
        return cgw(x_in, shp, dz, padding=2), dz.sum((0, 2, 3))

    def stats(t, r64):
        rn = float(r64.norm())
        rr = float((r64 * r64).sum())
        d = t - r64
        return dict(rel=float(d.norm()) / rn, alpha=float((d * r64).sum()) / rr,
                    resid=float((d - (float((d * r64).sum()) / rr) * r64).norm()) / rn)

    gpu = {6: lambda: nchw(W(14, (NS, 13, 13, 192))), 5: lambda: nchw(W(5, (NS, 22, 22, 96))),
           4: lambda: nchw(W(14, (NS, 20, 20, 96)))}[stop]().double()
    r64 = gemm(torch.float64)
    r32 = gemm(torch.float32).double()
    out = dict(stop=stop, gemm={6: "conv6 dgrad (fp32)", 5: "conv5 dgrad (fp32) + pool2 scatter",
                                4: "conv4 dgrad (fp32)"}[stop], items=items)
    for name, t in (("gpu", gpu), ("cpu32", r32)):
        out[name] = stats(t, r64)
        # what the previous layer's bias gradient sees: the per-channel sums of the output
        out[name]["chan_sum"] = stats(t.sum((0, 2, 3)), r64.sum((0, 2, 3)))["rel"]
    # the weight-gradient GEMM of the same layer (it ran before the data gradient)
    j = {6: 10, 5: 8, 4: 6}[stop]
    off = int(sum(a.size for a in P[:j]))
    gw = S[off:off + P[j].size].view(P[j].shape)
    gb = S[off + P[j].size:off + P[j].size + P[j + 1].size]
    w64, b64 = wgrad(torch.float64)
    w32, b32 = wgrad(torch.float32)
    out["wgrad"] = dict(gpu_w=stats(gw, w64), cpu32_w=stats(w32.double(), w64),
                        gpu_b=stats(gb, b64), cpu32_b=stats(b32.double(), b64))
    print("GEMM_DIAG", json.dumps(out))


if __name__ == "__main__":
    main()
