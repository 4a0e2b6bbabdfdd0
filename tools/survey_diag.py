"""Diagnostic (GPU box): where a libflsim build's worker-step gradient parts from fp64, against the
CPU fp32 port, tensor by tensor and activation by activation (SURVEY 8(c)'s criterion).

  python tools/survey_diag.py [--pkg DIR] [--dropout 0|1] [--items t,i,k ...]

--pkg: a directory holding another build's `flsim` package (e.g. the last all-fp32-MFMA tree, built
from git into tools/abfp32/pkg) to run instead of this tree's.  For one chunk it prints, per
parameter tensor, the relative errors of the GPU and of the CPU fp32 port against the fp64
reference -- all three given the GPU's own forward decisions -- the SURVEY ratio
e_gpu / (2 e_cpu + 1e-7 |g|), and the coherence |sum(err)| / |err| of each error (about 1 for
independent rounding errors, up to sqrt(n) for a systematic one); then the same errors of the
GPU's stored forward activations.
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pkg", default=None)
    ap.add_argument("--dropout", type=int, default=1)
    ap.add_argument("--items", nargs="*", default=["0,1,2"])
    args = ap.parse_args()
    pkg = args.pkg or os.path.join(REPO, "fl-distributed-delay_amd")
    for p in (os.path.join(REPO, "tests"), REPO, pkg):
        sys.path.insert(0, p)
    import numpy as np
    import torch
    import torch.nn.functional as F
    import _flips
    from flsim.data import DevicePool
    from flsim.engine import PN1Engine, PN1_SHAPES, worker_table
    from oracle import model_ref as MR
    from oracle import oracle as O

    dev = "cuda:0"
    items = [tuple(int(v) for v in s.split(",")) for s in args.items]
    nw = len(items)
    n = 128 * nw
    pool = O.make_pool(0)
    sim = MR.OracleSim(4, delay=2, pool=pool, dropout=bool(args.dropout))
    eng = PN1Engine(dev, chunk_workers=nw)
    dpool = DevicePool(dev, 0, pool)
    theta = torch.from_numpy(sim.theta.copy()).to(dev)
    eng.begin_epoch(theta)
    loss = torch.zeros(nw, device=dev)
    eng.run_chunk(theta, dpool, worker_table(items, dev), nw, 4, 0, bool(args.dropout), loss)
    S = torch.zeros(eng.P, device=dev)
    eng.end_epoch(S)
    torch.cuda.synchronize()
    g_gpu = S.cpu().numpy().astype(np.float64)
    xs, ys = zip(*[sim.batch(*it, dtype=torch.float64) for it in items])
    x, y = torch.cat(xs), torch.cat(ys)
    noise = _flips.noise_groups([(t, i) for (t, i, _) in items], n, bool(args.dropout))
    forced = _flips.gpu_decisions(eng, n)
    scale = 1.0 / 128
    g64, _ = _flips.grad(sim.theta, torch.float64, x, y, noise, scale, forced)
    g32, _ = _flips.grad(sim.theta, torch.float32, x, y, noise, scale, forced)
    out = {"pkg": pkg, "items": items, "dropout": args.dropout, "tensors": {}, "activations": {}}
    off = 0
    print(f"{'tensor':16s} {'|g|':>10s} {'e_gpu/|g|':>10s} {'e_cpu/|g|':>10s} {'ratio':>6s} "
          f"{'coh_gpu':>8s} {'coh_cpu':>8s} {'coh_g':>8s} {'a_gpu':>10s} {'a_cpu':>10s}")
    for name, shp in PN1_SHAPES:
        k = int(np.prod(shp))
        sl = slice(off, off + k)
        off += k
        r = g64[sl]
        dg, dc = g_gpu[sl] - r, g32[sl] - r
        nr, eg, ec = (float(np.linalg.norm(v)) for v in (r, dg, dc))
        rr = float(r @ r)
        rec = dict(norm=nr, e_gpu=eg / nr, e_cpu=ec / nr, ratio=eg / (2 * ec + 1e-7 * nr),
                   coh_gpu=abs(float(dg.sum())) / max(eg, 1e-300),
                   coh_cpu=abs(float(dc.sum())) / max(ec, 1e-300), n=k,
                   coh_g=abs(float(r.sum())) / max(nr, 1e-300),
                   alpha_gpu=float(dg @ r) / rr, alpha_cpu=float(dc @ r) / rr)
        out["tensors"][name] = rec
        print(f"{name:16s} {nr:10.3e} {rec['e_gpu']:10.3e} {rec['e_cpu']:10.3e} {rec['ratio']:6.2f} "
              f"{rec['coh_gpu']:8.2f} {rec['coh_cpu']:8.2f} {rec['coh_g']:8.2f} "
              f"{rec['alpha_gpu']:+10.2e} {rec['alpha_cpu']:+10.2e}")

    # forward activations: the GPU's stored tensors against the forced fp64 / fp32 forwards
    def acts(dt):
        P = [torch.tensor(a, dtype=dt) for a in MR.split_flat(sim.theta.astype(
            np.float64 if dt == torch.float64 else np.float32))]
        (w1, b1, w2, b2, w3, b3, w4, b4, w5, b5, w6, b6, l1w, l1b, l2w, l2b, _, _) = P
        nz = [t.to(dt) for t in noise] if noise is not None else [None] * 5
        mul = (lambda h, i: h if nz[i] is None else h * nz[i])      # noqa: E731
        m = (lambda key: forced[key].to(dt))                          # noqa: E731
        xx = x.to(dt)
        a = {}
        with torch.no_grad():
            h = F.conv2d(xx, w1, b1, padding=2) * m("a1")
            a["a1"] = h
            h = mul(_flips.gather(F.conv2d(h, w2, b2, padding=2), forced["i1"]) * m("i1m"), 0)
            a["d1"] = h
            h = F.conv2d(h, w3, b3, padding=2) * m("a3")
            a["a3"] = h
            h = mul(_flips.gather(F.conv2d(h, w4, b4, padding=2), forced["i2"]) * m("i2m"), 1)
            a["d2"] = h
            h = F.conv2d(h, w5, b5, padding=2) * m("a5")
            a["a5"] = h
            h = mul(_flips.gather(F.conv2d(h, w6, b6, padding=2), forced["i3"]) * m("i3m"), 2)
            h = h.reshape(n, -1)
            a["d3"] = h
            h = mul(F.linear(h, l1w, l1b) * m("e1"), 3)
            a["e1"] = h
            h = mul(F.linear(h, l2w, l2b) * m("e2"), 4)
            a["e2"] = h
        return a

    A64, A32 = acts(torch.float64), acts(torch.float32)
    NS = eng.max_samples
    nchw = lambda t: t.permute(0, 3, 1, 2)                                # noqa: E731
    W = lambda i, shp: eng.workspace_view(i, shp, torch.float32).cpu()[:n]   # noqa: E731
    gpu = dict(a1=nchw(W(1, (NS, 34, 34, 48))), d1=nchw(W(3, (NS, 18, 18, 48))),
               a3=nchw(W(4, (NS, 20, 20, 96))), d2=nchw(W(6, (NS, 11, 11, 96))),
               a5=nchw(W(7, (NS, 13, 13, 192))), d3=W(9, (NS, 9408)),
               e1=W(10, (NS, 512)), e2=W(11, (NS, 256)))
    print(f"{'activation':16s} {'|a|':>10s} {'e_gpu/|a|':>10s} {'e_cpu/|a|':>10s} {'ratio':>6s}")
    for k in gpu:
        r = A64[k].double()
        eg = float((gpu[k].double() - r).norm())
        ec = float((A32[k].double() - r).norm())
        nr = float(r.norm())
        rr = float((r * r).sum())
        ag = float(((gpu[k].double() - r) * r).sum()) / rr
        ac = float(((A32[k].double() - r) * r).sum()) / rr
        out["activations"][k] = dict(e_gpu=eg / nr, e_cpu=ec / nr, ratio=eg / max(ec, 1e-300),
                                     alpha_gpu=ag, alpha_cpu=ac)
        print(f"{k:16s} {nr:10.3e} {eg / nr:10.3e} {ec / nr:10.3e} {eg / max(ec, 1e-300):6.2f} "
              f"{ag:+10.2e} {ac:+10.2e}")
    print("SURVEY_DIAG", json.dumps(out))


if __name__ == "__main__":
    main()
