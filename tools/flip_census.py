"""Decision-flip census (GPU box): where the GPU's worker-step gradient differs from the fp64
oracle, is it arithmetic or discrete decisions?

For one explicit batch through the facade's entry point (flsim_pn1_fwd_bwd_input: 128-sample
groups, dropout keys (t, i + b * 2^20), CE mean over the n samples):
  g_gpu   the HIP gradient
  g_tf    fp64 with the GPU's own decisions (ReLU signs, pool argmax, dropout) -- "teacher forced"
  g_64    fp64 with its own decisions (the oracle)
  g_32    CPU fp32 with its own decisions
and per layer the count of decisions where the GPU (or CPU fp32) disagrees with fp64: ReLU signs
of conv1/3/5 and linear1/2, and the pooled max-pool + ReLU outputs of conv2/4/6 (argmax index or
zero/non-zero).  If |g_gpu - g_tf| is at fp32 accumulation level while |g_tf - g_64| carries the
whole gap, the gap is decision flips at near-zero pre-activations / near-tied windows.

  python tools/flip_census.py            (prints a table; profiles/r02*/flip_census.txt)
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "fl-distributed-delay_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from oracle import model_ref as MR  # noqa: E402
from oracle import oracle as O  # noqa: E402

DEV = "cuda:0"
GROUP = 1 << 20


def rel(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def pool_idx(z):
    """2x2 max-pool argmax (first max in row-major window order, torch's rule) -> [N,C,PH,PW]."""
    N, C, H, W = z.shape
    PH, PW = H // 2, W // 2
    w = z[:, :, :2 * PH, :2 * PW].reshape(N, C, PH, 2, PW, 2).permute(0, 1, 2, 4, 3, 5)
    w = w.reshape(N, C, PH, PW, 4)
    return torch.argmax(w, -1)      # torch.argmax returns the first maximal index


def gather(z, idx):
    N, C, PH, PW = idx.shape
    rows = 2 * torch.arange(PH).view(1, 1, PH, 1) + (idx >> 1)
    cols = 2 * torch.arange(PW).view(1, 1, 1, PW) + (idx & 1)
    return z[torch.arange(N).view(N, 1, 1, 1), torch.arange(C).view(1, C, 1, 1), rows, cols]


def forward(P, x, y, noise, forced=None):
    """PerformantNet1 forward + CE(mean) in P's dtype.  forced = the GPU's decisions (dict of
    masks / argmax), or None: own decisions.  Returns (loss, decisions)."""
    (w1, b1, w2, b2, w3, b3, w4, b4, w5, b5, w6, b6, l1w, l1b, l2w, l2b, l3w, l3b) = P
    dec = {}

    # the GPU stores post-dropout activations, so its masks include the dropout keep bits: own
    # decisions are taken the same way (sign & keep)
    def relu(z, key, nz=None):
        m = (z > 0) if forced is None else forced[key]
        if forced is None and nz is not None:
            m = m & (nz > 0)
        dec[key] = m
        return z * m.to(z.dtype)

    def pool(z, key, nz):
        idx = pool_idx(F.relu(z)) if forced is None else forced[key]
        dec[key] = idx
        p = gather(z, idx)
        m = ((p > 0) & (nz > 0)) if forced is None else forced[key + "m"]
        dec[key + "m"] = m
        return p * m.to(z.dtype)

    h = relu(F.conv2d(x, w1, b1, padding=2), "a1")
    h = pool(F.conv2d(h, w2, b2, padding=2), "i1", noise[0]) * noise[0]
    h = relu(F.conv2d(h, w3, b3, padding=2), "a3")
    h = pool(F.conv2d(h, w4, b4, padding=2), "i2", noise[1]) * noise[1]
    h = relu(F.conv2d(h, w5, b5, padding=2), "a5")
    h = (pool(F.conv2d(h, w6, b6, padding=2), "i3", noise[2]) * noise[2]).reshape(x.shape[0], -1)
    h = relu(F.linear(h, l1w, l1b), "e1", noise[3]) * noise[3]
    h = relu(F.linear(h, l2w, l2b), "e2", noise[4]) * noise[4]
    return F.cross_entropy(F.linear(h, l3w, l3b), y), dec


def grad(theta, dtype, x, y, noise, forced=None):
    P = [torch.tensor(a, dtype=dtype, requires_grad=True)
         for a in MR.split_flat(theta.astype(np.float64 if dtype == torch.float64 else np.float32))]
    loss, dec = forward(P, x.to(dtype), y, [nz.to(dtype) for nz in noise], forced)
    loss.backward()
    return torch.cat([p.grad.reshape(-1) for p in P]).double().numpy(), dec


def gpu_case(theta, x, y, index):
    from flsim.engine import PN1Engine, worker_table
    n = x.shape[0]
    groups = -(-n // 128)
    eng = PN1Engine(DEV, chunk_workers=groups)
    th = torch.from_numpy(theta.copy()).to(DEV)
    eng.begin_epoch(th)
    loss = torch.zeros(groups, device=DEV)
    wt = worker_table([(0, index + b * GROUP, 0) for b in range(groups)], DEV)
    eng.run_input(th, x.to(DEV), y.to(DEV), wt, 0, True, loss)
    S = torch.zeros(eng.P, device=DEV)
    eng.end_epoch(S)
    torch.cuda.synchronize()
    NS = groups * 128
    W = lambda i, shp, dt=torch.float32: eng.workspace_view(i, shp, dt).cpu()   # noqa: E731
    nchw = lambda a: a.permute(0, 3, 1, 2).contiguous()                          # noqa: E731
    ws = dict(a1=nchw(W(1, (NS, 34, 34, 48))), d1=nchw(W(3, (NS, 18, 18, 48))),
              a3=nchw(W(4, (NS, 20, 20, 96))), d2=nchw(W(6, (NS, 11, 11, 96))),
              a5=nchw(W(7, (NS, 13, 13, 192))), d3=W(9, (NS, 9408)).reshape(NS, 192, 7, 7),
              e1=W(10, (NS, 512)), e2=W(11, (NS, 256)),
              i1=nchw(W(19, (NS, 18, 18, 48), torch.uint8)).long(),
              i2=nchw(W(20, (NS, 11, 11, 96), torch.uint8)).long(),
              i3=nchw(W(21, (NS, 7, 7, 192), torch.uint8)).long())
    sl = slice(0, n)
    forced = dict(a1=ws["a1"][sl] > 0, a3=ws["a3"][sl] > 0, a5=ws["a5"][sl] > 0,
                  e1=ws["e1"][sl] > 0, e2=ws["e2"][sl] > 0,
                  i1=ws["i1"][sl], i2=ws["i2"][sl], i3=ws["i3"][sl],
                  i1m=ws["d1"][sl] > 0, i2m=ws["d2"][sl] > 0, i3m=ws["d3"][sl] > 0)
    return S.cpu().numpy().astype(np.float64), forced


def noise_for(index, n):
    groups = -(-n // 128)
    per = [MR.dropout_noise(0, 0, index + b * GROUP, 128, torch.float64) for b in range(groups)]
    return [torch.cat([p[s] for p in per])[:n] for s in range(len(per[0]))]


def flips(dec, ref):
    """Decision disagreements per layer; for the pooled layers an element counts when the
    argmax or the zero/non-zero outcome differs (dropped elements excluded by the mask)."""
    out = {}
    for k in ("a1", "a3", "a5", "e1", "e2"):
        out[k] = int((dec[k] != ref[k]).sum())
    for k in ("i1", "i2", "i3"):
        live = ref[k + "m"] | dec[k + "m"]
        out[k] = int(((dec[k] != ref[k]) & live).sum() + (dec[k + "m"] != ref[k + "m"]).sum())
    return out


def main():
    pool = O.make_pool(0)
    lut = O.normalize_lut()
    theta = MR.init_params(0)
    cases = [(1, 256, 2), (0, 256, 2), (2, 256, 2), (0, 256, 1), (1048577, 128, 2), (0, 128, 1)]
    print("index  n  seed | gpu-vs-tf  gpu-vs-64  cpu32-vs-64 | flips gpu vs fp64 "
          "(a1 i1 a3 i2 a5 i3 e1 e2) | flips cpu32 vs fp64")
    for index, n, seed in cases:
        rs = np.random.RandomState(seed)
        idx = rs.randint(0, pool[0].shape[0], n)
        x = torch.from_numpy(lut[pool[0][idx]])
        y = torch.from_numpy(pool[1][idx])
        noise = noise_for(index, n)
        g_gpu, forced = gpu_case(theta, x, y, index)
        g_tf, _ = grad(theta, torch.float64, x, y, noise, forced)
        g_64, d64 = grad(theta, torch.float64, x, y, noise)
        g_32, d32 = grad(theta, torch.float32, x, y, noise)
        fg = flips(forced, d64)
        fc = flips(d32, d64)
        order = ("a1", "i1", "a3", "i2", "a5", "i3", "e1", "e2")
        print(f"{index:7d} {n:3d} {seed:4d} | {rel(g_gpu, g_tf):.2e}  {rel(g_gpu, g_64):.2e}  "
              f"{rel(g_32, g_64):.2e} | {' '.join(str(fg[k]) for k in order)} | "
              f"{' '.join(str(fc[k]) for k in order)}", flush=True)


if __name__ == "__main__":
    main()
