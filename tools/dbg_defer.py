"""Diagnostic (GPU box): per-tensor differences of the facade's epoch gradient after two
fwd_bkwd calls, deferred chunk backward (FLSIM_FACADE_CHUNK=128) against a backward per call (0),
and of each against the fp64 oracle (not teacher-forced).

  python tools/dbg_defer.py
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (os.path.join(REPO, "tests"), REPO, os.path.join(REPO, "fl-distributed-delay_amd")):
    sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402


def run(defer, calls):
    os.environ["FLSIM_FACADE_CHUNK"] = defer
    from FL.agents import Central, Worker
    from FL.models import PerformantNet1
    torch.manual_seed(0)
    model = PerformantNet1().to("cuda:0")
    central = Central(model, torch.optim.Adam(model.parameters(), lr=0.001))
    ws = [Worker(nn.CrossEntropyLoss()) for _ in range(len(calls))]
    model.train()
    out = []
    for w, (x, y) in zip(ws, calls):
        w.model = model
        grads, lv = w.fwd_bkwd(x.cuda(), y.cuda())
        out.append(float(lv))
    g = torch.cat([t.reshape(-1) for t in grads]).double().cpu().numpy()
    del central
    return g, out


def main():
    from flsim.engine import PN1_SHAPES
    from oracle import oracle as O
    pool = O.make_pool(0)
    lut = O.normalize_lut()
    rs = np.random.RandomState(5)
    calls = []
    for _ in range(2):
        idx = rs.randint(0, pool[0].shape[0], 128)
        calls.append((torch.from_numpy(lut[pool[0][idx]]), torch.from_numpy(pool[1][idx])))
    ga, la = run("0", calls)
    gb, lb = run("128", calls)
    print("losses", la, lb, la == lb)
    off = 0
    for name, shp in PN1_SHAPES:
        n = int(np.prod(shp))
        a, b = ga[off:off + n], gb[off:off + n]
        print(f"{name:16s} rel {np.linalg.norm(a - b) / np.linalg.norm(b):.3e}  "
              f"max {np.abs(a - b).max():.3e}")
        off += n
    print("whole", np.linalg.norm(ga - gb) / np.linalg.norm(gb))


if __name__ == "__main__":
    main()
