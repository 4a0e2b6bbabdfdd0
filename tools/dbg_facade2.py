"""Debug: which worker keys / batch sizes disagree with the oracle (GPU box)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "fl-distributed-delay_amd"), os.path.join(REPO, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

import test_gpu_facade as T  # noqa: E402
from oracle import model_ref as MR  # noqa: E402
from oracle import oracle as O  # noqa: E402

pool = O.make_pool(0)
th0 = MR.init_params(0)


def rel(a, b):
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))


def oracle(x, y, i, train):
    if train:
        return T._oracle_grad(th0, [(x, y, i, 0)], torch.float64)[0]
    params = [torch.tensor(a, dtype=torch.float64, requires_grad=True)
              for a in MR.split_flat(th0.astype(np.float64))]
    MR.fwd_bkwd(params, x.to(torch.float64), y, None)
    return torch.cat([p.grad.reshape(-1) for p in params]).numpy()


for idx, n, train in ((1048577, 128, True), (1, 256, False), (0, 256, False), (2, 256, True),
                      (1, 256, True), (0, 256, True), (3, 384, True), (0, 384, True)):
    from FL.agents import Worker
    from flsim.engine import PN1_SHAPES, PN1_SIZES
    model, central = T._fresh_central()
    w = Worker(nn.CrossEntropyLoss())
    w.index = idx
    model.train(train)
    w.model = model
    x, y = T._batch(pool, n, 2)
    grads, loss = w.fwd_bkwd(x.to(T.DEV), y.to(T.DEV))
    g = torch.cat([t.reshape(-1) for t in grads]).cpu().numpy().astype(np.float64)
    go = oracle(x, y, idx, train)
    off = 0
    worst = []
    for (name, _), sz in zip(PN1_SHAPES, PN1_SIZES):
        worst.append((round(rel(g[off:off + sz], go[off:off + sz]), 6), name))
        off += sz
    print(idx, n, train, "total", rel(g, go), sorted(worst)[-4:], flush=True)
