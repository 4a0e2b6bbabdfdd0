"""Debug: the facade's mixed-batch epoch, piece by piece against the oracle (GPU box)."""
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


for order in ((128, 256), (256, 128), (128, 128), (256, 256)):
    from FL.agents import Worker
    model, central = T._fresh_central()
    ws = [Worker(nn.CrossEntropyLoss()) for _ in range(2)]
    model.train()
    bs = [T._batch(pool, order[0], 1), T._batch(pool, order[1], 2)]
    snaps = []
    for i, (w, (x, y)) in enumerate(zip(ws, bs)):
        w.model = model
        grads, _ = w.fwd_bkwd(x.to(T.DEV), y.to(T.DEV))
        snaps.append(torch.cat([t.reshape(-1) for t in grads]).cpu().numpy().astype(np.float64))
    ga, _ = T._oracle_grad(th0, [(bs[0][0], bs[0][1], 0, 0)], torch.float64)
    gb, _ = T._oracle_grad(th0, [(bs[1][0], bs[1][1], 1, 0)], torch.float64)
    print(order, "call1 vs ga", rel(snaps[0], ga), "delta vs gb", rel(snaps[1] - snaps[0], gb),
          "total", rel(snaps[1], ga + gb), flush=True)
