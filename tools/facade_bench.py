"""Throughput of the drop-in facade: the reference's server loop (main.py:126-188) written against
FL.agents / FL.models exactly as main.py calls them -- one Worker.fwd_bkwd per computing worker,
the slow worker's FIFO, Agg(rule) and Central.update_model -- at the bench workload (n = 1024,
delay 50, --throttle, 128-sample batches).

  python tools/facade_bench.py [--n_workers 1024] [--delay 50] [--epochs 3] [--batch_size 128]

Batches are drawn from a seeded u8 pool already on the device (the reference's
`images.to(device)` per batch is not timed: the bench measures the engine behind the API).
Prints one JSON line: executed worker-steps / s over the timed epochs (epoch 0 untimed warm-up).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (REPO, os.path.join(REPO, "fl-distributed-delay_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n_workers", type=int, default=1024)
    ap.add_argument("--delay", type=int, default=50)
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--batch_size", type=int, default=128)
    ap.add_argument("--model", default="PerformantNet1", choices=["PerformantNet1", "vgg11", "vgg11_bn"])
    args = ap.parse_args()
    from FL.agents import Agg, Central, Worker, rule
    from FL.models import PerformantNet1, vgg11, vgg11_bn
    from flsim.data import DevicePool

    dev = torch.device("cuda", 0)
    n, d, B = args.n_workers, args.delay, args.batch_size
    pool = DevicePool(dev, 0)
    lut = pool.lut
    npool = int(pool.imgs.shape[0])
    torch.manual_seed(0)
    model = {"vgg11": vgg11, "vgg11_bn": vgg11_bn}.get(args.model, PerformantNet1)().to(dev)
    central = Central(model, torch.optim.Adam(model.parameters(), lr=0.001))
    workers = [Worker(nn.CrossEntropyLoss()) for _ in range(n)]
    agg = Agg(rule)
    rs = np.random.RandomState(0)
    gen = torch.Generator(device=dev)
    gen.manual_seed(0)
    pesky, window, gone = [], 0, False
    timed_ws, timed_s, per_epoch = 0, 0.0, []
    for t in range(args.epochs):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        weight_ups, losses, ws = [], [], 0
        model.train()
        for i in range(n):
            rs.randint(0, n)                                     # main.py:138's draw
            idx = torch.randint(0, npool, (B,), device=dev, generator=gen)
            x = lut[pool.imgs[idx].long()].float()
            y = pool.labels[idx].long()
            if i == n - 1:                                       # main.py:150-166
                gone = False
                ups = None
                if t == 0 or t % d == 0:
                    workers[i].model = central.model
                    ups, _ = workers[i].fwd_bkwd(x, y)
                    ws += 1
                    pesky.append(ups)
                    ups = pesky.pop(0) if t > 0 else None
                if ups is not None:
                    weight_ups.append(ups)
                    gone = True
            elif window <= 0:                                    # main.py:167-178
                workers[i].model = central.model
                ups, lv = workers[i].fwd_bkwd(x, y)
                ws += 1
                weight_ups.append(ups)
                losses.append(lv)
                window = 1 if gone else 2
            if window > 0:
                window -= 1
        central.update_model(agg.rule(weight_ups))               # main.py:184,188
        avg = float(np.mean(losses))
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        per_epoch.append(dict(t=t, worker_steps=ws, s=round(dt, 4), loss=avg))
        if t > 0:
            timed_ws += ws
            timed_s += dt
    print(json.dumps({"metric": "facade worker-steps/s (FL.agents reference loop)",
                      "value": round(timed_ws / timed_s, 2) if timed_s else None,
                      "unit": "worker-steps/s", "model": args.model, "n_workers": n, "delay": d, "batch_size": B,
                      "timed_epochs": args.epochs - 1, "epochs": per_epoch}), flush=True)


if __name__ == "__main__":
    main()
