"""The facade's one-call forward (flsim_pn1_fwd_rows: one 128-sample fwd_bkwd's forward + loss) in
isolation: no backward, no host work between calls but the launch.  Prints the mean time per call
(ms) with a host sync after every call (what Worker.fwd_bkwd does for its loss) and without.

  python tools/fwd1_bench.py [--calls 300]
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

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=300)
    args = ap.parse_args()
    from flsim.engine import PN1Engine, worker_table
    from flsim.sim import default_theta
    dev = torch.device("cuda", 0)
    eng = PN1Engine(dev, chunk_workers=8)
    theta = default_theta(0, "PerformantNet1").to(dev)
    eng.begin_epoch(theta)
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    x = torch.randn(128, 3, 32, 32, device=dev, generator=g)
    y = torch.randint(0, 10, (128,), device=dev, generator=g)
    wt = worker_table([(0, 0, 0)], dev)
    loss = torch.zeros(1, device=dev)
    out = {}
    for sync in (True, False):
        for _ in range(20):
            eng.forward_rows(theta, x, y, wt, 0, True, loss, 0, 0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.calls):
            eng.forward_rows(theta, x, y, wt, 0, True, loss, 0, 0)
            if sync:
                loss.item()
        torch.cuda.synchronize()
        out["sync" if sync else "async"] = (time.perf_counter() - t0) / args.calls * 1e3
    print(json.dumps(dict(metric="one-call forward (128 samples) ms per call", **out)))


if __name__ == "__main__":
    main()
