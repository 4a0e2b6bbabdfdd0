"""Write configs[1]'s warm start (tests/golden/warm_n10.npz, the sha-pinned short oracle
pre-training of tests/golden/make_warm_start_n10.py) as a models.py PerformantNet1 state_dict:
the `--model_file warm_start.pt` file main.py:98-100 / bench.py --model_file load.

  python tools/warm_start_file.py [--out gpurun_out/warm_start_n10.pt]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "fl-distributed-delay_amd"),
                os.path.join(REPO, "tests", "golden")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/warm_start_n10.pt")
    args = ap.parse_args()
    from FL.models import PerformantNet1
    from flsim.engine import split_views
    from make_warm_start_n10 import dequantise
    w = np.load(os.path.join(REPO, "tests", "golden", "warm_n10.npz"))
    theta = torch.from_numpy(dequantise(w["codes"], w["scales"]))
    m = PerformantNet1()
    with torch.no_grad():
        for p, v in zip(m.parameters(), split_views(theta)):
            p.copy_(v)
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    torch.save(m.state_dict(), args.out)
    print("wrote", args.out)


if __name__ == "__main__":
    main()
