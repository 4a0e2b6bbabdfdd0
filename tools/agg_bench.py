"""Microbenchmark of the post-all-reduce server step (flsim_aggregate_adam_rule_push: rule() + Adam
from S_t in a buffer [+ the FIFO slot write]) at PerformantNet1's P, for the stream variants
(FLSIM_AGG_G = 0: LDS-staged k_agg_stream; 1, 2: register-array stream with 1 / 2 float4 groups per
thread).  Bytes are SURVEY 8(d)'s: 4P (1 + distinct stale + 3 + 3) [+ 4P for the slot write].

  python tools/agg_bench.py [--iters 50]

FLSIM_AGG_G acts only in a lab build of the library (make LAB=1, csrc/common.h): point FLSIM_LIB at
one to compare the variants; the product build runs its default stream.
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "fl-distributed-delay_amd")]
import torch  # noqa: E402

from flsim.engine import PN1_SIZES, Rule, aggregate_rule  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    dev = "cuda:0"
    P = sum(PN1_SIZES)
    S = torch.randn(P + 64, device=dev) * 1e-2
    st = torch.randn(P + 64, device=dev) * 1e-2
    slot = torch.empty(P + 64, device=dev)
    p = torch.randn(P + 64, device=dev)
    m = torch.zeros(P + 64, device=dev)
    v = torch.zeros(P + 64, device=dev)
    res = []
    for G in ("0", "1", "2"):
        os.environ["FLSIM_AGG_G"] = G
        for c, ns, out in [(512, 0, False), (1023, 0, False), (512, 1, False), (512, 1, True)]:
            rule = Rule(c + ns, [st] * ns, c=c)
            so = slot if out else None
            for _ in range(3):
                aggregate_rule(S, rule, p, m, v, 1, PN1_SIZES, S_out=so)
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                aggregate_rule(S, rule, p, m, v, 1, PN1_SIZES, S_out=so)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / args.iters * 1e3
            byts = 4 * P * (1 + ns + 6 + (1 if out else 0))
            r = dict(G=int(G), c=c, stale=ns, fifo_write=out, us=round(us, 2), bytes=byts,
                     GBps=round(byts / us / 1e3, 1), frac=round(byts / us / 1e3 / 8000, 4))
            res.append(r)
            print(json.dumps(r), flush=True)
    # float4 copy reference: 3 copies = read 3 + write 3 arrays of P floats
    a = [torch.randn(P, device=dev) for _ in range(6)]
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.iters):
        a[3].copy_(a[0])
        a[4].copy_(a[1])
        a[5].copy_(a[2])
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / args.iters * 1e3
    print(json.dumps(dict(reference="3 torch copies (6 streams)", us=round(us, 2),
                          GBps=round(6 * 4 * P / us / 1e3, 1))), flush=True)


if __name__ == "__main__":
    main()
