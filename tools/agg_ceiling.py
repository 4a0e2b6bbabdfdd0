"""Streaming ceilings at the aggregation paths' own sizes (GPU box): what a plain torch stream of the
same bytes reaches on this MI355X, to set the server-step kernels' fractions of 8 TB/s against.

  python tools/agg_ceiling.py [--iters 50]

Paths (bench.py's `aggregation` / `aggregation_stream` records, profiles/r05/configs):
  stream   k_agg_stream_reg after the all-reduce, PerformantNet1 P: 156.7 MB on a plain epoch,
           reads 4P, writes 3P floats (S_t, p, m, v -> p, m, v) -- ceiling: copy_ of the same
           bytes, and torch's own Adam-like ops over P
  fused    k_slab_step, PerformantNet1 (2.11 GB) and vgg11 (2.26 GB) / general order (2.16 GB): the
           weight-gradient slabs are read once, p, m, v written (~98 % reads) -- ceiling: torch.sum
           of the same bytes (a pure read stream) and copy_ of the same bytes
Prints one JSON line per case: GB/s and the fraction of 8 TB/s.
"""
import argparse
import json

import torch

PEAK = 8000.0


def timed(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3     # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    dev = "cuda:0"
    out = []

    def rec(case, nbytes, us, note):
        gbs = nbytes / (us * 1e-6) / 1e9
        out.append(dict(case=case, bytes=int(nbytes), us=round(us, 2), gbs=round(gbs, 1),
                        frac=round(gbs / PEAK, 4), note=note))
        print(json.dumps(out[-1]), flush=True)

    # stream size: P = 5,596,090 floats (PerformantNet1), 7P floats moved
    P = 5_596_090
    a = torch.randn(P * 7 // 2, device=dev)
    b = torch.empty_like(a)
    rec("stream_copy", 2 * a.numel() * 4, timed(lambda: b.copy_(a), args.iters),
        "copy_ of 3.5P floats each way (7P moved), the stream's byte count")
    p, m, v, s = (torch.randn(P, device=dev) for _ in range(4))

    def adam_like():        # torch's own ops for the same update (several launches)
        m.mul_(0.9).add_(s, alpha=0.1)
        v.mul_(0.999).addcmul_(s, s, value=0.001)
        p.addcdiv_(m, v.sqrt().add_(1e-8), value=-1e-3)
    rec("stream_torch_adam_ops", 7 * P * 4, timed(adam_like, args.iters),
        "torch's Adam-like ops over P: the stream's 7P bytes priced at their total time")
    del a, b, p, m, v, s
    torch.cuda.empty_cache()
    # fused sizes
    for case, nbytes in (("fused_pn1", 2_106_327_594), ("fused_vgg11", 2_257_906_160),
                         ("fused_general_order", 2_160_423_130)):
        n = nbytes // 4
        x = torch.randn(n, device=dev)
        rec(case + "_sum", n * 4, timed(lambda: x.sum(), args.iters), "torch.sum: pure read stream")
        half = torch.empty(n // 2, device=dev)
        rec(case + "_copy", (n // 2) * 8, timed(lambda: half.copy_(x[: n // 2]), args.iters),
            "copy_ of half the bytes each way")
        del x, half
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
