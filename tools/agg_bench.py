"""Microbenchmark of the fused aggregation+Adam kernel vs entry count c (debug helper)."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "fl-distributed-delay_amd")]
import torch
from flsim.engine import PN1Engine
dev = "cuda:0"
eng = PN1Engine(dev, chunk_workers=1)
P = eng.P
S = torch.randn(P, device=dev) * 1e-2
st = torch.randn(P, device=dev) * 1e-2
p = torch.randn(P, device=dev); m = torch.zeros(P, device=dev); v = torch.zeros(P, device=dev)
for c, ns in [(1, 0), (16, 0), (512, 0), (512, 1), (1023, 1)]:
    stale = [st] * ns
    for _ in range(3):
        eng.aggregate_adam(S, c, stale, p, m, v, 1)
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        eng.aggregate_adam(S, c, stale, p, m, v, 1)
    e1.record(); torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 20 * 1e3
    byts = 4 * P * (1 + ns + 6)
    print(f"c={c:5d} ns={ns} {us:8.1f} us  {byts/us/1e3:8.1f} GB/s")
# plain copy reference: read 4 write 3 arrays
a = [torch.randn(P, device=dev) for _ in range(7)]
e0.record()
for _ in range(20):
    a[4].copy_(a[0]); a[5].copy_(a[1]); a[6].copy_(a[2])
e1.record(); torch.cuda.synchronize()
us = e0.elapsed_time(e1) / 20 * 1e3
print(f"3 copies (6 streams) {us:.1f} us  {6*4*P/us/1e3:.1f} GB/s")
