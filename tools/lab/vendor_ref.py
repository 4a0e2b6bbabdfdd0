"""Reference points from the vendor libraries (rocBLAS/hipBLASLt via torch.matmul, MIOpen via
F.conv2d) for the PerformantNet1 GEMM shapes, fp32 (no TF32).  Development tool only."""
import time
import torch
import torch.nn.functional as F

torch.backends.cuda.matmul.allow_tf32 = False
torch.backends.cudnn.allow_tf32 = False
dev = "cuda"


def timeit(fn, iters=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


for (M, N, K, tag) in [(921600, 192, 1728, "conv6 fwd GEMM"), (4096 * 484, 96, 864, "conv4 fwd GEMM"),
                       (192, 1728, 921600, "conv6 wgrad GEMM"), (8192, 8192, 8192, "square 8192")]:
    a = torch.randn(M, K, device=dev)
    b = torch.randn(K, N, device=dev)
    ms = timeit(lambda: torch.matmul(a, b))
    print(f"matmul {tag:18s} {M}x{N}x{K}: {ms:8.3f} ms {2 * M * N * K / ms / 1e9:7.1f} TF/s", flush=True)
    del a, b

for (C, O, H, tag) in [(192, 192, 13, "conv6"), (96, 96, 20, "conv4"), (48, 48, 34, "conv2")]:
    x = torch.randn(2048, C, H, H, device=dev)
    w = torch.randn(O, C, 3, 3, device=dev)
    OH = H + 2
    fl = 2 * 2048 * OH * OH * O * C * 9
    ms = timeit(lambda: F.conv2d(x, w, padding=2))
    print(f"conv2d {tag} fwd N=2048: {ms:8.3f} ms {fl / ms / 1e9:7.1f} TF/s", flush=True)
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    y = F.conv2d(xr, wr, padding=2)
    g = torch.randn_like(y)
    ms = timeit(lambda: torch.autograd.grad(y, (xr, wr), g, retain_graph=True))
    print(f"conv2d {tag} bwd (dgrad+wgrad) N=2048: {ms:8.3f} ms {2 * fl / ms / 1e9:7.1f} TF/s", flush=True)
