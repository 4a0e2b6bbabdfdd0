"""Debug helper: vgg11_bn forward decisions of the GPU vs an fp64 forward (argmax / ReLU)."""
import sys
import numpy as np
import torch
import torch.nn.functional as F
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/tests")
sys.path.insert(0, "/root/repo/fl-distributed-delay_amd")
from oracle import oracle as O, model_ref as MR  # noqa: E402
from test_gpu_vgg_bn import _run  # noqa: E402
from flsim.engine import VGG11BNEngine  # noqa: E402

pool = O.make_pool(0)
for item in [(0, 0, 0), (0, 1, 2)]:
    sim = MR.OracleSim(4, delay=2, pool=pool, dropout=False, model="vgg11_bn")
    eng, g, loss, stats = _run(sim.theta, [item], False, pool)
    ids = {n: j for j, n in enumerate(VGG11BNEngine.WORKSPACE)}
    P = [torch.tensor(a) for a in MR.split_flat(sim.theta.astype(np.float64), "vgg11_bn")]
    x, y = sim.batch(*item, dtype=torch.float64)
    h = x
    j = 0
    pools = {0: ("i1", 16), 1: ("i2", 8), 3: ("i4", 4), 5: ("i6", 2), 7: ("i8", 1)}
    zs = {}
    for v in MR.VGG_CFG:
        if v == "M":
            continue
        cw, cb, gw, gb = P[4 * j:4 * j + 4]
        z = F.conv2d(h, cw, cb, padding=1)
        zg = eng.workspace_view(ids[f"z{j}"], (128, z.shape[2], z.shape[3], z.shape[1])).cpu().double().permute(0, 3, 1, 2)
        mg = eng.workspace_view(ids[f"bmean{j}"], (1, z.shape[1])).cpu().double()
        ig = eng.workspace_view(ids[f"binv{j}"], (1, z.shape[1])).cpu().double()
        mu = z.mean((0, 2, 3)); var = z.var((0, 2, 3), unbiased=False)
        print(item, j, "z rel %.2e" % (float((zg - z).norm() / z.norm())),
              "mean abs %.2e" % float((mg[0] - mu).abs().max()),
              "invstd rel %.2e" % float(((ig[0] - 1 / torch.sqrt(var + 1e-5)) * torch.sqrt(var + 1e-5)).abs().max()),
              "min var %.3e" % float(var.min()), "max |mu|/std %.2e" % float((mu.abs() / var.sqrt()).max()))
        h = F.relu(F.batch_norm(z, None, None, gw, gb, True, 0.1, 1e-5))
        if j in pools:
            name, ps = pools[j]
            hp, arg = F.max_pool2d(h, 2, 2, return_indices=True)
            W = h.shape[3]
            loc = (arg // W % 2) * 2 + (arg % W % 2)
            ig8 = eng.workspace_view(ids[name], (128, ps, ps, h.shape[1]), torch.uint8).cpu().permute(0, 3, 1, 2).long()
            mism = ((loc != ig8) & (hp > 0)).sum().item()
            print("   pool argmax mismatches (nonzero max):", mism, "of", hp.numel())
            h = hp
        j += 1
