"""Micro-benchmark of the fused server step (k_slab_step) on PerformantNet1's gradstate (GPU box):
the whole plan and each segment alone (FLSIM_STEP_UNITS), reduce-only and with rule() + Adam.

  python tools/step_bench.py
Prints per segment: units, slab MB, time (us), algorithmic GB/s.  Modes: ref (reference order,
k = 513), seq (k = 8100 with 72 stale entries among 6 arrays), c3 [T] (configs[3]'s epoch T).
The per-segment runs (FLSIM_STEP_UNITS, FLSIM_STEP_NO_INTERLEAVE) need a lab build of the library
(make LAB=1, csrc/common.h) under FLSIM_LIB.
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "fl-distributed-delay_amd")]
import torch  # noqa: E402

GEO = [(3, 4, 48, 48, 8192), (48, 48, 48, 432, 4096), (48, 48, 96, 432, 2048),
       (96, 96, 96, 864, 1024), (96, 96, 192, 864, 512), (192, 192, 192, 1728, 256)]
UNIT = 65536


def plan():
    """Mirror of slabstep.h plan_step for PerformantNet1's segments (pn1_net.hip)."""
    segs = []
    offs = [0, 1296, 1344, 22080, 22128, 63600, 63696, 146640, 146736, 312624, 312816, 644592,
            644784, 5461680, 5462192, 5593264, 5593520, 5596080, 5596090]
    j = 0
    for CI, CIP, CO, KP, ZW in GEO:
        segs.append((f"conv{j // 2 + 1}.w", ZW, CO * KP, False, CO * CI * 9))
        segs.append((f"conv{j // 2 + 1}.b", ZW, CO, True, CO))
        j += 2
    for name, Z, n in (("linear1.w", 8, 512 * 9408), ("linear1.b", 8, 512),
                       ("linear2.w", 64, 256 * 512), ("linear2.b", 64, 256),
                       ("linear3.w", 32, 2560), ("linear3.b", 32, 10)):
        segs.append((name, Z, n, True, n))
    out, u = [], 0
    segs = [(sg, o) for sg, o in zip(segs, offs)]
    iswide = [sg[3] and sg[2] % 4 == 0 and o % 4 == 0 and sg[4] % 32 == 0 and sg[2] >= 4096
              for sg, o in segs]
    cls = [0 if sg[2] < 4096 else (1 if iswide[i] else 2) for i, (sg, _) in enumerate(segs)]
    order = [i for c in range(3) for i in range(len(segs)) if cls[i] == c]
    for i in order:
        (name, Z, n, ident, numel), _ = segs[i]
        wide = iswide[i]
        tw = 1024 if wide else 256
        tiles = -(-n // tw)
        tf = tw * Z
        uf = UNIT // 4 if wide else UNIT
        if tf <= uf:
            tpu = max(1, min(uf // tf, tiles, 1 if wide else 4))
            units = -(-tiles // tpu)
        else:
            nz = -(-tf // uf)
            zc = (-(-Z // nz) + 3) // 4 * 4
            nz = -(-Z // zc)
            units = tiles * nz
        out.append((name, u, u + units, Z * n * 4, numel))
        u += units
    return out, u


def main():
    from flsim.engine import PN1Engine, Rule
    dev = "cuda:0"
    eng = PN1Engine(dev, chunk_workers=128)
    P = eng.P
    theta = torch.randn(P + 64, device=dev) * 0.05
    m = torch.zeros_like(theta)
    v = torch.zeros_like(theta)
    stale = torch.randn(P + 64, device=dev) * 1e-3
    eng.begin_epoch(theta)
    S = torch.zeros(P + 64, device=dev)
    segs, total = plan()
    mode = sys.argv[1] if len(sys.argv) > 1 else "ref"
    if mode == "seq":          # a configs[3]-like general order: k = 8100, 72 events, 6 arrays
        import numpy as np
        from flsim.engine import ProgramStager
        rs = np.random.RandomState(0)
        arrs = [torch.randn(P + 64, device=dev) * 1e-3 for _ in range(6)]
        pos = np.sort(rs.choice(8100, 72, replace=False))
        ev = list(zip(pos.tolist(), rs.randint(0, 6, 72).tolist()))
        rule = Rule(8100, arrs, events=ev, stager=ProgramStager(dev))
        print("seq program words", int(rule.c_rule.info[0]))
    elif mode == "c3":         # configs[3]'s own programs: the heterogeneous schedule's epoch T
        import numpy as np
        from flsim.engine import ProgramStager
        from flsim.schedule import Schedule, heterogeneous_delays
        T = int(sys.argv[2]) if len(sys.argv) > 2 else 3
        n = 16384
        sch = Schedule(n, heterogeneous_delays(n), True)
        for _ in range(T + 1):
            plan_t = sch.next_epoch()
        fast = np.nonzero(plan_t.fast)[0]
        sw = np.asarray([w for (w, _) in plan_t.stale])
        pos = np.searchsorted(fast, sw) + np.arange(len(sw))
        srcs = sorted({src for (_, src) in plan_t.stale})
        arr = [srcs.index(src) for (_, src) in plan_t.stale]
        arrs = [torch.randn(P + 64, device=dev) * 1e-3 for _ in srcs]
        rule = Rule(plan_t.c_t + plan_t.s_t, arrs, events=list(zip(pos.tolist(), arr)),
                    stager=ProgramStager(dev))
        print(f"configs[3] epoch {T}: k {plan_t.c_t + plan_t.s_t}, {len(arr)} stale entries, "
              f"{len(srcs)} arrays, {int(rule.c_rule.info[0])} macro words")
    else:
        rule = Rule(513, [stale], c=512)

    def timeit(fn, reps=20):
        fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / reps * 1e3

    full_red = timeit(lambda: eng.end_epoch(S))
    full_step = timeit(lambda: eng.server_step(None, rule, theta, m, v, 5))
    slab = sum(s[3] for s in segs)
    print(f"plan: {total} units, slabs {slab / 1e6:.1f} MB")
    print(f"FULL reduce-only {full_red:8.1f} us  {(slab + 4 * P) / full_red / 1e3:7.1f} GB/s")
    print(f"FULL step        {full_step:8.1f} us  {(slab + 4 * P * 7) / full_step / 1e3:7.1f} GB/s")
    os.environ["FLSIM_STEP_NO_INTERLEAVE"] = "1"
    t = timeit(lambda: eng.server_step(None, rule, theta, m, v, 5))
    os.environ.pop("FLSIM_STEP_NO_INTERLEAVE")
    print(f"FULL step, plan order (no interleave) {t:8.1f} us")
    for name, u0, u1, sb, numel in segs:
        os.environ["FLSIM_STEP_UNITS"] = f"{u0},{u1}"
        t = timeit(lambda: eng.server_step(None, rule, theta, m, v, 5))
        byts = sb + 4 * numel * 7
        print(f"{name:10s} units {u1 - u0:5d}  slab {sb / 1e6:7.1f} MB  {t:8.1f} us  "
              f"{byts / t / 1e3:7.1f} GB/s", flush=True)
    os.environ.pop("FLSIM_STEP_UNITS")


if __name__ == "__main__":
    main()
