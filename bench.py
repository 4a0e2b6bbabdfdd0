"""bench.py -- simulated worker-steps/s of the FL server loop (BASELINE.json metric).

  python bench.py [--gpus N --steps K --warmup W]
  (N > 1: python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1
           --master-port P bench.py --gpus N --steps K --warmup W)

Workload (SURVEY 8d, config C3 headline line): n_workers = 1024, delay = 50, --throttle,
PerformantNet1, 128 samples per worker-step, synthetic CIFAR-shaped u8 pool resident in HBM,
torch default init (seed 0), Adam lr 1e-3.  A "step" is one server epoch (main.py:126-188):
schedule, every computing worker's fwd/bwd (worker-batched HIP kernels), [one RCCL all-reduce],
fused cascade-mean + Adam.  value = executed worker-steps (128-sample fwd+bwd units, summed over
the job) / wall time of the K timed epochs (max over ranks).

Extra objects on the JSON line: roofline (dominant GEMM kernel, HIP events recorded by
libflsim.so on its launch stream over the timed region), aggregation (the fused
rule()+Adam kernel's algorithmic HBM GB/s), cpu_baseline (the oracle's CPU port of the
reference loop on this host, bounded sample, rank 0 at N = 1 only).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (REPO, os.path.join(REPO, "fl-distributed-delay_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "simulated worker-steps/sec (node) @1024 workers, delay 50; aggregation HBM GB/s"
MFMA_F32_PEAK_TFLOPS = 157.3     # MI355X_MICROARCH.md: fp32 matrix (v_mfma_f32_16x16x4_f32)
# the split-bf16 GEMMs (gemm_x6.h) issue six bf16 products per fp32 product on the bf16 matrix
# cores (~2.5 PF/s dense, MI355X_MICROARCH.md): their fp32-equivalent peak
MFMA_X6_PEAK_TFLOPS = 2500.0 / 6
# probe names of the GEMMs that run on gemm_x6_kernel (pn1_net.hip, vgg_net.hip): the forwards
# and the linear weight gradients.  Every data gradient runs on the fp32 MFMA since round 5, every
# conv weight gradient since round 6
X6_KERNELS = {f"conv{i}_fwd" for i in range(2, 7)} | {"linear1_fwd", "linear1_wgrad"}
VGG_X6_KERNELS = {f"vgg_conv{i}_fwd" for i in range(1, 9)} | \
    {f"vgg_linear{i}_{p}" for i in (1, 2) for p in ("fwd", "wgrad")}
HBM_PEAK_GBPS = 8000.0           # MI355X_MICROARCH.md: HBM3E spec


def _load_traffic():
    """HBM bytes per launch from the PMC passes of tools/gpu_profile.sh (FETCH_SIZE x 2 per the
    gfx950 correction + WRITE_SIZE, MI355X_MICROARCH.md), written by tools/pmc_traffic.py into
    profiles/traffic.json.  {kernel: {"bytes_per_launch": B, "source": "..."}}; {} if absent."""
    path = os.path.join(REPO, "profiles", "traffic.json")
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return {}


TRAFFIC = _load_traffic()


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--n_workers", type=int, default=1024)
    ap.add_argument("--delay", type=int, default=50)
    ap.add_argument("--no-throttle", action="store_true")
    ap.add_argument("--delays", choices=["reference", "heterogeneous"], default="reference",
                    help="reference: one slow worker (n-1) with --delay; heterogeneous: configs[3] "
                         "spec (10%% slow workers, geometric delays up to 1000)")
    ap.add_argument("--chunk", type=int, default=128,
                    help="workers per worker-batched launch (128 = 16,384 samples, the largest the "
                         "32-bit index budget allows; fastest for every model, profiles/r01e)")
    ap.add_argument("--model", choices=["PerformantNet1", "vgg11", "vgg11_bn"],
                    default="PerformantNet1",
                    help="PerformantNet1 (main.py:97, the metric's model), vgg11 (configs[4]: "
                         "--model vgg11 --n_workers 4096 --delay 1000) or vgg11_bn")
    ap.add_argument("--configs0-epochs", type=int, default=3,
                    help="epochs of configs[0] (n=10, d=50) timed by the CPU baseline")
    ap.add_argument("--no-tick-window", action="store_true",
                    help="do not pre-roll untimed epochs to put the first tick (t = delay) and the "
                         "epoch after it inside the timed window")
    ap.add_argument("--semantics", choices=["reference", "torch1", "independent"],
                    default="reference",
                    help="weight_ups entries: aliased S_t (the reference under torch 2.x), zero "
                         "stale entries (torch 1.x) or distinct per-worker gradients")
    ap.add_argument("--model_file", type=str, default=None,
                    help="warm start (main.py:98-100): a models.py state_dict, e.g. configs[1]'s "
                         "warm_start.pt from tools/make_warm_start.py")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-stream", action="store_true",
                    help="skip timing the post-all-reduce server step (k_agg_stream) after the "
                         "timed window at N = 1")
    ap.add_argument("--no-probe", action="store_true")
    ap.add_argument("--force-dist", action="store_true",
                    help="run the N > 1 code path at world size 1 (launch under torchrun "
                         "--nproc-per-node 1): process group init, the per-epoch all-reduce of "
                         "[S_t | losses] (RCCL with --backend nccl) and the streaming server step "
                         "after it, instead of the fused single-GPU step")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                    help="torch.distributed backend for N > 1 (nccl = RCCL over xGMI). gloo is for "
                         "rehearsing the N > 1 path with several ranks on one GPU (slow collective)")
    return ap.parse_args()


def host_cpu_info():
    """CPU model, logical CPUs this job may run on, the cgroup CPU quota, and the physical cores
    among the allowed CPUs; threads = the physical cores (capped by the quota when one is set)."""
    aff = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else \
        list(range(os.cpu_count() or 1))
    model, phys, cur = None, set(), {}
    try:
        with open("/proc/cpuinfo") as f:
            for line in f.read().split("\n") + [""]:
                if not line.strip():
                    if cur.get("processor") is not None and int(cur["processor"]) in set(aff):
                        phys.add((cur.get("physical id", "0"), cur.get("core id", cur["processor"])))
                    cur = {}
                    continue
                k, _, v = line.partition(":")
                cur[k.strip()] = v.strip()
                if k.strip() == "model name" and model is None:
                    model = v.strip()
    except OSError:
        pass
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    cores = len(phys) or len(aff)
    threads = cores if quota is None else max(1, min(cores, int(quota)))
    return dict(cpu_model=model, logical_cpus_allowed=len(aff), physical_cores_allowed=cores,
                cgroup_cpu_quota=quota, omp_num_threads=os.environ.get("OMP_NUM_THREADS"),
                threads=threads)


def cpu_baseline(n, delay, throttle, model="PerformantNet1", configs0_epochs=3):
    """The oracle's CPU port of the reference loop on this host's cores:
      1. one FULL epoch 0 of the bench workload: every computing worker's fwd_bkwd
         (agents.py:32-40, sequential, accumulating into the shared gradient), rule() =
         torch.stack(entries).mean(0) per tensor over the aliased entries (main.py:23-25) and one
         torch.optim.Adam step (agents.py:9-21) -> executed worker-steps / s;
      2. configs[0]: n = 10, delay 50, no throttle, the port's whole server loop for a few epochs
         -> per-epoch time and worker-steps / s."""
    from oracle import model_ref as MR
    from oracle import oracle as O
    info = host_cpu_info()
    torch.set_num_threads(info["threads"])
    pool = O.make_pool(0)
    sim = MR.OracleSim(n, delay=delay, throttle=throttle, pool=pool, model=model)
    sched = O.schedule(n, O.reference_delays(n, delay), throttle, 1)
    ks = O.worker_k_sequence(0, n, 1)[0]
    active = np.nonzero(sched.computes[0])[0]
    items = [(0, int(i), int(ks[i])) for i in active]
    params = [torch.tensor(a, requires_grad=True) for a in MR.split_flat(sim.theta, model)]
    opt = torch.optim.Adam(params, lr=1e-3)
    sim.grad_of(sim.theta, items[:1])          # warm the CPU kernels
    t0 = time.perf_counter()
    g, _ = sim.grad_of(sim.theta, items)
    gl = [torch.from_numpy(a) for a in MR.split_flat(g, model)]
    k = int(sched.c_t[0] + sched.s_t[0])
    fin = [torch.stack([x] * k).mean(0) for x in gl]
    for p, f in zip(params, fin):
        p.grad = f
    opt.step()
    dt = time.perf_counter() - t0
    # a second, shorter sample of the same per-worker loop (the first 128 of those workers) as a
    # repeat of the measurement: the CPU rate varies with the box and its neighbours
    nr = min(128, len(items))
    t2 = time.perf_counter()
    sim.grad_of(sim.theta, items[:nr])
    rep = dict(worker_steps=nr, value=round(nr / (time.perf_counter() - t2), 3))
    c0 = None
    if configs0_epochs:
        s0 = MR.OracleSim(10, delay=50, throttle=False, pool=pool, model=model)
        s0.epoch()                                   # warm
        ws0 = 0
        t1 = time.perf_counter()
        for _ in range(configs0_epochs):
            s0.epoch()
            ws0 += len(s0.trace[-1]["items"])
        d0 = time.perf_counter() - t1
        c0 = dict(workload="configs[0]: n_workers=10, delay=50, no throttle (epochs 1..%d)"
                  % configs0_epochs, worker_steps_per_s=round(ws0 / d0, 3),
                  s_per_epoch=round(d0 / configs0_epochs, 3))
    return dict(value=len(items) / dt, unit="worker-steps/s", cores=info["threads"], kind="port",
                sample=f"one full epoch 0 of the bench workload: {len(items)} {model} fwd_bkwd "
                       f"(n={n}, d={delay}, {'throttle' if throttle else 'no throttle'}) + rule() "
                       f"over the {k} entries + one Adam step; torch CPU, {info['threads']} threads, "
                       f"{dt:.1f} s",
                repeat=rep, host=info, configs0=c0)


def stream_step_probe(sim, iters=20):
    """The server step every N > 1 run ends its epochs with, timed on this GPU after the timed
    window (untimed for `value`): rule() + Adam from S_t in a buffer, the stream that follows the
    all-reduce (flsim_aggregate_adam_rule_push), on copies of the run's theta / m / v, for the
    reference's two entry lists at n = 1024: a plain throttled epoch (k = c_t = 512) and the tick
    epoch t = d (c_t = 512 + the stale S_{t-d}).  A tick epoch builds and all-reduces S_t in the
    FIFO slot it pushes (sim.py epoch), so its stream writes no second copy.  Bytes: SURVEY 8(d)
    4P (1 + stale + 6).  Launch times from the probe."""
    from flsim._lib import KernelProbe
    from flsim.engine import Rule
    P, dev = sim.P, sim.device
    S = torch.randn(sim.Ppad, device=dev, generator=torch.Generator(device=dev).manual_seed(1))
    S.mul_(1e-3)
    st = S.flip(0).contiguous()
    p, m, v = sim.theta.clone(), sim.m.clone(), sim.v.clone()
    out = {}
    for name, rule, so, nbytes in (
            ("plain_k512", Rule(512, [], c=512), None, 4 * P * 7),
            ("tick_k513_in_slot", Rule(513, [st], c=512), None, 4 * P * 8)):
        for _ in range(3):
            sim.engine.aggregate_rule(S, rule, p, m, v, max(sim.step, 1), S_out=so)
        torch.cuda.synchronize()
        pr = KernelProbe(capacity=4096)
        for _ in range(iters):
            sim.engine.aggregate_rule(S, rule, p, m, v, max(sim.step, 1), S_out=so)
        torch.cuda.synchronize()
        rec = pr.read().get("aggregate_adam")
        pr.close()
        if not rec:
            continue
        cnt, ms, _ = rec
        us = ms / cnt * 1e3
        out[name] = dict(avg_launch_us=round(us, 2), bytes=nbytes,
                         bytes_8d=4 * P * (7 + len(rule.arrays)),
                         achieved=round(nbytes / us / 1e3, 1), unit="GB/s",
                         frac=round(nbytes / us / 1e3 / HBM_PEAK_GBPS, 4),
                         frac_8d=round(4 * P * (7 + len(rule.arrays)) / us / 1e3 /
                                       HBM_PEAK_GBPS, 4))
    return dict(kernel="k_agg_stream_reg (rule() + Adam from S_t after the all-reduce)",
                bound="hbm", peak=HBM_PEAK_GBPS, **out) if out else None


def main():
    args = parse()
    # stdout carries exactly ONE line, the JSON result: RCCL prints a version banner on stdout when
    # its communicator starts (profiles/r05/bench_forcedist.json), so the process's stdout goes to
    # stderr and the result line is written to a saved copy of the original stdout
    sys.stdout.flush()
    result_fd = os.dup(1)
    os.dup2(2, 1)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world > 1:
        raise SystemExit(f"--gpus {args.gpus} != WORLD_SIZE {world}")
    dist_on = world > 1 or args.force_dist
    if args.force_dist and "MASTER_ADDR" not in os.environ:
        raise SystemExit("--force-dist: launch under torch.distributed.run (MASTER_ADDR unset)")
    if args.backend == "gloo":   # rehearsal: ranks may share the box's GPU(s)
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if dist_on:
        if args.backend == "nccl":
            torch.distributed.init_process_group("nccl", device_id=dev)
        else:
            torch.distributed.init_process_group("gloo")
    from flsim._lib import KernelProbe
    from flsim.sim import FLSimulation, load_model_file

    theta0 = buffers = None
    if args.model_file:
        theta0, buffers = load_model_file(args.model_file, args.model)
    throttle = not args.no_throttle
    delays = None
    if args.delays == "heterogeneous":
        from flsim.schedule import heterogeneous_delays
        delays = heterogeneous_delays(args.n_workers)
    sim = FLSimulation(args.n_workers, delay=args.delay, delays=delays, throttle=throttle,
                       chunk_workers=args.chunk, device=dev, model=args.model, theta0=theta0,
                       semantics=args.semantics, distributed=dist_on)
    if buffers:
        sim.engine.load_buffers(buffers)
    flop_per_ws = sim.engine.FLOP_PER_WORKER_STEP
    # untimed pre-roll so the timed window holds the first tick (t = delay: the slow worker's
    # stale entry S_{t-d} joins rule()) and the 1023-worker epoch after it, when that is cheap
    pre = 0
    if not args.no_tick_window and delays is None and 0 < args.delay <= 100:
        pre = max(0, args.delay - args.warmup - args.steps // 2)
    for _ in range(pre + args.warmup):
        sim.epoch(sync_loss=False)
    torch.cuda.synchronize()
    probe = None if args.no_probe else KernelProbe(capacity=64 * 1024)
    sim.time_collective = dist_on
    sim.rank_worker_steps = []
    if dist_on:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    # per-epoch device time from events on the compute stream (no host synchronisation in the
    # window): which timed epochs hold a tick and what the steady-state epochs alone achieve
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    t0 = time.perf_counter()
    evs[0].record()
    ws = 0
    for j in range(args.steps):
        sim.epoch(sync_loss=False)
        ws += int(sim.trace[-1].computes.sum())
        evs[j + 1].record()
    torch.cuda.synchronize()
    if dist_on:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    epoch_ms = [evs[j].elapsed_time(evs[j + 1]) for j in range(args.steps)]
    coll_ms = sim.collective_ms()
    rank_ws = int(sum(sim.rank_worker_steps))
    if dist_on:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    losses = sim.losses()
    rank_ws_all = [rank_ws]
    if dist_on:
        t = torch.tensor([rank_ws], device=dev, dtype=torch.int64)
        g = [torch.zeros_like(t) for _ in range(world)]
        torch.distributed.all_gather(g, t)
        rank_ws_all = [int(x.item()) for x in g]

    kern = probe.read() if probe else {}
    if probe:
        probe.close()
    # the rule() + Adam kernel of the timed epochs: the fused slab step at world = 1, the
    # streaming kernel after the all-reduce at world > 1 (general order: the _seq forms)
    agg_recs = {k: kern.pop(k) for k in ("slab_step", "slab_step_seq", "aggregate_adam",
                                         "aggregate_adam_seq", "slab_sum") if k in kern}
    agg_name = max((k for k in agg_recs if k != "slab_sum"), key=lambda k: agg_recs[k][1],
                   default=None)
    agg_rec = agg_recs.get(agg_name)
    roofline = None
    if kern:
        name, (cnt, ms, fl) = max(kern.items(), key=lambda kv: kv[1][1])
        avg_s = ms / cnt / 1e3
        achieved = fl / cnt / avg_s / 1e12
        gemm_ms = sum(v[1] for v in kern.values())
        gemm_fl = sum(v[2] for v in kern.values())
        x6 = name in X6_KERNELS or name in VGG_X6_KERNELS
        traffic = TRAFFIC.get(name) if args.model == "PerformantNet1" else None
        if traffic and traffic.get("math") != ("bf16x6" if x6 else "fp32"):
            traffic = None      # profiles/traffic.json was counted on the other kernel
        peak = MFMA_X6_PEAK_TFLOPS if x6 else MFMA_F32_PEAK_TFLOPS
        roofline = dict(bound="mfma", kernel=name, achieved=round(achieved, 2),
                        peak=round(peak, 1), unit="TFLOP/s",
                        frac=round(achieved / peak, 4),
                        math=("bf16x6 split on the bf16 MFMA (fp32-equivalent FLOP/s against "
                              "2.5 PF/s / 6)" if x6 else "fp32 MFMA"),
                        traffic=traffic["bytes_per_launch"] if traffic else None,
                        traffic_source=traffic["source"] if traffic else None,
                        launches=cnt, avg_launch_ms=round(ms / cnt, 4),
                        alg_flop_per_launch=fl / cnt,
                        all_gemms=dict(achieved=round(gemm_fl / (gemm_ms / 1e3) / 1e12, 2),
                                       share_of_step=round(gemm_ms / 1e3 / elapsed, 3),
                                       executed_tflop=round(gemm_fl / 1e12, 3)),
                        per_kernel={k: dict(launches=c, avg_ms=round(m / c, 4),
                                            tflops=round(f / (m / 1e3) / 1e12, 1))
                                    for k, (c, m, f) in sorted(kern.items())})
        # chunks of <= FLSIM_CONCURRENT_BWD samples (default 2048: configs[1]) run each weight
        # gradient on a second stream beside its data gradient, and FLSIM_PIPELINE=1 overlaps a
        # chunk's forward with the previous chunk's backward: the per-kernel durations then
        # include the other stream's share of the chip
        conc = int(os.environ.get("FLSIM_CONCURRENT_BWD", "2048"))
        roofline["overlapped_streams"] = bool(
            (args.model == "PerformantNet1" and sim.engine.max_samples <= conc) or
            os.environ.get("FLSIM_PIPELINE", "0") != "0")
    agg = None
    if agg_rec:
        cnt, ms, byts = agg_rec
        gbps = byts / (ms / 1e3) / 1e9
        kname = {"slab_step": "k_slab_step (fused slab reduction + rule() + Adam)",
                 "slab_step_seq": "k_slab_step (fused, general entry order)",
                 "aggregate_adam": "k_agg_stream (rule() + Adam from S_t)",
                 "aggregate_adam_seq": "k_agg_stream (general entry order)"}[agg_name]
        # profiles/traffic.json is measured on the default workload (PerformantNet1, n = 1024,
        # one GPU): only borrowed for that workload and the same kernel
        same = args.model == "PerformantNet1" and delays is None and not dist_on and \
            args.n_workers == 1024
        traffic = TRAFFIC.get(agg_name) if same else None
        agg = dict(kernel=kname, probe=agg_name, bound="hbm", achieved=round(gbps, 1),
                   peak=HBM_PEAK_GBPS, unit="GB/s", frac=round(gbps / HBM_PEAK_GBPS, 4),
                   launches=cnt, avg_launch_us=round(ms / cnt * 1e3, 2),
                   alg_bytes_per_launch=int(byts / cnt),
                   traffic=traffic["bytes_per_launch"] if traffic else None,
                   traffic_source=traffic["source"] if traffic else None,
                   ticks_in_window=sum(1 for p in sim.trace[-args.steps:] if p.stale))
        if traffic and traffic.get("trace_avg_ns"):
            # the same kernel timed by the rocprofv3 kernel trace of that profile (no event
            # packets around it): context for `achieved`, which stays the live measurement
            rus = traffic["trace_avg_ns"] / 1e3
            agg.update(rocprof_avg_launch_us=round(rus, 2))

    # the timed epochs one by one: a tick epoch (t % d == 0: the slow worker computes and its
    # stale entry joins rule()) and the epoch after it (every fast worker computes) are marked;
    # steady_state = the other epochs alone
    window = []
    for j, plan in enumerate(sim.trace[-args.steps:]):
        prev = sim.trace[-args.steps + j - 1] if len(sim.trace) > args.steps - j else None
        window.append(dict(t=int(plan.t), worker_steps=int(plan.computes.sum()),
                           ms=round(epoch_ms[j], 3), tick=bool(plan.stale),
                           after_tick=bool(prev is not None and prev.stale)))
    steady = [w for w in window if not w["tick"] and not w["after_tick"]]
    steady_state = None
    if steady:
        sw, sms = sum(w["worker_steps"] for w in steady), sum(w["ms"] for w in steady)
        steady_state = dict(epochs=len(steady), worker_steps=sw,
                            worker_steps_per_s=round(sw / (sms / 1e3), 3),
                            note="job worker-steps of the timed epochs that are neither a tick "
                                 "nor the epoch after one / their device time on rank 0")
    # SURVEY 8(d)'s aggregation bytes for the same launches: 4P (1 + distinct stale + 3 + 3), the
    # rule() + Adam traffic without the slab reduction the fused step also streams
    agg8d = None
    if agg_rec and agg_name in ("slab_step", "slab_step_seq"):
        P = sim.P
        ticks = [w for w in window if w["tick"]]
        cnt, ms, _ = agg_rec
        b8 = 4.0 * P * (1 + 6) * cnt + 4.0 * P * sum(len({src for _, src in p.stale})
                                                     for p in sim.trace[-args.steps:])
        agg8d = dict(kernel=agg["kernel"], bytes_basis="SURVEY 8(d): 4P(1 + distinct stale + 6)",
                     alg_bytes_per_launch=int(b8 / cnt), avg_launch_us=agg["avg_launch_us"],
                     achieved=round(b8 / (ms / 1e3) / 1e9, 1), unit="GB/s",
                     frac=round(b8 / (ms / 1e3) / 1e9 / HBM_PEAK_GBPS, 4),
                     ticks_in_window=len(ticks),
                     note="the fused launch also streams the weight-gradient slabs "
                          "(aggregation.alg_bytes_per_launch); this is the rule()+Adam share "
                          "priced at the whole launch time")
    agg_stream = None
    if not dist_on and probe is not None and args.model == "PerformantNet1" and not args.no_stream:
        agg_stream = stream_step_probe(sim)

    value = ws / elapsed
    cpu = None
    if rank == 0 and not dist_on and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.n_workers, args.delay, throttle, args.model, args.configs0_epochs)
    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 3), "unit": "worker-steps/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f32",
            # fp32 in, fp32 accumulate; the k-contiguous convolution GEMMs split each fp32 operand
            # into three bf16 parts and sum six exact partial products on the bf16 matrix cores
            # (gemm_x6.h): fp32 accuracy, not a reduced-precision mode
            "math": "bf16x6 split of the fp32 operands, fp32 accumulate (conv2-6 forwards, "
                    "linear1 forward and weight gradient; VGG forwards and linear weight "
                    "gradients); fp32 MFMA for the rest: every data gradient and every conv "
                    "weight gradient",
            "data": f"synthetic: seeded CIFAR-shaped u8 pool in HBM, "
                    + (f"{args.model} warm-started from {os.path.basename(args.model_file)}"
                       if args.model_file else f"models.py-init {args.model}")
                    + " (no network for CIFAR10)",
            "config": {"workload": f"FL server epochs, n_workers={args.n_workers}, "
                                   + (f"delay={args.delay}" if delays is None else
                                      "heterogeneous delays (configs[3] spec)")
                                   + f", throttle={throttle}, {args.model}, "
                                   + (f"{args.semantics} entries, "
                                      if args.semantics != "reference" else "")
                                   + "128 samples/worker-step, Adam lr 1e-3",
                       "executed_worker_steps": ws, "chunk_workers": args.chunk,
                       "timed_epochs": [sim.trace[-args.steps].t, sim.trace[-1].t],
                       "backend": (args.backend if dist_on else None),
                       "world_size": (torch.distributed.get_world_size() if dist_on else 1),
                       "force_dist": bool(args.force_dist),
                       "parallelism": f"workers sharded over {world} GPU(s), "
                                      f"{'1 RCCL all-reduce/step' if dist_on and args.backend == 'nccl' else '1 gloo all-reduce/step (rehearsal)' if dist_on else 'no collective'}"},
            # executed GEMM FLOPs of this rank (the probe's per-launch counts: conv6 skips its
            # never-pooled border) / wall time / the fp32 MFMA peak (the bf16x6 GEMMs count their
            # fp32-equivalent FLOPs, so this can pass 1); the nominal SURVEY 8d count beside it
            "mfma_efficiency_whole_step": (round(roofline["all_gemms"]["executed_tflop"] /
                                                 (elapsed * MFMA_F32_PEAK_TFLOPS), 4)
                                           if roofline else None),
            "nominal_mfma_efficiency": round(value * flop_per_ws / 1e12 /
                                             (MFMA_F32_PEAK_TFLOPS * world), 4),
            "roofline": roofline,
            "aggregation": agg,
            "aggregation_8d": agg8d,
            "aggregation_stream": agg_stream,
            "window": window,
            "steady_state": steady_state,
            "collective": (dict(backend=args.backend,
                                per_epoch_ms=[round(x, 3) for x in coll_ms],
                                mean_ms=round(float(np.mean(coll_ms)), 3),
                                bytes_per_epoch=4 * int(sim.comm.numel()))
                           if coll_ms else None),
            "rank_worker_steps": rank_ws_all,
            "cpu_baseline": cpu,
            "gpu_vs_cpu": round(value / cpu["value"], 1) if cpu else None,
            "last_loss": losses[-1] if losses else None,
        }
        with os.fdopen(result_fd, "w") as out:
            out.write(json.dumps(line) + "\n")
    else:
        os.close(result_fd)
    if dist_on:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
