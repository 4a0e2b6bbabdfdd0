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
    ap.add_argument("--cpu-sample", type=int, default=160,
                    help="worker-steps in the CPU sample (~10-30 s of host work)")
    ap.add_argument("--semantics", choices=["reference", "torch1", "independent"],
                    default="reference",
                    help="weight_ups entries: aliased S_t (the reference under torch 2.x), zero "
                         "stale entries (torch 1.x) or distinct per-worker gradients")
    ap.add_argument("--model_file", type=str, default=None,
                    help="warm start (main.py:98-100): a models.py state_dict, e.g. configs[1]'s "
                         "warm_start.pt from tools/make_warm_start.py")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-probe", action="store_true")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                    help="torch.distributed backend for N > 1 (nccl = RCCL over xGMI). gloo is for "
                         "rehearsing the N > 1 path with several ranks on one GPU (slow collective)")
    return ap.parse_args()


def cpu_baseline(n, delay, throttle, n_ws, model="PerformantNet1"):
    """The oracle's CPU port of the reference loop (torch CPU, all host cores of this job): the
    first n_ws fwd_bkwd of epoch 0 (agents.py:32-40, sequential, accumulating), then rule()
    (torch.stack(...).mean(0) per tensor, main.py:23-25) over those entries and one Adam step
    (agents.py:9-21).  Returns executed worker-steps / s."""
    from oracle import model_ref as MR
    from oracle import oracle as O
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    pool = O.make_pool(0)
    sim = MR.OracleSim(n, delay=delay, throttle=throttle, pool=pool, model=model)
    sched = O.schedule(n, O.reference_delays(n, delay), throttle, 1)
    ks = O.worker_k_sequence(0, n, 1)[0]
    active = np.nonzero(sched.computes[0])[0][:n_ws]
    items = [(0, int(i), int(ks[i])) for i in active]
    params = [torch.tensor(a, requires_grad=True) for a in MR.split_flat(sim.theta, model)]
    opt = torch.optim.Adam(params, lr=1e-3)
    sim.grad_of(sim.theta, items[:1])          # warm the CPU kernels
    t0 = time.perf_counter()
    g, _ = sim.grad_of(sim.theta, items)
    gl = [torch.from_numpy(a) for a in MR.split_flat(g, model)]
    fin = [torch.stack([x] * len(items)).mean(0) for x in gl]
    for p, f in zip(params, fin):
        p.grad = f
    opt.step()
    dt = time.perf_counter() - t0
    return dict(value=len(items) / dt, unit="worker-steps/s", cores=threads, kind="port",
                sample=f"{len(items)} {model} fwd_bkwd of epoch 0 (n={n}, d={delay}, "
                       f"{'throttle' if throttle else 'no throttle'}) + rule() over them + one "
                       f"Adam step; torch CPU, {threads} threads, {dt:.1f} s")


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world > 1:
        raise SystemExit(f"--gpus {args.gpus} != WORLD_SIZE {world}")
    if args.backend == "gloo":   # rehearsal: ranks may share the box's GPU(s)
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
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
                       semantics=args.semantics)
    if buffers:
        sim.engine.load_buffers(buffers)
    flop_per_ws = sim.engine.FLOP_PER_WORKER_STEP
    for _ in range(args.warmup):
        sim.epoch(sync_loss=False)
    torch.cuda.synchronize()
    probe = None if args.no_probe else KernelProbe(capacity=64 * 1024)
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ws = 0
    for _ in range(args.steps):
        sim.epoch(sync_loss=False)
        ws += int(sim.trace[-1].computes.sum())
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    losses = sim.losses()

    kern = probe.read() if probe else {}
    if probe:
        probe.close()
    agg_rec = kern.pop("aggregate_adam", None)
    roofline = None
    if kern:
        name, (cnt, ms, fl) = max(kern.items(), key=lambda kv: kv[1][1])
        avg_s = ms / cnt / 1e3
        achieved = fl / cnt / avg_s / 1e12
        gemm_ms = sum(v[1] for v in kern.values())
        gemm_fl = sum(v[2] for v in kern.values())
        traffic = TRAFFIC.get(name) if args.model == "PerformantNet1" else None
        roofline = dict(bound="mfma", kernel=name, achieved=round(achieved, 2),
                        peak=MFMA_F32_PEAK_TFLOPS, unit="TFLOP/s",
                        frac=round(achieved / MFMA_F32_PEAK_TFLOPS, 4),
                        traffic=traffic["bytes_per_launch"] if traffic else None,
                        traffic_source=traffic["source"] if traffic else None,
                        launches=cnt, avg_launch_ms=round(ms / cnt, 4),
                        alg_flop_per_launch=fl / cnt,
                        all_gemms=dict(achieved=round(gemm_fl / (gemm_ms / 1e3) / 1e12, 2),
                                       share_of_step=round(gemm_ms / 1e3 / elapsed, 3)),
                        per_kernel={k: dict(launches=c, avg_ms=round(m / c, 4),
                                            tflops=round(f / (m / 1e3) / 1e12, 1))
                                    for k, (c, m, f) in sorted(kern.items())})
    agg = None
    if agg_rec:
        cnt, ms, byts = agg_rec
        gbps = byts / (ms / 1e3) / 1e9
        # profiles/traffic.json is measured on the default (PerformantNet1) workload
        traffic = TRAFFIC.get("aggregate_adam") if args.model == "PerformantNet1" else None
        agg = dict(kernel="k_aggregate_adam", bound="hbm", achieved=round(gbps, 1),
                   peak=HBM_PEAK_GBPS, unit="GB/s", frac=round(gbps / HBM_PEAK_GBPS, 4),
                   launches=cnt, avg_launch_us=round(ms / cnt * 1e3, 2),
                   alg_bytes_per_launch=int(byts / cnt),
                   traffic=traffic["bytes_per_launch"] if traffic else None,
                   traffic_source=traffic["source"] if traffic else None)
        if traffic and traffic.get("trace_avg_ns"):
            # the same launch timed by the rocprofv3 kernel trace of that profile (no event
            # packets around it): context for `achieved`, which stays the live measurement
            rus = traffic["trace_avg_ns"] / 1e3
            agg.update(rocprof_avg_launch_us=round(rus, 2),
                       rocprof_frac=round(byts / cnt / (rus * 1e-6) / 1e9 / HBM_PEAK_GBPS, 4))

    value = ws / elapsed
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.n_workers, args.delay, throttle, args.cpu_sample, args.model)
    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 3), "unit": "worker-steps/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f32",
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
                       "parallelism": f"workers sharded over {world} GPU(s), "
                                      f"{'1 RCCL all-reduce/step' if world > 1 and args.backend == 'nccl' else '1 gloo all-reduce/step (rehearsal)' if world > 1 else 'no collective'}"},
            "mfma_efficiency_whole_step": round(value * flop_per_ws / 1e12 /
                                                (MFMA_F32_PEAK_TFLOPS * world), 4),
            "roofline": roofline,
            "aggregation": agg,
            "cpu_baseline": cpu,
            "gpu_vs_cpu": round(value / cpu["value"], 1) if cpu else None,
            "last_loss": losses[-1] if losses else None,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
