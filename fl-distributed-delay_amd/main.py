"""Drop-in for the reference's main.py (main.py:37-212) on MI355X.

Same flags and defaults (main.py:38-53): --n_workers --n_epochs --batch_size --learning_rate
--delay --model_file --throttle.  The training loop (main.py:126-188) runs as flsim.sim
.FLSimulation: host schedule, worker-batched HIP forward/backward, fused rule()+Adam; with
`torchrun --nproc-per-node N` the computing workers are sharded over N GPUs with one RCCL
all-reduce per epoch.  'Avg. Loss' per epoch (main.py:185) goes to --log (JSONL; tensorboard is
not installed) and stdout.

Differences forced by the environment: the data is a seeded synthetic CIFAR-shaped
pool (no network for CIFAR10); RNG streams are seeded (--seed) and dropout / sampling use the
counter-based spec; test-accuracy evaluation (main.py:196-210) is not part of the hot path yet.
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)

import torch  # noqa: E402


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument('--n_workers', type=int, default=5, help='number of FL workers')
    p.add_argument('--n_epochs', type=int, default=1000, help='number of train epochs')
    p.add_argument('--batch_size', type=int, default=128, help='samples per worker-step')
    p.add_argument('--learning_rate', type=float, default=0.001, help='Adam learning rate')
    p.add_argument('--delay', type=int, default=100, help='delay in between slow worker')
    p.add_argument('--model_file', type=str, help='path to model to load (pretrained)')
    p.add_argument('--throttle', action='store_true', help='gradient throttling')
    # build flags
    p.add_argument('--seed', type=int, default=0)
    p.add_argument('--semantics', default='reference', choices=['reference', 'torch1'],
                   help='stale entry = S_{t-d} (torch>=2 aliasing) or zeros (torch 1.x)')
    p.add_argument('--no-dropout', action='store_true')
    p.add_argument('--chunk', type=int, default=32, help='workers per worker-batched launch')
    p.add_argument('--log', type=str, default=None, help='JSONL scalar log (Avg. Loss)')
    return p.parse_args(argv)


def main(argv=None):
    args = parse(argv)
    if args.batch_size != 128:
        raise SystemExit("the HIP engine is built for --batch_size 128 (the reference default)")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if not torch.cuda.is_available():
        raise SystemExit("no HIP device: flsim has no CPU path")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        torch.distributed.init_process_group("nccl", device_id=dev)
    rank = torch.distributed.get_rank() if world > 1 else 0
    from flsim.sim import FLSimulation, default_theta
    theta0 = default_theta(args.seed)
    if args.model_file is not None:                       # main.py:98-100
        from FL.models import PerformantNet1
        m = PerformantNet1()
        m.load_state_dict(torch.load(args.model_file, map_location="cpu", weights_only=True))
        theta0 = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
    if rank == 0:
        print(dev)
    sim = FLSimulation(args.n_workers, delay=args.delay, throttle=args.throttle,
                       lr=args.learning_rate, seed=args.seed, semantics=args.semantics,
                       dropout=not args.no_dropout, chunk_workers=args.chunk, device=dev,
                       theta0=theta0)
    log = open(args.log, "w") if (args.log and rank == 0) else None
    t0 = time.time()
    for t in range(args.n_epochs):
        loss = sim.epoch()
        if rank == 0:
            rec = {"tag": "Avg. Loss", "value": loss, "step": t, "wall": time.time() - t0,
                   "executed_worker_steps": int(sim.trace[-1].computes.sum())}
            if log:
                log.write(json.dumps(rec) + "\n")
                log.flush()
            if t % 10 == 0 or t == args.n_epochs - 1:
                print(f"epoch {t} Avg. Loss {loss:.5f}", flush=True)
    if log:
        log.close()
    if rank == 0:
        print('Done training')
    if world > 1:
        torch.distributed.destroy_process_group()
    return sim


if __name__ == '__main__':
    main()
