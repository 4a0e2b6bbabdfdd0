"""Drop-in for the reference's main.py (main.py:37-212) on MI355X.

Same flags and defaults (main.py:38-53): --n_workers --n_epochs --batch_size --learning_rate
--delay --model_file --throttle.  The training loop (main.py:126-188) runs as flsim.sim
.FLSimulation: host schedule, worker-batched HIP forward/backward, fused rule()+Adam; with
`torchrun --nproc-per-node N` the computing workers are sharded over N GPUs with one RCCL
all-reduce per epoch.  'Avg. Loss' per epoch (main.py:185) goes to --log (JSONL; tensorboard is
not installed) and stdout.

Test accuracy every 100 epochs and at the end (main.py:190,196-210) runs on the device
(FLSimulation.evaluate, dropout off) and is logged as 'Avg. Test Accuracy' and 'Class 9 Test
Accuracy'.  --save_model writes saved_model_{t}.pt state_dicts every 100 epochs (main.py:192-194,
reference default off).  --checkpoint / --resume save and continue the whole simulation state.

Differences forced by the environment: without --data_dir the data is a seeded
synthetic CIFAR-shaped pool (no network for CIFAR10; --data_dir reads a local copy of the
CIFAR-10 binary distribution); RNG streams are seeded (--seed) and dropout / sampling use the
counter-based spec.
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
    p.add_argument('--semantics', default='reference', choices=['reference', 'torch1', 'independent'],
                   help='stale entry = S_{t-d} (torch>=2 aliasing), zeros (torch 1.x) or the slow '
                        "worker's own gradient with distinct per-worker entries (independent)")
    p.add_argument('--no-dropout', action='store_true')
    p.add_argument('--chunk', type=int, default=128,
                   help='workers per worker-batched launch (max 128 = 16,384 samples)')
    p.add_argument('--model', default='PerformantNet1', choices=['PerformantNet1', 'vgg11', 'vgg11_bn'],
                   help='models.py network (main.py:97 builds PerformantNet1; vgg11 = configs[4]; '
                        'vgg11_bn = models.py:106-108)')
    p.add_argument('--log', type=str, default=None,
                   help="JSONL scalar log ('Avg. Loss', 'Avg. Test Accuracy', 'Class 9 ...')")
    p.add_argument('--data_dir', type=str, default=None,
                   help='local cifar-10-batches-bin directory (default: synthetic pool)')
    p.add_argument('--eval_every', type=int, default=100, help='main.py:196 (0 = only at end)')
    p.add_argument('--save_model', action='store_true', help='main.py:192-194 saved_model_{t}.pt')
    p.add_argument('--checkpoint', type=str, default=None, help='write a resumable checkpoint')
    p.add_argument('--checkpoint_every', type=int, default=0)
    p.add_argument('--resume', type=str, default=None, help='continue from a checkpoint')
    return p.parse_args(argv)


def main(argv=None):
    args = parse(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if not torch.cuda.is_available():
        raise SystemExit("no HIP device: flsim has no CPU path")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        torch.distributed.init_process_group("nccl", device_id=dev)
    rank = torch.distributed.get_rank() if world > 1 else 0
    from flsim.sim import FLSimulation, default_theta, load_model_file
    theta0 = default_theta(args.seed, args.model)
    buffers = None
    if args.model_file is not None:                       # main.py:98-100
        theta0, buffers = load_model_file(args.model_file, args.model)
    if rank == 0:
        print(dev)
    pool = test_pool = None
    if args.data_dir:
        from flsim.data import load_cifar10_bin
        pool, test_pool = load_cifar10_bin(args.data_dir)
    sim = FLSimulation(args.n_workers, delay=args.delay, throttle=args.throttle,
                       lr=args.learning_rate, seed=args.seed, semantics=args.semantics,
                       dropout=not args.no_dropout, chunk_workers=args.chunk, device=dev,
                       theta0=theta0, pool=pool, test_pool=test_pool, model=args.model,
                       batch_size=args.batch_size)
    if buffers:
        sim.engine.load_buffers(buffers)
    if args.resume:
        sim.restore(args.resume)
    log = open(args.log, "a" if args.resume else "w") if (args.log and rank == 0) else None
    t0 = time.time()

    def emit(tag, value, t):
        if rank != 0:
            return
        rec = {"tag": tag, "value": value, "step": t, "wall": time.time() - t0}
        if log:
            log.write(json.dumps(rec) + "\n")
            log.flush()

    t = len(sim.trace) - 1
    for t in range(len(sim.trace), args.n_epochs):
        loss = sim.epoch()
        emit("Avg. Loss", loss, t)                                     # main.py:185
        if rank == 0 and (t % 10 == 0 or t == args.n_epochs - 1):
            print(f"epoch {t} Avg. Loss {loss:.5f}", flush=True)
        if args.save_model and t % 100 == 0 and t > 0 and rank == 0:   # main.py:192-194
            torch.save(sim.model_state_dict(), "saved_model_{}.pt".format(t))
        if args.eval_every and t % args.eval_every == 0 and t > 0:     # main.py:196-203
            acc, per = sim.evaluate()
            emit("Avg. Test Accuracy", acc, t)
            emit("Class 9 Test Accuracy", per[-1], t)
            if rank == 0:
                print(f"Accuracy of the network on the {len(sim._test.labels)} test images: "
                      f"{int(acc)} %", flush=True)
        if args.checkpoint and args.checkpoint_every and (t + 1) % args.checkpoint_every == 0 \
                and rank == 0:
            sim.save_checkpoint(args.checkpoint)
    acc, per = sim.evaluate()                                           # main.py:205-210
    emit("Avg. Test Accuracy", acc, t)
    emit("Class 9 Test Accuracy", per[-1], t)
    if rank == 0:
        print(f"Accuracy of the network on the {len(sim._test.labels)} test images: {int(acc)} %")
    if args.checkpoint and rank == 0:
        sim.save_checkpoint(args.checkpoint)
    if log:
        log.close()
    if rank == 0:
        print('Done training')
    if world > 1:
        torch.distributed.destroy_process_group()
    return sim


if __name__ == '__main__':
    main()
