"""FLSimulation: the server loop of main.py:126-188 on MI355X.

Per epoch t (one "server step"):
  1. schedule scan on the host (flsim_sched_epoch; main.py:137-181) and the dataset draws
     k_i = np.random.randint(0, n) for every worker (main.py:138, seeded stream);
  2. the workers that compute this epoch are split into contiguous blocks, one per rank
     (torch.distributed; one process per GPU), and each rank runs its block as worker-batched
     chunks of `chunk_workers` x 128 samples through the HIP forward/backward; all of them use
     theta_t, so their gradients simply add (agents.py:35) -- S_t;
  3. world > 1: ONE all-reduce (RCCL) of [S_t partial | per-worker losses | per-worker BatchNorm
     statistics (vgg11_bn)]; BatchNorm running buffers advance over every computing worker's
     call in worker order;
  4. a slow worker that computed stores S_t in its FIFO (main.py:156,161: the entry is an alias
     of the epoch's .grad tensors, so under torch >= 2 it holds S_t); popped entries (main.py:162)
     are the stale gradients S_{t-d};
  5. fused rule() + Adam on the device: c_t copies of S_t and the stale entries (main.py:184,188);
  6. 'Avg. Loss' = np.mean of the fast workers' losses (main.py:172,185).
"""
from __future__ import annotations

import os

import numpy as np
import torch

from .data import DevicePool, make_test_pool
from .engine import PN1_SIZES, ProgramStager, Rule, engine_class, padded, split_views
from .schedule import Schedule, reference_delays

SEMANTICS = ("reference", "torch1", "independent")
# checkpoint format: 2 records the model, the optimizer hyper-parameters and the throttle cap, and
# the reference's --delay 0 slow worker as DELAY_ZERO (restore() migrates format 1)
CKPT_FORMAT = "flsim-checkpoint-2"


def default_theta(seed=0, model="PerformantNet1"):
    """torch default init of the model (PerformantNet1 as main.py:97 builds it, or vgg11) under
    torch.manual_seed(seed) (CPU RNG), flattened in named_parameters order."""
    from FL import models
    torch.manual_seed(seed)
    m = models.PerformantNet1() if model == "PerformantNet1" else getattr(models, model)()
    return torch.cat([p.detach().reshape(-1) for p in m.parameters()])


def load_model_file(path, model="PerformantNet1"):
    """--model_file (main.py:49-50,98-100): `model.load_state_dict(torch.load(path))` on the
    models.py module, then the flat theta0 in named_parameters order and the module's buffers
    (vgg11_bn running statistics; empty for the others).  The file is a plain state_dict, so it
    is read with weights_only=True; a missing or mismatched key raises load_state_dict's
    RuntimeError exactly as the reference would."""
    from FL import models
    m = getattr(models, model)()
    m.load_state_dict(torch.load(path, map_location="cpu", weights_only=True))
    theta0 = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
    return theta0, dict(m.named_buffers())


class FLSimulation:
    def __init__(self, n_workers, delay=100, delays=None, throttle=False, lr=1e-3, seed=0,
                 semantics="reference", dropout=True, chunk_workers=128, device=None, theta0=None,
                 group=None, max_throttle=32, pool=None, betas=(0.9, 0.999), eps=1e-8,
                 engine=None, device_pool=None, test_pool=None, model="PerformantNet1",
                 fused=True, keep_S=False, batch_size=128, distributed=None,
                 collective="torch"):
        if semantics not in SEMANTICS:
            raise NotImplementedError(f"semantics {semantics!r} (supported: {SEMANTICS})")
        self.n = int(n_workers)
        if self.n < 1:
            raise ValueError("n_workers must be >= 1")
        self.delays = np.asarray(delays if delays is not None else reference_delays(self.n, delay),
                                 np.int32)
        self.delay_arg = delay
        self.throttle = bool(throttle)
        self.lr, self.betas, self.eps = float(lr), tuple(betas), float(eps)
        self.seed = int(seed)
        self.semantics = semantics
        self.dropout = bool(dropout)
        # fused: at world = 1 the epoch ends in ONE launch, slabs -> S_t -> rule() + Adam
        # (flsim_<net>_server_step); keep_S also writes S_t into comm[:P] (tests, debugging)
        self.fused = bool(fused)
        self.keep_S = bool(keep_S)
        # pipelined chunks (PN1), FLSIM_PIPELINE=1: off by default -- +0.4 % on the headline
        # (961 -> 965 worker-steps/s, profiles/r03d) but the per-kernel live timing then measures
        # overlapped kernels
        self.pipeline = os.environ.get("FLSIM_PIPELINE", "0") != "0"
        self.group = group
        self.model = model
        # --batch_size B (main.py:43-44): every worker-step is G = ceil(B/128) 128-sample groups
        # (the engine's unit; WorkerRec.pad = B, include/flsim.h), the last one padded
        self.batch_size = int(batch_size)
        if self.batch_size < 1:
            raise ValueError("batch_size must be >= 1")
        self.G = -(-self.batch_size // 128)
        if self.batch_size != 128 and semantics == "independent":
            raise NotImplementedError("independent entries with --batch_size != 128")
        dist = torch.distributed
        if dist.is_available() and dist.is_initialized():
            self.rank = dist.get_rank(group)
            self.world = dist.get_world_size(group)
        else:
            self.rank, self.world = 0, 1
        # distributed: the world > 1 code path (sharding, the one all-reduce per epoch, the
        # streaming server step after it).  Default: on iff world > 1; True at world = 1 runs that
        # path over a one-rank process group (bench.py --force-dist: RCCL on a single GPU)
        self.distributed = self.world > 1 if distributed is None else bool(distributed)
        if self.distributed and not (dist.is_available() and dist.is_initialized()):
            raise RuntimeError("distributed=True needs an initialised torch.distributed group")
        # the epoch's one all-reduce: "torch" = torch.distributed (RCCL with the nccl backend);
        # "flsim" = the C-ABI's flsim_allreduce_sum over RCCL (include/flsim.h), its unique id
        # shipped over the process group; "flsim-local" (world 1) = the C-ABI's one-rank
        # communicator, which never touches RCCL
        if collective not in ("torch", "flsim", "flsim-local"):
            raise ValueError(f"collective {collective!r}")
        if collective == "flsim-local" and self.world != 1:
            raise ValueError("collective='flsim-local' is the one-rank communicator")
        self.collective = collective
        self._comm = None
        if self.distributed and collective != "torch":
            from .comm import Comm
            if collective == "flsim":
                box = [Comm.unique_id() if self.rank == 0 else None]
                dist.broadcast_object_list(box, src=dist.get_global_rank(group, 0)
                                           if group is not None else 0, group=group)
                self._comm = Comm(self.world, self.rank, box[0])
            else:
                self._comm = Comm()
        self.device = torch.device(device) if device is not None else \
            torch.device("cuda", torch.cuda.current_device())
        # engine / device_pool are injectable only so tests can drive the sharding and
        # collective logic with a CPU stand-in (gloo); the product path always builds PN1Engine
        # a chunk never needs more workers than the run has (the workspace scales with it)
        self.engine = engine if engine is not None else \
            engine_class(model)(self.device, min(int(chunk_workers), self.n * self.G))
        if self.batch_size != 128 and getattr(self.engine, "STATS_PER_WORKER", 0):
            raise NotImplementedError("BatchNorm models: one BatchNorm batch is one 128-sample "
                                      "fwd_bkwd call (--batch_size 128)")
        self.pool = device_pool if device_pool is not None else \
            DevicePool(self.device, self.seed, pool)
        self.max_throttle = int(max_throttle)
        self.sched = Schedule(self.n, self.delays, self.throttle, max_throttle)
        self.rs = np.random.RandomState(self.seed)   # main.py:138 np.random stream
        P = self.engine.P
        self.P = P
        self.Ppad = padded(P)
        th = default_theta(self.seed, model) if theta0 is None else torch.as_tensor(theta0)
        self.theta = th.to(self.device, torch.float32).contiguous().clone()
        self.m = torch.zeros_like(self.theta)
        self.v = torch.zeros_like(self.theta)
        self.step = 0
        # [S_t | losses of the computing workers | their per-call BatchNorm statistics (vgg11_bn)]
        # -- one all-reduce per epoch when world > 1 (each rank fills only its workers' rows)
        self.nstat = int(getattr(self.engine, "STATS_PER_WORKER", 0))
        if self.nstat and semantics == "independent":
            raise NotImplementedError("independent entries with BatchNorm models")
        self.stats_off = self.Ppad + padded(self.n * self.G)
        self.comm = torch.zeros(self.stats_off + self.n * self.nstat, device=self.device)
        self._stager = ProgramStager(self.device)
        self.stale_store = {}     # epoch -> [slot tensor, refcount]
        self.free_slots = []
        self.trace = []
        self.loss_log = []        # per epoch: float (synced) or (device tensor, fast mask)
        self._test_src = test_pool  # (imgs, labels) of the test split, or None = synthetic
        self._test = None
        # measurement (bench.py): worker-steps this rank executed per epoch, and when enabled the
        # per-epoch collective bracketed by events on the compute stream (RCCL's own stream is
        # joined back into it by the blocking all_reduce, so the pair spans the collective and the
        # wait for the slowest rank)
        self.rank_worker_steps = []
        self.time_collective = False
        self.coll_events = []

    # ---------------------------------------------------------------------------------------------
    def _slot(self, n=None):
        """A FIFO slot of >= n floats (default Ppad): a released one when one is large enough."""
        n = self.Ppad if n is None else n
        for j in range(len(self.free_slots) - 1, -1, -1):
            if self.free_slots[j].numel() >= n:
                return self.free_slots.pop(j)
        slot = torch.empty(n, device=self.device)
        slot[self.P:].zero_()     # the [P, Ppad) padding and the tail enter the all-reduce
        return slot

    def _worker_table(self, t, workers, ks):
        """WorkerRec (t, i, k, 0) of this rank's computing workers, copied host->device from a
        pinned staging buffer (asynchronous: the host never waits for the GPU here).  With
        --batch_size B != 128 each worker is G records (t, i + g * 2^20, k, B), g < G."""
        G = self.G
        if G > 1 or self.batch_size != 128:
            workers = np.repeat(np.asarray(workers, np.int64), G)
            grp = np.tile(np.arange(G, dtype=np.int64), len(workers) // G)
        n = len(workers)
        if getattr(self, "_wt_cap", 0) < max(1, n):
            cap = max(1, n)
            pin = self.device.type == "cuda"
            self._wt_host = [torch.empty((cap, 4), dtype=torch.int32, pin_memory=pin)
                             for _ in range(2)]
            self._wt_dev = torch.empty((cap, 4), dtype=torch.int32, device=self.device)
            self._wt_ev = [None, None]
            self._wt_cap = cap
            self._wt_i = 0
        j = self._wt_i = self._wt_i ^ 1
        if self._wt_ev[j] is not None:
            self._wt_ev[j].synchronize()          # staging buffer j free again (2 epochs ago)
        h = self._wt_host[j][:n].numpy()
        h[:, 0] = t
        h[:, 2] = ks[workers]
        if G > 1 or self.batch_size != 128:
            h[:, 1] = workers + (grp << 20)
            h[:, 3] = self.batch_size
        else:
            h[:, 1] = workers
            h[:, 3] = 0
        dev = self._wt_dev[:n]
        if n:
            dev.copy_(self._wt_host[j][:n], non_blocking=True)
        if self.device.type == "cuda":
            ev = torch.cuda.Event()
            ev.record()
            self._wt_ev[j] = ev
        return dev

    def _reduce(self, buf):
        if self._comm is not None:
            self._comm.all_reduce_sum(buf)          # flsim_allreduce_sum (C-ABI, RCCL)
        else:
            torch.distributed.all_reduce(buf, group=self.group)

    def _all_reduce(self, buf):
        """The epoch's one collective (RCCL over xGMI: the nccl backend or the C-ABI's)."""
        if self.time_collective and self.device.type == "cuda":
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            self._reduce(buf)
            e1.record()
            self.coll_events.append((e0, e1))
        else:
            self._reduce(buf)

    def collective_ms(self):
        """Per-epoch collective times (ms) recorded since the last call (synchronises)."""
        if not self.coll_events:
            return []
        self.coll_events[-1][1].synchronize()
        out = [a.elapsed_time(b) for a, b in self.coll_events]
        self.coll_events = []
        return out

    def _rule(self, plan, stale):
        """weight_ups of this epoch as a Rule: k = c_t + s_t entries, the stale ones in append
        (worker-index) order; identical arrays (several FIFOs popping the same epoch) share one
        array index."""
        k = plan.c_t + plan.s_t
        order = self._entry_order(plan)
        if order is None:       # reference order: c_t copies of S_t, then the stale entries
            return Rule(k, stale, c=plan.c_t)
        uniq, ev = [], []
        for pos, a in zip(order[0], stale):
            j = next((q for q, u in enumerate(uniq) if u is a), None)
            if j is None:
                uniq.append(a)
                j = len(uniq) - 1
            ev.append((pos, j))
        return Rule(k, uniq, events=ev, stager=self._stager)

    @staticmethod
    def _entry_order(plan):
        """None when weight_ups is [S_t] * c_t followed by <= 8 stale entries (the reference:
        one slow worker, index n-1); else (positions of the stale entries in weight_ups, None):
        entries are appended in worker-index order (main.py:136-178)."""
        if not plan.stale:
            return None
        fast = np.nonzero(plan.fast)[0]
        sw = np.asarray([w for (w, _) in plan.stale], np.int64)
        if len(sw) <= 8 and (len(fast) == 0 or fast.max() < sw.min()):
            return None
        pos = np.searchsorted(fast, sw) + np.arange(len(sw))
        return [int(x) for x in pos], None

    def chunks(self, lo, hi):
        """[lo, hi) in the fewest launches of <= chunk_workers workers, sizes within one of each
        other (no short tail chunk running the GEMMs at low occupancy)."""
        n = hi - lo
        if n <= 0:
            return []
        k = -(-n // self.engine.chunk_workers)
        b = [lo + (j * n) // k for j in range(k + 1)]
        return list(zip(b[:-1], b[1:]))

    def shard(self, active):
        lo = (len(active) * self.rank) // self.world
        hi = (len(active) * (self.rank + 1)) // self.world
        return lo, hi

    def epoch(self, sync_loss=True):
        # raises IndexError like rule() on an empty weight_ups, ZeroDivisionError like main.py:158
        # under --delay 0
        plan = self.sched.next_epoch()
        t = plan.t
        ks = self.rs.randint(0, self.n, size=self.n)
        if self.semantics == "independent":
            return self._epoch_independent(plan, ks, sync_loss)
        active = np.nonzero(plan.computes)[0]
        lo, hi = self.shard(active)
        eng = self.engine
        G = self.G                               # 128-sample groups (units) per worker-step
        fused = self.fused and not self.distributed and hasattr(eng, "server_step")
        pushes = plan.pushed and self.semantics == "reference"
        # An epoch that pushes S_t onto the FIFO and ends with the streaming server step (world > 1,
        # or an engine without the fused step) builds S_t -- and all-reduces it -- straight in the
        # slot it pushes, a whole [S_t | losses] comm buffer: the stream then reads S_t from the slot
        # and writes no second copy (4P fewer HBM bytes at every tick).  BatchNorm runs
        # keep the shared buffer (their comm buffer also holds n x the per-call statistics).
        # (keep_S: S_t stays in comm[:P], where the caller reads it)
        in_slot = pushes and not fused and not self.nstat and not self.keep_S
        comm = self._slot(self.stats_off) if in_slot else self.comm
        S = comm[:self.P]
        losses = comm[self.Ppad:self.Ppad + len(active) * G]
        stats = comm[self.stats_off:self.stats_off + len(active) * self.nstat].view(
            len(active), self.nstat)
        if self.distributed:
            losses.zero_()
            stats.zero_()
        eng.begin_epoch(self.theta)
        wt = self._worker_table(t, active[lo:hi], ks)      # one async upload per epoch
        chunks = self.chunks(lo * G, hi * G)
        # several chunks: pipelined (chunk i's forward beside chunk i-1's backward, two
        # workspaces); the library joins the backward stream at end_epoch / server_step
        pipe = self.pipeline and len(chunks) > 1 and getattr(eng, "PIPELINE", False) and \
            not self.nstat
        for j, (c0, c1) in enumerate(chunks):
            if pipe:
                eng.run_chunk_async(self.theta, self.pool, wt[c0 - lo * G:c1 - lo * G], c1 - c0,
                                    self.n, self.seed, self.dropout, losses[c0:c1], j)
                continue
            kw = {"stats_out": stats[c0:c1]} if self.nstat else {}
            eng.run_chunk(self.theta, self.pool, wt[c0 - lo * G:c1 - lo * G], c1 - c0, self.n,
                          self.seed, self.dropout, losses[c0:c1], **kw)
        if not fused or self.keep_S:
            eng.end_epoch(S)
        self.rank_worker_steps.append(hi - lo)
        if self.distributed:
            end = self.stats_off + len(active) * self.nstat if self.nstat else \
                self.Ppad + len(active) * G
            self._all_reduce(comm[:end])
        if self.nstat:   # BatchNorm running buffers: every computing worker's call, in order
            eng.update_running(stats, len(active))
        push = None
        if pushes:
            n_push = int(sum(1 for i in range(self.n) if self.delays[i] != 0 and plan.computes[i]))
            push = comm if in_slot else self._slot()
            if fused and self.keep_S:
                push[:self.P].copy_(S)
            # otherwise the server step writes S_t into the slot in its own pass: the fused
            # slab step (world = 1) or the stream after the all-reduce (world > 1)
            self.stale_store[t] = [push, n_push]
        stale = []
        for (_, src) in plan.stale:
            if self.semantics == "reference":
                entry = self.stale_store[src]
                stale.append(entry[0])
            else:
                stale.append(None)
        self.step += 1
        rule = self._rule(plan, stale)
        hp = dict(lr=self.lr, betas=self.betas, eps=self.eps)
        if fused and not self.keep_S:
            eng.server_step(push, rule, self.theta, self.m, self.v, self.step, **hp)
        elif fused:
            eng.aggregate_rule(S, rule, self.theta, self.m, self.v, self.step, **hp)
        else:
            eng.aggregate_rule(S, rule, self.theta, self.m, self.v, self.step,
                               S_out=None if in_slot else push, **hp)
        for (_, src) in plan.stale:
            if self.semantics == "reference":
                entry = self.stale_store[src]
                entry[1] -= 1
                if entry[1] == 0:
                    self.free_slots.append(entry[0])
                    del self.stale_store[src]
        fast_pos = np.nonzero(plan.fast[active])[0]
        self.trace.append(plan)
        if sync_loss:
            lv = self._worker_losses(losses.detach().cpu().numpy())[fast_pos]
            val = float(np.mean(lv.astype(np.float32))) if len(lv) else float("nan")
            self.loss_log.append(val)
            return val
        self.loss_log.append((losses.detach().clone(), fast_pos))
        return None

    def _worker_losses(self, lv):
        """Per-worker CrossEntropyLoss(mean) from the per-group values (group sum / 128):
        sum over the worker's groups * 128 / B (agents.py:40's lossval per call)."""
        if self.G == 1 and self.batch_size == 128:
            return lv
        tot = lv.reshape(-1, self.G).astype(np.float64).sum(1)
        return (tot * 128.0 / self.batch_size).astype(np.float32)

    def _epoch_independent(self, plan, ks, sync_loss):
        """Independent-entry semantics: every weight_ups entry is a distinct
        per-worker gradient and a slow worker's FIFO holds its own gradient.  Slow workers with
        the same delay d tick together (t == 0 or t % d == 0) and pop together d epochs later, so
        their FIFO entries are kept as ONE slot per delay class holding the class's summed
        gradient: each class is one worker-batched launch, owned by rank d mod world.  The fast
        workers are sharded as usual.  Each rank adds the popped class slots it owns to its
        partial sum, so the one all-reduce combines the partial sums of all k entries; mean =
        sum / k, then the same Adam step, replicated."""
        from .schedule import DELAY_ZERO
        t = plan.t
        eng = self.engine
        active = np.nonzero(plan.computes)[0]
        slow_mask = self.delays[active] != 0
        fast, slow = active[~slow_mask], active[slow_mask]

        def dclass(i):
            d = int(self.delays[i])
            return 0 if d == DELAY_ZERO else abs(d)
        classes = {}
        for i in slow:
            classes.setdefault(dclass(i), []).append(int(i))
        own = [(d, ws) for d, ws in sorted(classes.items()) if d % self.world == self.rank]
        lo, hi = self.shard(fast)
        S = self.comm[:self.P]
        losses = self.comm[self.Ppad:self.Ppad + len(fast)]
        if self.distributed:
            losses.zero_()
        own_workers = np.asarray([i for _, ws in own for i in ws], np.int64)
        wt = self._worker_table(t, np.concatenate([own_workers, fast[lo:hi]]), ks)
        cw = self.engine.chunk_workers
        if getattr(self, "_slow_loss", None) is None or self._slow_loss.numel() < cw:
            self._slow_loss = torch.zeros(cw, device=self.device)
        off = 0
        for d, ws in own:                        # one FIFO slot per delay class (its sum)
            eng.begin_epoch(self.theta)
            n_ws = len(ws)
            k = -(-n_ws // cw)
            for j in range(k):
                c0, c1 = (j * n_ws) // k, ((j + 1) * n_ws) // k
                eng.run_chunk(self.theta, self.pool, wt[off + c0:off + c1], c1 - c0, self.n,
                              self.seed, self.dropout, self._slow_loss[:c1 - c0])
            slot = self._slot()
            eng.end_epoch(slot[:self.P])
            self.stale_store[(d, t)] = slot
            off += n_ws
        ns = off
        eng.begin_epoch(self.theta)
        for c0, c1 in self.chunks(lo, hi):
            eng.run_chunk(self.theta, self.pool, wt[ns + c0 - lo:ns + c1 - lo], c1 - c0, self.n,
                          self.seed, self.dropout, losses[c0:c1])
        eng.end_epoch(S)
        for (i, src) in plan.stale:              # popped entries, added once per class slot
            key = (dclass(int(i)), int(src))
            if key[0] % self.world == self.rank and key in self.stale_store:
                slot = self.stale_store.pop(key)
                S.add_(slot[:self.P])
                self.free_slots.append(slot)
        self.rank_worker_steps.append(hi - lo + len(own_workers))
        if self.distributed:
            self._all_reduce(self.comm[:self.Ppad + len(fast)])
        self.step += 1
        eng.aggregate_adam_sum(S, len(fast) + len(plan.stale), self.theta, self.m, self.v,
                               self.step, self.lr, self.betas, self.eps)
        self.trace.append(plan)
        if sync_loss:
            lv = losses.detach().cpu().numpy()
            val = float(np.mean(lv.astype(np.float32))) if len(lv) else float("nan")
            self.loss_log.append(val)
            return val
        self.loss_log.append((losses.detach().clone(), np.arange(len(fast))))
        return None

    def losses(self):
        out = []
        for e in self.loss_log:
            if isinstance(e, tuple):
                lv = self._worker_losses(e[0].cpu().numpy())[e[1]]
                out.append(float(np.mean(lv.astype(np.float32))) if len(lv) else float("nan"))
            else:
                out.append(e)
        self.loss_log = list(out)
        return out

    # ---------------------------------------------------------------------------------------------
    def evaluate(self):
        """util.print_test_accuracy (util.py:31-45) as main.py:190,196-210 uses it: the central
        model in eval mode (dropout off) over the whole test split, batches in order.  Returns
        (accuracy %, [per-class accuracy %] * 10).  The reference logs np.mean of the first as
        'Avg. Test Accuracy' and means the last class's entry as 'Class 9 Test Accuracy'
        (main.py:203 indexes the scalar util returns; here the per-class list exists)."""
        if self._test is None:
            src = self._test_src if self._test_src is not None else make_test_pool(self.seed)
            self._test = DevicePool(self.device, self.seed, src)
        pred = self.engine.evaluate(self.theta, self._test)
        labels = self._test.labels
        ok = (pred == labels)
        acc = 100.0 * int(ok.sum()) / int(labels.numel())
        per = []
        for c in range(10):
            sel = labels == c
            nc = int(sel.sum())
            per.append(100.0 * int((ok & sel).sum()) / nc if nc else float("nan"))
        return acc, per

    def model_state_dict(self):
        """The models.py module's state_dict (torch.save-compatible with the reference's
        main.py:98-100 / :192-194 load_state_dict / save); BatchNorm buffers follow their
        module's parameters, as nn.Module.state_dict orders them."""
        from collections import OrderedDict
        shapes = self.engine.SHAPES
        bufs = self.engine.buffer_state()
        out = OrderedDict()
        for (name, _), v in zip(shapes, split_views(self.theta, shapes)):
            out[name] = v.detach().cpu().clone()
            mod = name.rsplit(".", 1)[0]
            if name.endswith(".bias"):
                for bname, b in bufs:
                    if bname.rsplit(".", 1)[0] == mod:
                        out[bname] = b
        return out

    # -- checkpoint / resume ----------------------------------------------------------------------
    def checkpoint(self):
        """Everything needed to continue bit-for-bit: theta, Adam m/v/step, the epoch counter,
        the FIFO'd stale gradients still referenced, the loss log.  The schedule and the numpy
        k-draws are deterministic scans and are replayed on restore."""
        if self.semantics == "independent":
            raise NotImplementedError("checkpoint of the independent-entry semantics")
        return {
            "format": CKPT_FORMAT,
            "config": {"n": self.n, "delays": torch.from_numpy(self.delays.copy()),
                       "model": self.model,
                       "throttle": self.throttle, "seed": self.seed, "semantics": self.semantics,
                       "dropout": self.dropout, "lr": self.lr, "betas": list(self.betas),
                       "eps": self.eps, "max_throttle": self.max_throttle,
                       "batch_size": self.batch_size},
            "epoch": len(self.trace), "step": self.step,
            "theta": self.theta.detach().cpu(), "m": self.m.detach().cpu(),
            "v": self.v.detach().cpu(),
            "stale": {int(src): (slot[:self.P].detach().cpu(), int(rc))
                      for src, (slot, rc) in self.stale_store.items()},
            "loss_log": [float(x) for x in self.losses()],
            "buffers": dict(getattr(self.engine, "buffer_state", list)()),
        }

    def save_checkpoint(self, path):
        torch.save(self.checkpoint(), path)

    def restore(self, ck):
        """Resume from checkpoint() / save_checkpoint() output (a dict, or a path loaded with
        weights_only=True).  The simulation must be fresh and built with the same config."""
        if isinstance(ck, (str, bytes)) or hasattr(ck, "__fspath__"):
            ck = torch.load(ck, map_location="cpu", weights_only=True)
        fmt = ck.get("format")
        if fmt not in (CKPT_FORMAT, "flsim-checkpoint-1"):
            raise ValueError("not an flsim checkpoint")
        cfg = dict(ck["config"])
        mine = {"n": self.n, "throttle": self.throttle, "seed": self.seed,
                "semantics": self.semantics, "dropout": self.dropout, "model": self.model,
                "lr": self.lr, "betas": list(self.betas), "eps": self.eps,
                "max_throttle": self.max_throttle, "batch_size": self.batch_size}
        delays = cfg["delays"].numpy().astype(np.int32)
        if fmt == "flsim-checkpoint-1":
            # format 1 (round 1) had no model / optimizer / throttle-cap keys (they were the
            # defaults) and stored the slow worker of --delay 0 as 0 (now DELAY_ZERO)
            import warnings
            from .schedule import DELAY_ZERO
            for k, v in (("model", "PerformantNet1"), ("lr", 1e-3), ("betas", [0.9, 0.999]),
                         ("eps", 1e-8), ("max_throttle", 32), ("batch_size", 128)):
                if k not in cfg:
                    cfg[k] = v
                    warnings.warn(f"format-1 checkpoint: {k} not recorded, taken as {v!r}")
            delays = np.where((delays == 0) & (self.delays == DELAY_ZERO), DELAY_ZERO, delays)
        for k, v in mine.items():
            if cfg.get(k) != v:
                raise ValueError(f"checkpoint {k}={cfg.get(k)!r} differs from this run ({v!r})")
        if not np.array_equal(delays, self.delays):
            raise ValueError("checkpoint delays differ from this run")
        if self.trace:
            raise ValueError("restore() needs a fresh simulation")
        T = int(ck["epoch"])
        for _ in range(T):                    # replay the integer scan and the k-draws
            self.trace.append(self.sched.next_epoch())
            self.rs.randint(0, self.n, size=self.n)
        self.step = int(ck["step"])
        self.theta.copy_(ck["theta"].to(self.device))
        self.m.copy_(ck["m"].to(self.device))
        self.v.copy_(ck["v"].to(self.device))
        self.stale_store = {}
        for src, (vals, rc) in ck["stale"].items():
            slot = self._slot()
            slot[:self.P].copy_(vals.to(self.device))
            self.stale_store[int(src)] = [slot, int(rc)]
        self.loss_log = list(ck["loss_log"])
        if ck.get("buffers"):
            self.engine.load_buffers(ck["buffers"])

    def executed_worker_steps(self, plan):
        return int(plan.computes.sum())

    def param_views(self):
        return split_views(self.theta, self.engine.SHAPES)


__all__ = ["FLSimulation", "default_theta", "PN1_SIZES"]
