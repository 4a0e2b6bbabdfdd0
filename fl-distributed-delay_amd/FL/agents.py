"""Drop-in for the reference's FL/agents.py (agents.py:1-45) on MI355X.

Same classes, signatures and aliasing semantics; the arithmetic runs in libflsim.so:

  Worker.fwd_bkwd(inp, outp)   agents.py:32-40 -> flsim_<net>_fwd_bwd_input (HIP fwd/bwd of the
                               central model); gradients accumulate over the workers of an epoch
                               exactly like .grad (agents.py:35) and the returned list holds
                               views of ONE flat buffer (every worker of the epoch gets the same
                               tensors, as in the reference)
  Agg(rule)                    agents.py:43-45; use FL.agents.rule (== main.py:23-25's mean) to
                               get the fused path: it returns a lazy mean that Central consumes
  Central.update_model(ups)    agents.py:9-21 -> flsim_aggregate_adam_rule (cascade mean over the
                               entries in any order + Adam with the optimizer's lr/betas/eps);
                               parameters live in one flat device buffer, model.parameters() are
                               views of it

The .grad views fwd_bkwd returns are filled lazily (_LazyGrad): the gradient stays in the
engine's split-K slabs until a torch function first touches a view (then the slabs are reduced
into the buffer, so user code always reads the accumulated .grad) or until update_model, which
then runs the fused server step: one slab reduction per epoch instead of one per call.

Batches (main.py:43-44 --batch_size): any size up to 16,384 samples.  The engine pads a batch to
whole groups of 128 samples (padding adds nothing) and scales the CrossEntropyLoss gradient by
1/n, so the gradient is the reference's mean over the n samples.  Dropout masks follow the
build's Philox spec: group b of worker i's batch in epoch t is keyed
(t, i + b * 2^20).

Worker.index is the worker's position in the worker list: workers are numbered in creation order
from the last Central (main.py:110-113 builds Central, then the workers).

vgg11_bn(): the module's BatchNorm running_mean / running_var alias the engine's device buffer;
every train-mode fwd_bkwd call advances them (and num_batches_tracked) as nn.BatchNorm2d does
(with staged calls: when the buffers are next read, _LazyBuffer); batches must be 128 samples
(one BatchNorm batch per call).

Staged calls (PerformantNet1, vgg11, vgg11_bn; 128-sample batches): fwd_bkwd stages the batch and
returns a _LazyLoss that reads as agents.py:40's 0-d float32 array; the staged calls run as one
worker-batched pass when a loss, a .grad view or a BatchNorm buffer is read, or the chunk is due
(FLSIM_FACADE_LAZY_LOSS=0: a call's forward runs at once).

Requirements (raise otherwise): the model is FL.models.PerformantNet1, vgg11() or vgg11_bn() on
a HIP device, the optimizer is torch.optim.Adam without weight decay / amsgrad / maximize.
There is no CPU fallback.
"""
from __future__ import annotations

import os
import weakref

import numpy as np
import torch

from flsim.engine import (ProgramStager, Rule, engine_for_parameters, padded, split_views,
                          worker_table)

_CONTEXTS = weakref.WeakKeyDictionary()    # model -> _ModelContext (dies with the model)
_NEXT_WORKER = [0]                          # Worker.index of the next Worker()
MAX_BATCH = 16384                           # samples per fwd_bkwd call (32-bit index budget)
GROUP_KEY_STRIDE = 1 << 20                  # dropout key of 128-sample group b: i + b * 2^20


# Tensor methods and properties that read only metadata or the storage handle: a lazy gradient
# view answers them without reducing the slabs first
_META = set()
for _n in ("untyped_storage", "data_ptr", "size", "dim", "numel", "stride", "storage_offset",
           "element_size", "is_contiguous", "__len__", "nelement", "ndimension", "get_device"):
    if hasattr(torch.Tensor, _n):
        _META.add(getattr(torch.Tensor, _n))
for _n in ("shape", "dtype", "device", "is_cuda", "requires_grad", "grad_fn", "is_leaf", "layout",
           "ndim", "is_sparse", "is_quantized", "is_meta", "names", "grad"):
    _pr = getattr(torch.Tensor, _n, None)
    if _pr is not None and hasattr(_pr, "__get__"):
        _META.add(_pr.__get__)
# .data and ._base hand out another tensor over the same storage: they reduce the slabs first and
# the tensor they return is itself lazy, so a later read through it (p.grad.data.sum() after more
# fwd_bkwd calls) reduces again instead of reading a stale partial sum
_ALIASING = {getattr(torch.Tensor, _n).__get__ for _n in ("data", "_base")
             if hasattr(getattr(torch.Tensor, _n, None), "__get__")}
del _n, _pr


class _LazyGrad(torch.Tensor):
    """A .grad view of the epoch's flat gradient buffer G whose contents are produced on first
    use.  fwd_bkwd leaves the worker's gradient in the engine's split-K slabs; any torch function
    or method that reads (or writes) one of these views first reduces the slabs into G
    (flsim_<net>_end_epoch), so every read sees exactly what the reference's accumulated .grad
    holds (agents.py:35).  Central.update_model instead runs the fused server step (slabs -> S_t
    -> rule() + Adam, S_t written into G) when nothing has been read: the reference loop of
    main.py:126-188 then reduces the slabs once per epoch, not once per fwd_bkwd call."""

    @classmethod
    def __torch_function__(cls, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        if func not in _META:
            seen = []
            for a in list(args) + list(kwargs.values()):
                for x in (a if isinstance(a, (list, tuple)) else (a,)):
                    if isinstance(x, _LazyGrad):
                        ctx = x.__dict__.get("_flsim_ctx")
                        ctx = ctx() if ctx is not None else None
                        if ctx is not None and all(c is not ctx for c in seen):
                            seen.append(ctx)
                            ctx.flush(touched=True)
        with torch._C.DisableTorchFunctionSubclass():
            out = func(*args, **kwargs)
        if func in _ALIASING and isinstance(out, torch.Tensor) and args and \
                isinstance(args[0], _LazyGrad):
            if not isinstance(out, _LazyGrad):
                out = torch.Tensor._make_subclass(_LazyGrad, out, False)
            if "_flsim_ctx" not in out.__dict__:
                out.__dict__["_flsim_ctx"] = args[0].__dict__.get("_flsim_ctx")
        return out

    def __repr__(self, *, tensor_contents=None):
        return repr(self.as_subclass(torch.Tensor))


class _LazyBuffer(torch.Tensor):
    """A vgg11_bn running buffer (running_mean / running_var / num_batches_tracked) of a facade
    with staged calls: any torch function or method that touches it first runs the staged calls
    (their BatchNorm statistics fold into the running buffers there), so every read sees what the
    reference's module holds after each train-mode call (nn.BatchNorm2d)."""

    @classmethod
    def __torch_function__(cls, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        if func not in _META:
            for a in list(args) + list(kwargs.values()):
                for x in (a if isinstance(a, (list, tuple)) else (a,)):
                    if isinstance(x, _LazyBuffer):
                        ctx = x.__dict__.get("_flsim_ctx")
                        ctx = ctx() if ctx is not None else None
                        if ctx is not None and ctx.block is not None:
                            ctx.flush_backward()
        with torch._C.DisableTorchFunctionSubclass():
            return func(*args, **kwargs)

    def __repr__(self, *, tensor_contents=None):
        return repr(self.as_subclass(torch.Tensor))


def _lazy_views(flat, shapes, ctx):
    ref = weakref.ref(ctx)
    out = []
    for v in split_views(flat, shapes):
        g = torch.Tensor._make_subclass(_LazyGrad, v, False)
        g.__dict__["_flsim_ctx"] = ref
        out.append(g)
    return out


class _ModelContext:
    """Flat parameter / optimizer-state buffers and the engine of one central model."""

    def __init__(self, model, seed=0):
        self.engine_cls = engine_for_parameters(n for n, _ in model.named_parameters())
        self.shapes = self.engine_cls.SHAPES
        dev = next(model.parameters()).device
        if dev.type != "cuda":
            raise RuntimeError("move the model to the GPU first (main.py:105 model.to(device))")
        self.device = dev
        with torch.no_grad():
            flat = torch.cat([p.detach().reshape(-1).float() for p in model.parameters()])
        self.P = flat.numel()
        self.theta = torch.zeros(padded(self.P), device=dev)
        self.theta[:self.P].copy_(flat)
        for p, view in zip(model.parameters(), split_views(self.theta[:self.P], self.shapes)):
            p.data = view                       # parameters alias the flat buffer
        self.m = torch.zeros_like(self.theta)
        self.v = torch.zeros_like(self.theta)
        self.params = list(model.parameters())
        # Deferred backward (PerformantNet1): every fwd_bkwd call of an epoch runs on theta_t, so
        # a call runs only its forward + loss (what agents.py:40 returns) into the next rows of a
        # chunk workspace, and the backward of up to `defer_rows` samples of calls runs as ONE
        # worker-batched pass (flsim_pn1_bwd_rows) when the chunk is full or the gradient is
        # needed (a .grad view is touched, update_model, evaluation, a parameter change).
        # FLSIM_FACADE_CHUNK = workers (128-sample groups) per deferred backward at most; 0: a
        # backward per call.  The chunk workspace starts at 8 workers and grows between epochs to
        # what an epoch used (so a 4-worker loop holds 1.6 GB, a 1024-worker one 2 x 26 GB).
        cw = int(os.environ.get("FLSIM_FACADE_CHUNK", "128"))
        lazy = os.environ.get("FLSIM_FACADE_LAZY_LOSS", "1") != "0"
        self.defer_max = 0
        # (vgg11_bn defers only with the lazy loss: its calls are always staged, see below)
        if cw > 0 and (self.engine_cls.PREFIX in ("pn1", "vgg11") or
                       (self.engine_cls.PREFIX == "vgg11_bn" and lazy)):
            self.defer_max = min(cw, MAX_BATCH // 128) * 128
        self.engine = self.engine_cls(dev, chunk_workers=min(self.defer_max // 128, 8) or 1)
        self.defer_rows = self.engine.max_samples if self.defer_max else 0
        # Deferred forward (PerformantNet1 and vgg11, 128-sample calls): a call only stages its
        # batch into the chunk's next rows and returns a _LazyLoss; the forward + loss of the
        # staged calls runs as one batched pass (flush_forward; vgg11: forward, loss and backward
        # together, the batched engine's chunk) when a loss is read or the backward is due.
        # FLSIM_FACADE_LAZY_LOSS=0: every call runs its forward now and returns a plain array
        # (vgg11: its forward and backward, as before).  vgg11_bn: the staged calls' BatchNorm
        # statistics fold into the running buffers in call order at the flush; the module's
        # running_mean / running_var / num_batches_tracked are then _LazyBuffer views that run the
        # staged calls first whenever they are read.
        self.lazy_loss = lazy
        self.block = None            # _LossBlock of the staged calls whose forward has not run
        self.epoch_rows = 0          # rows forwarded this epoch
        self.pending = 0             # rows forwarded whose backward is not queued yet
        self.pending_dropout = None  # their dropout flag (one per backward pass)
        self.theta_run = None        # the theta this epoch's packed weights / rows were run with
        self.version = None          # parameter versions when theta_run was taken
        self.bn_stats = None
        self.bns = []
        if self.engine.STATS_PER_WORKER:
            self._alias_buffers(model)
            self.bn_stats = torch.zeros(self.engine.STATS_PER_WORKER, device=dev)
        self.seed = seed
        self.t = 0               # epoch counter (dropout RNG key)
        self.G = None            # flat gradient buffer of the current epoch (p.grad views)
        self.dirty = False       # G lags the slabs (fwd_bkwd ran since the last reduction)
        self.touched = False     # a .grad view was used this epoch: update_model reads G
        # pipelined fwd_bkwd (PN1): a call's backward runs beside the next call's forward;
        # FLSIM_FACADE_PIPELINE=0 turns it off
        self.pipeline = os.environ.get("FLSIM_FACADE_PIPELINE", "1") != "0"
        self.slot = 0
        self.carry = None        # gradient accumulated before an engine resize this epoch
        self.packed = False
        self.step = 0
        self.loss_buf = torch.zeros(64, device=dev)
        self.stager = ProgramStager(dev)
        self.users = {}          # Worker.index -> id(Worker) of this epoch's fwd_bkwd calls
        self.views = None        # the epoch's .grad views of G
        self.rec_table = None    # device WorkerRec rows (t, i) of epoch rec_t
        self.rec_t = -1

    def _alias_buffers(self, model):
        """BatchNorm running buffers become views of the engine's device buffer (loaded from the
        module first, e.g. after main.py:99 load_state_dict)."""
        bns = [mod for mod in model.modules() if isinstance(mod, torch.nn.BatchNorm2d)]
        views = self.engine.running_views()
        assert len(bns) == len(views)
        self.engine.num_batches_tracked = int(bns[0].num_batches_tracked)
        lazy = self.defer_max > 0
        ref = weakref.ref(self)

        def wrap(t):
            t = torch.Tensor._make_subclass(_LazyBuffer, t, False)
            t.__dict__["_flsim_ctx"] = ref
            return t
        for mod, (_, rm, rv) in zip(bns, views):
            with torch._C.DisableTorchFunctionSubclass():
                rm.copy_(mod.running_mean.detach().reshape(-1))
                rv.copy_(mod.running_var.detach().reshape(-1))
            if lazy:
                mod.running_mean = wrap(rm)
                mod.running_var = wrap(rv)
                mod.num_batches_tracked = wrap(mod.num_batches_tracked.detach())
            else:
                mod.running_mean.data = rm
                mod.running_var.data = rv
        self.bns = bns

    def ensure_capacity(self, n_samples):
        """An engine whose workspace holds n_samples.  Growing it mid-epoch keeps what the epoch
        has accumulated: the new engine's slabs start at zero, so the running sum so far is
        carried and added back after every later reduction (agents.py:35 keeps accumulating)."""
        if n_samples > MAX_BATCH:
            raise ValueError(f"batch of {n_samples} samples: the HIP engine takes at most "
                             f"{MAX_BATCH} per fwd_bkwd call")
        cw = -(-n_samples // 128)
        if cw > self.engine.chunk_workers:
            old = self.engine
            if self.G is not None:
                # the old engine's slabs, reduced by the old engine before it goes away (flush
                # runs end_epoch on self.engine, so this comes before the replacement)
                self.flush()
                self.carry = self.G.clone()
            self.engine = self.engine_cls(self.device, chunk_workers=cw)
            if old.STATS_PER_WORKER:        # the running buffers stay where the module sees them
                self.engine.running = old.running
                self.engine.num_batches_tracked = old.num_batches_tracked
            self.packed = False
            if self.defer_rows:
                self.defer_rows = self.engine.max_samples
                self.defer_max = max(self.defer_max, self.defer_rows)
        if cw > self.loss_buf.numel():
            self.loss_buf = torch.zeros(cw, device=self.device)

    def worker_rec(self, index, groups):
        """Device WorkerRec rows (epoch t, index + b * 2^20) of a call: one-group calls slice a
        table of the epoch's records uploaded once (grown by doubling), not one upload each."""
        if groups != 1:
            return worker_table([(self.t, index + b * GROUP_KEY_STRIDE, 0)
                                 for b in range(groups)], self.device)
        tab = self.rec_table
        if tab is None or self.rec_t != self.t or index >= tab.shape[0]:
            size = max(64, 2 * (index + 1), 0 if tab is None else tab.shape[0])
            tab = worker_table([(self.t, i, 0) for i in range(size)], self.device)
            self.rec_table, self.rec_t = tab, self.t
        return tab[index:index + 1]

    def claim(self, worker):
        """Dropout keys are (epoch, Worker.index): two different Worker objects computing with
        the same index in one epoch would draw identical masks.  That happens only when the
        indices were reset under live workers (a second Central built after them, or workers
        built before the Central), so it is refused instead of silently correlating the masks."""
        prev = self.users.setdefault(worker.index, id(worker))
        if prev != id(worker):
            raise ValueError(f"two Workers share index {worker.index} in one epoch (Worker "
                             "indices restart at 0 when a Central is built: build the Central "
                             "first, then the workers, as main.py:110-113 does)")

    def _param_version(self):
        return sum(p._version for p in self.params)

    def prepare_rows(self):
        """theta_run for this call's forward rows.  The first call of an epoch packs theta_t
        (begin_epoch).  A parameter written in place since then (load_state_dict, an in-place op
        under no_grad) is seen by the reference's next forward: the pending rows' backward runs
        first with the theta their forwards used, the epoch's gradient so far is carried, and
        the new theta is packed."""
        v = self._param_version()
        if self.packed and v == self.version:
            return self.theta_run
        if self.theta_run is None:
            self.theta_run = torch.empty_like(self.theta)
        if self.packed:
            self.flush()
            self.carry = self.G.clone()
        self.theta_run.copy_(self.theta)
        self.engine.begin_epoch(self.theta_run)
        self.packed = True
        self.version = v
        return self.theta_run

    def flush_forward(self):
        """Run the forward + loss of the staged calls (one worker-batched pass over their rows);
        their _LazyLoss values are then ready on the stream."""
        b = self.block
        if b is None:
            return
        self.block = None
        n = len(b.indices)
        wt = worker_table([(self.t, i, 0) for i in b.indices], self.device)
        b.dev = torch.empty(n, device=self.device)
        if self.bns:
            # vgg11_bn: forward, loss, backward and each call's BatchNorm statistics in one
            # chunk, then nn.BatchNorm2d's running updates of the n calls in call order
            assert b.row0 == 0 and self.pending == n * 128
            stats = torch.empty(n * self.engine.STATS_PER_WORKER, device=self.device)
            self.engine.fwd_bwd_loaded_rows(self.theta_run, n * 128, wt, self.seed, b.dropout,
                                            b.dev, stats)
            self.pending = 0
            self.engine.update_running(stats, n)
            with torch._C.DisableTorchFunctionSubclass():
                for mod in self.bns:
                    mod.num_batches_tracked.fill_(self.engine.num_batches_tracked)
        elif hasattr(self.engine, "fwd_bwd_loaded_rows"):
            # vgg11: forward, loss and backward of the staged rows [0, n * 128) in one chunk
            assert b.row0 == 0 and self.pending == n * 128
            self.engine.fwd_bwd_loaded_rows(self.theta_run, n * 128, wt, self.seed, b.dropout,
                                            b.dev)
            self.pending = 0
        else:
            self.engine.forward_loaded_rows(self.theta_run, b.row0, n * 128, wt, self.seed,
                                            b.dropout, b.dev, b.slot)

    def flush_backward(self):
        """Queue the backward of the pending forward rows (one worker-batched pass)."""
        self.flush_forward()
        if self.pending:
            self.engine.backward_rows(self.theta_run, self.pending, self.pending_dropout,
                                      self.slot)
            self.slot ^= 1               # the next rows go to the other workspace
            self.pending = 0

    def flush(self, touched=False):
        """G = the epoch's gradient so far: the slab reduction fwd_bkwd left pending.  touched:
        user code read or wrote a .grad view, so from now on G (not the slabs) is the epoch's
        gradient for update_model (an in-place change of a .grad is seen)."""
        self.touched = self.touched or touched
        self.flush_backward()
        if not self.dirty:
            return
        self.dirty = False
        self.engine.end_epoch(self.G)
        if self.carry is not None:
            self.G.add_(self.carry)

    def new_epoch(self):
        if self.defer_rows and self.defer_rows < min(self.epoch_rows, self.defer_max):
            # the last epoch's calls did not fit one deferred chunk: a larger workspace (the
            # epoch's gradient is consumed, nothing is pending)
            cw = -(-min(self.epoch_rows, self.defer_max) // 128)
            old = self.engine
            self.engine = self.engine_cls(self.device, chunk_workers=cw)
            if old.STATS_PER_WORKER:        # the running buffers stay where the module sees them
                self.engine.running = old.running
                self.engine.num_batches_tracked = old.num_batches_tracked
            self.defer_rows = self.engine.max_samples
            self.slot = 0
        self.epoch_rows = 0
        self.t += 1
        self.users = {}
        self.G = None
        self.views = None
        self.dirty = False
        self.touched = False
        self.carry = None
        self.packed = False


def _context(model):
    ctx = _CONTEXTS.get(model)
    if ctx is None:
        ctx = _ModelContext(model)
        _CONTEXTS[model] = ctx
    return ctx


class _LazyMean(list):
    """What FL.agents.rule returns: the weight_ups list, reduced inside Central.update_model."""

    def __init__(self, ups_list):
        super().__init__()
        self.ups_list = ups_list


def rule(ups_list):
    """main.py:23-25 (element-wise mean of the gradient lists), evaluated lazily and fused with
    the Adam step in Central.update_model."""
    if len(ups_list) == 0:
        raise IndexError("list index out of range")        # main.py:25 ups_list[0]
    return _LazyMean(ups_list)


class Central:
    """agents.py:4-24."""

    def __init__(self, model, optim, encryption=False):
        self.model = model
        self.optim = optim
        g = optim.param_groups[0]
        if not isinstance(optim, torch.optim.Adam) or g.get("weight_decay", 0) != 0 or \
                g.get("amsgrad", False) or g.get("maximize", False):
            raise NotImplementedError("fused update implements torch.optim.Adam "
                                      "(main.py:106: Adam(lr), no weight decay / amsgrad)")
        self.ctx = _context(model)
        _NEXT_WORKER[0] = 0          # main.py:112-113: the workers built next are 0 .. n-1

    def _sync_optimizer_state(self):
        ctx = self.ctx
        for p, mv, vv in zip(self.model.parameters(), split_views(ctx.m[:ctx.P], ctx.shapes),
                             split_views(ctx.v[:ctx.P], ctx.shapes)):
            self.optim.state[p] = {"step": torch.tensor(float(ctx.step)), "exp_avg": mv,
                                   "exp_avg_sq": vv}

    def _rule_of(self, ups):
        """(S, Rule) for weight_ups: the entries that are this epoch's gradient buffer are S_t;
        every other entry (a stale FIFO entry, main.py:161-165) is an array, in list order."""
        ctx = self.ctx
        entries = [u[0] for u in ups.ups_list]
        S = ctx.G if ctx.G is not None else torch.zeros(padded(ctx.P), device=ctx.device)
        sbase = S.untyped_storage().data_ptr()
        arrays, bases, events = [], [], []
        for pos, e in enumerate(entries):
            b = e.untyped_storage().data_ptr()
            if b == sbase:
                continue
            if b not in bases:
                bases.append(b)
                arrays.append(_flat_of(e, ctx))
            events.append((pos, bases.index(b)))
        k = len(entries)
        c = k - len(events)
        if len(events) <= 8 and all(p >= c for p, _ in events):    # reference order
            return S, Rule(k, [arrays[j] for _, j in events], c=c)
        return S, Rule(k, arrays, events=events, stager=ctx.stager)

    def update_model(self, ups):
        """agents.py:9-21: install the aggregated gradient, Adam step, clear .grad."""
        ctx = self.ctx
        g = self.optim.param_groups[0]
        eng = ctx.engine
        if isinstance(ups, _LazyMean):
            S, r = self._rule_of(ups)
        else:
            if len(ups) != len(ctx.shapes):
                raise IndexError("list index out of range")
            S = torch.cat([u.detach().reshape(-1).float() for u in ups])
            S = torch.nn.functional.pad(S, (0, padded(ctx.P) - ctx.P))
            r = Rule(1, [], c=1)
        ctx.step += 1
        hp = dict(lr=g["lr"], betas=g["betas"], eps=g["eps"])
        if isinstance(ups, _LazyMean) and ctx.G is not None and ctx.carry is None and \
                not ctx.touched and hasattr(eng, "server_step"):
            # fused: this epoch's slabs -> S_t (also written into G, which the FIFO entries of
            # main.py:156,161 alias) -> rule() + Adam, one pass
            ctx.flush_backward()
            eng.server_step(ctx.G, r, ctx.theta, ctx.m, ctx.v, ctx.step, **hp)
            ctx.dirty = False
        else:
            ctx.flush()
            eng.aggregate_rule(S, r, ctx.theta, ctx.m, ctx.v, ctx.step, **hp)
        for p in self.model.parameters():        # optim.zero_grad() (set_to_none, torch >= 2)
            p.grad = None
        self._sync_optimizer_state()
        ctx.new_epoch()

    def init_adv(self, model):
        self.adv = model


def _flat_of(view, ctx):
    """The flat gradient buffer a returned .grad view belongs to."""
    st = view.untyped_storage()
    n = st.nbytes() // 4
    flat = torch.empty(0, device=ctx.device).set_(st, 0, (n,), (1,))
    if n < ctx.P:
        raise ValueError("gradient entry is not a flsim gradient buffer")
    return flat


class _LossBlock:
    """The staged 128-sample calls of one deferred forward: rows [row0, row0 + 128 * len) of
    workspace `slot`, their Worker indices (dropout keys) and, once flush_forward has run, their
    losses (`dev`, fetched to the host once, on the first read of any of them)."""

    def __init__(self, ctx, row0, slot, dropout):
        self.ctx = weakref.ref(ctx)
        self.row0, self.slot, self.dropout = row0, slot, dropout
        self.indices = []
        self.dev = None
        self.host = None

    def value(self, g):
        if self.host is None:
            if self.dev is None:
                ctx = self.ctx()
                if ctx is None:
                    raise RuntimeError("the model of this loss was freed before its forward ran")
                ctx.flush_forward()
            self.host = self.dev.cpu().numpy()
            self.dev = None
        return self.host[g]


class _LazyLoss:
    """What Worker.fwd_bkwd returns as the loss of a deferred 128-sample call: agents.py:40's
    `lossval.detach().cpu().numpy()` (a 0-d float32 array), computed on first read.  Reading it
    (np.mean over a list of them as main.py:181 does, float(), print, arithmetic, any ndarray
    attribute) runs the forward of the calls staged so far as one batched pass and fetches their
    losses in one copy; the value is the per-call forward's, bit for bit."""

    __slots__ = ("_block", "_g", "_arr")
    __array_priority__ = 1000

    def __init__(self, block, g):
        self._block, self._g, self._arr = block, g, None

    def _value(self):
        if self._arr is None:
            self._arr = np.asarray(np.float32(self._block.value(self._g)), np.float32)
            self._block = None
        return self._arr

    def __array__(self, dtype=None, copy=None):
        a = self._value()
        return a if dtype is None else a.astype(dtype)

    def __array_ufunc__(self, ufunc, method, *inputs, **kwargs):
        inputs = tuple(x._value() if isinstance(x, _LazyLoss) else x for x in inputs)
        return getattr(ufunc, method)(*inputs, **kwargs)

    def __getattr__(self, name):
        return getattr(self._value(), name)

    def __float__(self):
        return float(self._value())

    def __int__(self):
        return int(self._value())

    def __bool__(self):
        return bool(self._value())

    def __repr__(self):
        return repr(self._value())

    def __str__(self):
        return str(self._value())

    def __format__(self, spec):
        return format(self._value(), spec)

    def __reduce__(self):
        return (np.asarray, (self._value(),))

    def __neg__(self):
        return -self._value()

    def __abs__(self):
        return abs(self._value())


def _binop(name):
    def f(self, other):
        other = other._value() if isinstance(other, _LazyLoss) else other
        return getattr(self._value(), name)(other)
    f.__name__ = name
    return f


for _op in ("add", "sub", "mul", "truediv", "floordiv", "pow", "mod"):
    setattr(_LazyLoss, f"__{_op}__", _binop(f"__{_op}__"))
    setattr(_LazyLoss, f"__r{_op}__", _binop(f"__r{_op}__"))
for _op in ("lt", "le", "gt", "ge", "eq", "ne"):
    setattr(_LazyLoss, f"__{_op}__", _binop(f"__{_op}__"))
_LazyLoss.__hash__ = None                # as ndarray
del _op


class Worker:
    """agents.py:27-40."""

    def __init__(self, loss, key=None):
        self.model = None
        self.loss = loss
        self.index = _NEXT_WORKER[0]     # position in the worker list (main.py:112-113)
        _NEXT_WORKER[0] += 1

    def fwd_bkwd(self, inp, outp):
        if not isinstance(self.loss, torch.nn.CrossEntropyLoss) or \
                getattr(self.loss, "reduction", "mean") != "mean":
            raise NotImplementedError("fused loss implements nn.CrossEntropyLoss(mean)")
        ctx = _context(self.model)
        ctx.claim(self)
        n = int(inp.shape[0])
        if int(outp.shape[0]) != n:
            raise ValueError(f"Expected input batch_size ({n}) to match target batch_size "
                             f"({int(outp.shape[0])}).")
        ctx.ensure_capacity(n)
        eng = ctx.engine
        theta = ctx.theta
        defer = bool(ctx.defer_rows)
        rows_api = defer and eng.PREFIX == "pn1"     # one-call forwards into chunk rows
        if defer:
            theta = ctx.prepare_rows()
        elif not ctx.packed:
            eng.begin_epoch(theta)
            ctx.packed = True
        if ctx.G is None:
            ctx.G = torch.zeros(padded(ctx.P), device=ctx.device)
            # the epoch's .grad views: every call returns the same tensors (agents.py:37-39 hands
            # out the parameters' own .grad, the same objects for every worker of the epoch)
            ctx.views = _lazy_views(ctx.G[:ctx.P], ctx.shapes, ctx)
        groups = -(-n // 128)
        lazy_call = defer and ctx.lazy_loss and n == 128
        wt = None if lazy_call else ctx.worker_rec(self.index, groups)
        lb = ctx.loss_buf[:groups]
        kw = {}
        if ctx.bn_stats is not None:
            if not self.model.training or n != 128:
                raise NotImplementedError("vgg11_bn: the HIP engine runs BatchNorm in train mode "
                                          "on 128-sample batches (main.py:43-44, 132)")
            kw = {} if lazy_call else {"stats_out": ctx.bn_stats}   # staged: at the flush
        x = inp.to(ctx.device, torch.float32)
        lazy = None
        if defer and not lazy_call and not rows_api:
            # vgg11, a call that is not staged: the staged calls run first, then this call's
            # forward and backward at once (the workspace rows are the staged calls')
            ctx.flush_backward()
            eng.run_input(theta, x, outp.to(ctx.device), wt, ctx.seed, self.model.training, lb)
        elif defer:
            # this call's forward + loss into the chunk's next rows; the backward waits for the
            # chunk (one batched pass, flush_backward)
            training = bool(self.model.training)
            rows = groups * 128
            if ctx.pending and (ctx.pending + rows > ctx.defer_rows or
                                training != ctx.pending_dropout):
                ctx.flush_backward()
            if lazy_call:
                # staged only: the forward runs with the other staged calls (flush_forward)
                eng.load_rows(x, outp.to(ctx.device), ctx.pending, ctx.slot)
                if ctx.block is None:
                    ctx.block = _LossBlock(ctx, ctx.pending, ctx.slot, training)
                lazy = _LazyLoss(ctx.block, len(ctx.block.indices))
                ctx.block.indices.append(self.index)
            else:
                ctx.flush_forward()          # the staged block's rows stay contiguous
                eng.forward_rows(theta, x, outp.to(ctx.device), wt, ctx.seed, training, lb,
                                 ctx.pending, ctx.slot)
            ctx.pending += rows
            ctx.epoch_rows += rows
            ctx.pending_dropout = training
        elif ctx.bn_stats is None and getattr(eng, "PIPELINE", False) and ctx.pipeline:
            # the backward overlaps the next call's forward (the loss below needs only this
            # forward); the .grad views join it on first use, update_model in its server step
            ctx.slot ^= 1
            eng.run_input_async(theta, x, outp.to(ctx.device), wt, ctx.seed, self.model.training,
                                lb, ctx.slot)
        else:
            eng.run_input(theta, x, outp.to(ctx.device), wt, ctx.seed, self.model.training, lb,
                          **kw)
        if ctx.bn_stats is not None and not lazy_call:   # nn.BatchNorm2d's running update
            eng.update_running(ctx.bn_stats, 1)
            for mod in ctx.bns:
                mod.num_batches_tracked.fill_(eng.num_batches_tracked)
        ctx.dirty = True                         # G = the running sum on first read (flush)
        grads = ctx.views
        for p, gv in zip(ctx.params, grads):
            if p.grad is not gv:
                p.grad = gv                      # agents.py:35: accumulated in place
        if lazy is not None:
            return list(grads), lazy
        # CrossEntropyLoss(mean) over the n samples: group sums / n (padding contributes 0)
        tot = lb.item() if groups == 1 else float(lb.double().sum().cpu())
        lossval = np.float32(tot * 128.0 / n)
        return list(grads), np.asarray(lossval, np.float32)


class Agg:
    """agents.py:43-45."""

    def __init__(self, rule):
        self.rule = rule
