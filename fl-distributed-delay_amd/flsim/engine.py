"""Worker-batched network engines: device buffers + the C-ABI calls of one epoch.

  begin_epoch(theta)      pack theta_t, zero the gradient slabs        (start of main.py:126)
  run_chunk(...)          worker-batched fwd/bwd of a chunk of workers (agents.py:32-40, xN)
  end_epoch(S)            S_t = sum of the epoch's gradients           (agents.py:35 accumulation)
  aggregate_adam(...)     fused rule() + Central.update_model          (main.py:23-25,184,188)

PN1Engine runs models.py:PerformantNet1 (the model main.py:97 builds) through flsim_pn1_*;
VGG11Engine runs models.py:vgg11() (models.py:50-103, configs[4]'s larger CNN) through
flsim_vgg11_*; VGG11BNEngine runs vgg11_bn() (models.py:106-108) through flsim_vgg11_bn_* and
keeps its BatchNorm running buffers.  Both entry-point families share one contract (include/flsim.h).
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from ._lib import MAX_ARRAYS, FlsimRule, WorkerRec, check, lib, ptr, stream_ptr

# named_parameters() order of models.py:PerformantNet1 (models.py:13-25)
PN1_SHAPES = [
    ("conv1.weight", (48, 3, 3, 3)), ("conv1.bias", (48,)),
    ("conv2.weight", (48, 48, 3, 3)), ("conv2.bias", (48,)),
    ("conv3.weight", (96, 48, 3, 3)), ("conv3.bias", (96,)),
    ("conv4.weight", (96, 96, 3, 3)), ("conv4.bias", (96,)),
    ("conv5.weight", (192, 96, 3, 3)), ("conv5.bias", (192,)),
    ("conv6.weight", (192, 192, 3, 3)), ("conv6.bias", (192,)),
    ("linear1.weight", (512, 9408)), ("linear1.bias", (512,)),
    ("linear2.weight", (256, 512)), ("linear2.bias", (256,)),
    ("linear3.weight", (10, 256)), ("linear3.bias", (10,)),
]
# named_parameters() order of models.py:vgg11() (features = make_layers(cfg 'A'),
# models.py:80-98; classifier models.py:57-65)
VGG11_SHAPES = [
    ("features.0.weight", (64, 3, 3, 3)), ("features.0.bias", (64,)),
    ("features.3.weight", (128, 64, 3, 3)), ("features.3.bias", (128,)),
    ("features.6.weight", (256, 128, 3, 3)), ("features.6.bias", (256,)),
    ("features.8.weight", (256, 256, 3, 3)), ("features.8.bias", (256,)),
    ("features.11.weight", (512, 256, 3, 3)), ("features.11.bias", (512,)),
    ("features.13.weight", (512, 512, 3, 3)), ("features.13.bias", (512,)),
    ("features.16.weight", (512, 512, 3, 3)), ("features.16.bias", (512,)),
    ("features.18.weight", (512, 512, 3, 3)), ("features.18.bias", (512,)),
    ("classifier.1.weight", (512, 512)), ("classifier.1.bias", (512,)),
    ("classifier.4.weight", (512, 512)), ("classifier.4.bias", (512,)),
    ("classifier.6.weight", (10, 512)), ("classifier.6.bias", (10,)),
]
# named_parameters() order of models.py:vgg11_bn() (make_layers(cfg 'A', batch_norm=True):
# Conv2d, BatchNorm2d, ReLU per conv, models.py:88-89) and its BatchNorm buffers
_BN_IDX = (0, 4, 8, 11, 15, 18, 22, 25)      # conv module index in features; BatchNorm = +1
VGG11_BN_SHAPES = []
for _j, (_, _shp) in enumerate(VGG11_SHAPES[:16:2]):
    _co = _shp[0]
    VGG11_BN_SHAPES += [(f"features.{_BN_IDX[_j]}.weight", _shp),
                        (f"features.{_BN_IDX[_j]}.bias", (_co,)),
                        (f"features.{_BN_IDX[_j] + 1}.weight", (_co,)),
                        (f"features.{_BN_IDX[_j] + 1}.bias", (_co,))]
VGG11_BN_SHAPES += VGG11_SHAPES[16:]
VGG11_BN_BUFFERS = [(f"features.{i + 1}", int(shp[0]))
                    for i, (_, shp) in zip(_BN_IDX, VGG11_SHAPES[:16:2])]
PN1_SIZES = [int(np.prod(s)) for _, s in PN1_SHAPES]
VGG11_SIZES = [int(np.prod(s)) for _, s in VGG11_SHAPES]
SAMPLES_PER_WORKER = 128


def padded(n, q=64):
    return (n + q - 1) // q * q


def split_views(flat, shapes=PN1_SHAPES):
    out, off = [], 0
    for _, shp in shapes:
        n = int(np.prod(shp))
        out.append(flat[off:off + n].view(shp))
        off += n
    return out


class NetEngine:
    """Gradient state + chunk workspace of one network on one device; PREFIX selects the C-ABI
    family (flsim_<PREFIX>_*), SHAPES its named_parameters layout."""

    PREFIX = None
    MODEL = None
    SHAPES = None
    FLOP_PER_WORKER_STEP = None     # algorithmic fwd + dgrad + wgrad FLOPs of 128 samples
    STATS_PER_WORKER = 0            # per-call statistics the model's buffers need (BatchNorm)

    def __init__(self, device, chunk_workers=32):
        self.device = torch.device(device)
        self.SIZES = [int(np.prod(s)) for _, s in self.SHAPES]
        self.P = int(self._fn("param_count")())
        assert self.P == sum(self.SIZES)
        self.chunk_workers = int(chunk_workers)
        self.max_samples = self.chunk_workers * SAMPLES_PER_WORKER
        self.gradstate = torch.empty(int(self._fn("gradstate_bytes")()), dtype=torch.uint8,
                                     device=self.device)
        self.workspace = torch.empty(int(self._fn("workspace_bytes")(self.max_samples)),
                                     dtype=torch.uint8, device=self.device)

    def _fn(self, name):
        return getattr(lib(), f"flsim_{self.PREFIX}_{name}")

    def __del__(self):
        # the caching allocator may give this gradstate's address to a later engine: the
        # library's slab-row table for it must not outlive the buffer (flsim_pn1_release)
        gs = getattr(self, "gradstate", None)
        try:
            if gs is not None and hasattr(lib(), f"flsim_{self.PREFIX}_release"):
                self._fn("release")(ptr(gs))
        except Exception:      # interpreter teardown: the library may already be gone
            pass

    # -- per-epoch gradient --------------------------------------------------------------------
    def begin_epoch(self, theta):
        check(self._fn("begin_epoch")(ptr(self.gradstate), ptr(theta), stream_ptr()))

    def _stats_arg(self, stats_out):
        """The extra bn_stats argument of a BatchNorm model's entry points (none otherwise)."""
        if not self.STATS_PER_WORKER:
            return ()
        return (ptr(stats_out) if stats_out is not None else None,)

    def run_chunk(self, theta, pool, workers_dev, n_chunk, n_workers_total, seed, dropout,
                  loss_out, backward=True, stats_out=None):
        """stats_out (BatchNorm models): device float[n_chunk][STATS_PER_WORKER] for the
        per-call statistics that update_running() folds into the running buffers."""
        self.last_workspace = self.workspace
        check(self._fn("fwd_bwd_chunk")(
            ptr(self.gradstate), ptr(self.workspace), self.max_samples, ptr(theta),
            ptr(pool.imgs), ptr(pool.labels), ptr(pool.list_a), int(pool.list_a.numel()),
            ptr(pool.list_b), int(pool.list_b.numel()), ptr(pool.lut), ptr(workers_dev),
            int(n_chunk), int(n_workers_total), ctypes.c_uint64(seed), int(bool(dropout)),
            int(bool(backward)), ptr(loss_out), *self._stats_arg(stats_out), stream_ptr()))

    # pipelined chunks (PN1Engine): chunk i's forward on the current stream overlaps chunk i-1's
    # backward on the library's backward stream; two workspaces alternate
    PIPELINE = False

    def run_chunk_async(self, theta, pool, workers_dev, n_chunk, n_workers_total, seed, dropout,
                        loss_out, slot):
        if getattr(self, "workspace2", None) is None:
            self.workspace2 = torch.empty_like(self.workspace)
        ws = self.workspace if slot % 2 == 0 else self.workspace2
        self.last_workspace = ws
        check(lib().flsim_pn1_fwd_bwd_chunk_async(
            ptr(self.gradstate), ptr(ws), self.max_samples, ptr(theta),
            ptr(pool.imgs), ptr(pool.labels), ptr(pool.list_a), int(pool.list_a.numel()),
            ptr(pool.list_b), int(pool.list_b.numel()), ptr(pool.lut), ptr(workers_dev),
            int(n_chunk), int(n_workers_total), ctypes.c_uint64(seed), int(bool(dropout)),
            ptr(loss_out), stream_ptr()))

    def run_input_async(self, theta, x, y, workers_dev, seed, dropout, loss_out, slot):
        """run_input with the backward pipelined (PN1Engine): the loss is ready on the current
        stream after the forward; the gradient is complete for every later entry point."""
        if getattr(self, "workspace2", None) is None:
            self.workspace2 = torch.empty_like(self.workspace)
        ws = self.workspace if slot % 2 == 0 else self.workspace2
        self.last_workspace = ws
        x = x.contiguous()
        y = y.to(torch.int64).contiguous()
        check(lib().flsim_pn1_fwd_bwd_input_async(
            ptr(self.gradstate), ptr(ws), self.max_samples, ptr(theta), ptr(x), ptr(y),
            int(x.shape[0]), ptr(workers_dev), ctypes.c_uint64(seed), int(bool(dropout)),
            ptr(loss_out), stream_ptr()))

    def _slot_workspace(self, slot):
        if getattr(self, "workspace2", None) is None:
            self.workspace2 = torch.empty_like(self.workspace)
        return self.workspace if slot % 2 == 0 else self.workspace2

    def forward_rows(self, theta, x, y, workers_dev, seed, dropout, loss_out, row0, slot):
        """The facade's deferred backward (PN1Engine): forward + loss of an explicit batch into
        workspace rows [row0, row0 + ceil(n/128)*128) of workspace `slot`; the loss is ready on
        the current stream.  backward_rows() later runs the backward of all rows at once."""
        ws = self._slot_workspace(slot)
        self.last_workspace = ws
        x = x.contiguous()
        y = y.to(torch.int64).contiguous()
        check(lib().flsim_pn1_fwd_rows(
            ptr(self.gradstate), ptr(ws), self.max_samples, int(row0), ptr(theta), ptr(x), ptr(y),
            int(x.shape[0]), ptr(workers_dev), ctypes.c_uint64(seed), int(bool(dropout)),
            ptr(loss_out), stream_ptr()))

    def load_rows(self, x, y, row0, slot):
        """The facade's deferred forward (PN1Engine): stage an explicit batch into workspace rows
        [row0, row0 + ceil(n/128)*128) of workspace `slot`; nothing is computed yet."""
        ws = self._slot_workspace(slot)
        self.last_workspace = ws
        x = x.contiguous()
        y = y.to(torch.int64).contiguous()
        check(self._fn("load_rows")(ptr(self.gradstate), ptr(ws), self.max_samples, int(row0),
                                    ptr(x), ptr(y), int(x.shape[0]), stream_ptr()))

    def forward_loaded_rows(self, theta, row0, n_rows, workers_dev, seed, dropout, loss_out,
                            slot):
        """Forward + loss of the staged rows [row0, row0 + n_rows) of workspace `slot` as one
        batched pass (every 128-row group one whole batch): loss_out[g] = group g's mean loss."""
        ws = self._slot_workspace(slot)
        check(lib().flsim_pn1_fwd_loaded_rows(
            ptr(self.gradstate), ptr(ws), self.max_samples, int(row0), int(n_rows), ptr(theta),
            ptr(workers_dev), ctypes.c_uint64(seed), int(bool(dropout)), ptr(loss_out),
            stream_ptr()))

    def backward_rows(self, theta, n_rows, dropout, slot):
        """The backward of rows [0, n_rows) of workspace `slot` (forward_rows) into the epoch's
        slabs, on the library's backward stream (the next slot's forwards overlap it)."""
        check(lib().flsim_pn1_bwd_rows(ptr(self.gradstate), ptr(self._slot_workspace(slot)),
                                       self.max_samples, int(n_rows), ptr(theta),
                                       int(bool(dropout)), stream_ptr()))

    def evaluate_input(self, theta, x):
        """Predictions for an explicit NCHW fp32 batch (util.py:31-45's model(images) in eval
        mode): device int32 tensor of argmax indices."""
        x = x.to(self.device, torch.float32).contiguous()
        n = int(x.shape[0])
        pred = torch.empty(n, dtype=torch.int32, device=self.device)
        extra = (ptr(self.running),) if self.STATS_PER_WORKER else ()
        self.last_workspace = self.workspace
        check(self._fn("eval_input")(ptr(self.gradstate), ptr(self.workspace), self.max_samples,
                                     ptr(theta), ptr(x), n, *extra, ptr(pred), stream_ptr()))
        return pred

    def run_input(self, theta, x, y, workers_dev, seed, dropout, loss_out, backward=True,
                  stats_out=None):
        x = x.contiguous()
        y = y.to(torch.int64).contiguous()
        self.last_workspace = self.workspace
        check(self._fn("fwd_bwd_input")(
            ptr(self.gradstate), ptr(self.workspace), self.max_samples, ptr(theta), ptr(x), ptr(y),
            int(x.shape[0]), ptr(workers_dev), ctypes.c_uint64(seed), int(bool(dropout)),
            int(bool(backward)), ptr(loss_out), *self._stats_arg(stats_out), stream_ptr()))

    def evaluate(self, theta, pool, first=0, n_images=None):
        """Predictions (argmax of the logits, dropout off) for pool images [first, first + n):
        util.print_test_accuracy's forward (util.py:31-45).  Returns a device int32 tensor."""
        n = int(pool.imgs.shape[0]) - first if n_images is None else int(n_images)
        pred = torch.empty(n, dtype=torch.int32, device=self.device)
        extra = (ptr(self.running),) if self.STATS_PER_WORKER else ()
        self.last_workspace = self.workspace
        check(self._fn("eval_pool")(
            ptr(self.gradstate), ptr(self.workspace), self.max_samples, ptr(theta), ptr(pool.imgs),
            int(first), n, ptr(pool.lut), *extra, ptr(pred), stream_ptr()))
        return pred

    # -- model buffers (BatchNorm running statistics; none for the other models) ----------------
    def update_running(self, stats, n_workers):
        """nn.BatchNorm2d's per-call running update for n_workers calls in worker order."""

    def buffer_state(self):
        """The model's buffers as state_dict entries (OrderedDict order of models.py)."""
        return []

    def load_buffers(self, state):
        """Restore buffer_state() output (names -> tensors)."""

    def end_epoch(self, grad_out):
        check(self._fn("end_epoch")(ptr(self.gradstate), ptr(grad_out), stream_ptr()))

    def server_step(self, S_out, rule, theta, m, v, step, lr=1e-3, betas=(0.9, 0.999), eps=1e-8):
        """world = 1: the epoch's slabs -> S_t [-> S_out] -> rule() + Adam in one launch
        (flsim_<net>_server_step).  rule: a Rule."""
        check(self._fn("server_step")(
            ptr(self.gradstate), ptr(S_out), ctypes.byref(rule.c_rule), ptr(theta), ptr(m), ptr(v),
            int(step), float(lr), float(betas[0]), float(betas[1]), float(eps), stream_ptr()))

    def _workspace_bytes_at(self, which, n):
        off = ctypes.c_long()
        check(self._fn("workspace_offset")(which, self.max_samples, ctypes.byref(off)))
        ws = getattr(self, "last_workspace", None)      # the last pass's (pipelined: alternating)
        ws = self.workspace if ws is None else ws
        return ws[off.value:off.value + n]

    def workspace_view(self, which, shape, dtype=torch.float32, samples=None):
        """Debug view of a workspace tensor by id (PN1Engine.WORKSPACE / VGG11Engine.WORKSPACE).
        A tensor the engine stores in the split-bf16 form (HM + L parts, csrc/split.h) comes back
        as its fp32 values, (h + m) + l, which is exact: a copy, not a view."""
        n = int(np.prod(shape)) * torch.tensor([], dtype=dtype).element_size()
        lpart = self.split_part(which)
        if lpart < 0 or dtype != torch.float32:
            return self._workspace_bytes_at(which, n).view(dtype).view(shape)
        units = int(np.prod(shape)) // 4
        hm = self._workspace_bytes_at(which, n).view(torch.int16).view(units, 2, 4)
        lo = self._workspace_bytes_at(lpart, n // 2).view(torch.int16).view(units, 4)

        def f32(b):         # bf16 bits -> fp32 (exact)
            return (b.to(torch.int32) << 16).view(torch.float32)
        vals = (f32(hm[:, 0]) + f32(hm[:, 1])) + f32(lo)
        if self.slice_major(which):
            # stored [N][C/16][H][W][16] (loaders.h XsSrcSM): back to [N][H][W][C]
            n, h, w, c = shape
            return vals.view(n, c // 16, h, w, 16).permute(0, 2, 3, 1, 4).reshape(shape)
        return vals.view(shape)

    def slice_major(self, which):
        """True when workspace tensor `which` is stored channel-slice-major (PN1's a1, d1, a3)."""
        try:
            fn = self._fn("workspace_slice_major")
        except AttributeError:
            return False
        return bool(fn(which))

    def split_part(self, which):
        """Workspace id of tensor `which`'s L part when it is stored split, else -1."""
        fn = getattr(self, "_split_fn", None)
        if fn is None:
            try:
                fn = self._fn("workspace_split_part")
            except AttributeError:
                fn = lambda w: -1      # noqa: E731  (networks whose tensors are all fp32)
            self._split_fn = fn
        return int(fn(which))

    # -- server step ------------------------------------------------------------------------------
    def aggregate_adam(self, S, c, stale, theta, m, v, step, lr=1e-3, betas=(0.9, 0.999),
                       eps=1e-8):
        """stale: list of device tensors (or None = zero entry)."""
        aggregate_adam(S, c, stale, theta, m, v, step, self.SIZES, lr, betas, eps)

    def aggregate_adam_sum(self, S, k, theta, m, v, step, lr=1e-3, betas=(0.9, 0.999), eps=1e-8):
        aggregate_adam_sum(S, k, theta, m, v, step, self.SIZES, lr, betas, eps)

    def aggregate_rule(self, S, rule, theta, m, v, step, lr=1e-3, betas=(0.9, 0.999), eps=1e-8,
                       S_out=None):
        """rule() + Adam from S_t in a buffer; S_out (optional): S_t is also written there in
        the same pass (the FIFO slot of a tick epoch at world > 1)."""
        aggregate_rule(S, rule, theta, m, v, step, self.SIZES, lr, betas, eps, S_out=S_out)


class PN1Engine(NetEngine):
    PREFIX = "pn1"
    MODEL = "PerformantNet1"
    PIPELINE = True
    SHAPES = PN1_SHAPES
    FLOP_PER_WORKER_STEP = 147_641_499_648
    WORKSPACE = ("x0 a1 a2 d1 a3 a4 d2 a5 a6 d3 e1 e2 dh1 dh2 gx gy loss_s dlog y i1 i2 i3").split()


class VGG11Engine(NetEngine):
    PREFIX = "vgg11"
    MODEL = "vgg11"
    SHAPES = VGG11_SHAPES
    FLOP_PER_WORKER_STEP = 117_276_672_000          # 916,224,000 FLOP/sample x 128
    WORKSPACE = ("x0 d1 d2 a3 d4 a5 d6 a7 f0 e1 e2 dh1 dh2 ga gb gy loss_s dlog y "
                 "i1 i2 i4 i6 i8").split()

    def _slot_workspace(self, slot):
        return self.workspace                 # one workspace: the vgg11 facade has no pipeline

    def fwd_bwd_loaded_rows(self, theta, n_rows, workers_dev, seed, dropout, loss_out):
        """The facade's deferred fwd_bkwd: forward, loss and backward of the staged rows
        [0, n_rows) (load_rows) as one batched chunk; loss_out[g] = call g's loss."""
        check(lib().flsim_vgg11_fwd_bwd_loaded_rows(
            ptr(self.gradstate), ptr(self.workspace), self.max_samples, int(n_rows), ptr(theta),
            ptr(workers_dev), ctypes.c_uint64(seed), int(bool(dropout)), ptr(loss_out),
            stream_ptr()))


class VGG11BNEngine(NetEngine):
    """models.py:106-108 vgg11_bn() through flsim_vgg11_bn_*.  Holds the model's BatchNorm
    buffers: `running` = [running_mean | running_var] per layer on the device (zeros / ones at
    construction, nn.BatchNorm2d's init) and the num_batches_tracked counter (the same for every
    layer: each fwd_bkwd call updates all of them)."""
    PREFIX = "vgg11_bn"
    MODEL = "vgg11_bn"
    SHAPES = VGG11_BN_SHAPES
    FLOP_PER_WORKER_STEP = 117_276_672_000          # the GEMMs of vgg11 (BatchNorm is streaming)
    STATS_PER_WORKER = 5504
    WORKSPACE = ("x0 d1 d2 a3 d4 a5 d6 a7 f0 e1 e2 dh1 dh2 ga gb gy loss_s dlog y "
                 "i1 i2 i4 i6 i8 " + " ".join(f"z{j}" for j in range(8)) + " " +
                 " ".join(f"bmean{j}" for j in range(8)) + " " +
                 " ".join(f"binv{j}" for j in range(8))).split()

    def __init__(self, device, chunk_workers=32):
        super().__init__(device, chunk_workers)
        assert int(lib().flsim_vgg11_bn_stats_per_worker()) == self.STATS_PER_WORKER
        self.running = torch.cat([torch.cat([torch.zeros(c), torch.ones(c)])
                                  for _, c in VGG11_BN_BUFFERS]).to(self.device)
        self.num_batches_tracked = 0

    def _slot_workspace(self, slot):
        return self.workspace                 # one workspace: the vgg11_bn facade has no pipeline

    def fwd_bwd_loaded_rows(self, theta, n_rows, workers_dev, seed, dropout, loss_out,
                            stats_out):
        """The facade's deferred fwd_bkwd: forward, loss and backward of the staged rows
        [0, n_rows) as one batched chunk; stats_out[g] = call g's BatchNorm statistics (for
        update_running), loss_out[g] = its loss."""
        check(lib().flsim_vgg11_bn_fwd_bwd_loaded_rows(
            ptr(self.gradstate), ptr(self.workspace), self.max_samples, int(n_rows), ptr(theta),
            ptr(workers_dev), ctypes.c_uint64(seed), int(bool(dropout)), ptr(loss_out),
            ptr(stats_out), stream_ptr()))

    def update_running(self, stats, n_workers):
        n = int(n_workers)
        if n:
            check(lib().flsim_vgg11_bn_update_running(ptr(self.running), ptr(stats), n,
                                                      stream_ptr()))
        self.num_batches_tracked += n

    def running_views(self):
        """[(name, running_mean view, running_var view)] per BatchNorm layer."""
        out, off = [], 0
        for name, c in VGG11_BN_BUFFERS:
            out.append((name, self.running[off:off + c], self.running[off + c:off + 2 * c]))
            off += 2 * c
        return out

    def buffer_state(self):
        out = []
        for name, rm, rv in self.running_views():
            out += [(f"{name}.running_mean", rm.detach().cpu().clone()),
                    (f"{name}.running_var", rv.detach().cpu().clone()),
                    (f"{name}.num_batches_tracked",
                     torch.tensor(self.num_batches_tracked, dtype=torch.int64))]
        return out

    def load_buffers(self, state):
        for name, rm, rv in self.running_views():
            rm.copy_(state[f"{name}.running_mean"].to(self.device))
            rv.copy_(state[f"{name}.running_var"].to(self.device))
        self.num_batches_tracked = int(state[f"{VGG11_BN_BUFFERS[0][0]}.num_batches_tracked"])


ENGINES = {"PerformantNet1": PN1Engine, "vgg11": VGG11Engine, "vgg11_bn": VGG11BNEngine}


def engine_class(model):
    if model not in ENGINES:
        raise NotImplementedError(f"model {model!r}: the HIP engine implements {sorted(ENGINES)}")
    return ENGINES[model]


def engine_for_parameters(names):
    """The engine class whose named_parameters layout is `names` (a models.py module)."""
    names = list(names)
    for cls in ENGINES.values():
        if names == [n for n, _ in cls.SHAPES]:
            return cls
    raise NotImplementedError("the HIP engine implements FL.models.PerformantNet1, vgg11 and "
                              "vgg11_bn")


def aggregate_adam(S, c, stale, theta, m, v, step, sizes, lr=1e-3, betas=(0.9, 0.999), eps=1e-8):
    """Fused rule() + Adam (main.py:23-25 + agents.py:9-21) over a flat parameter vector whose
    tensors have numel `sizes` (named_parameters order).  stale: device tensors or None (zeros)."""
    ns = len(stale)
    arr = (ctypes.c_void_p * max(1, ns))(*[(t.data_ptr() if t is not None else None)
                                           for t in stale])
    csz = (ctypes.c_long * len(sizes))(*[int(n) for n in sizes])
    check(lib().flsim_aggregate_adam(
        ptr(S), int(c), arr, ns, ptr(theta), ptr(m), ptr(v), sum(int(n) for n in sizes), csz, len(sizes),
        int(step), float(lr), float(betas[0]), float(betas[1]), float(eps), stream_ptr()))


def aggregate_adam_sum(S, k, theta, m, v, step, sizes, lr=1e-3, betas=(0.9, 0.999), eps=1e-8):
    """Independent-entry semantics: S = the sum of the k distinct weight_ups entries; mean = S / k
    then the same Adam step (flsim_aggregate_adam_sum)."""
    csz = (ctypes.c_long * len(sizes))(*[int(n) for n in sizes])
    check(lib().flsim_aggregate_adam_sum(
        ptr(S), int(k), ptr(theta), ptr(m), ptr(v), sum(int(n) for n in sizes), csz, len(sizes),
        int(step), float(lr), float(betas[0]), float(betas[1]), float(eps), stream_ptr()))


def cascade_program(k, events):
    """rule()'s summation program (host, flsim_cascade_program) for k entries whose non-S_t
    entries are events = [(position, array index)] (positions increasing).  -> (int32 words,
    info[4]).  The words are the device's macro form (csrc/cascade.h): (lo, hi) pairs."""
    ev = np.asarray(events, np.int32).reshape(-1, 2)
    pos = np.ascontiguousarray(ev[:, 0])
    arr = np.ascontiguousarray(ev[:, 1])
    cap = 2 * (72 + 40 * (len(ev) + 8))    # macro pairs (lo, hi) + the fetch-pad pair
    prog = np.zeros(cap, np.int32)
    info = np.zeros(4, np.int32)
    vp = ctypes.c_void_p
    check(lib().flsim_cascade_program(int(k), pos.ctypes.data_as(vp), arr.ctypes.data_as(vp),
                                      len(ev), prog.ctypes.data_as(vp), cap,
                                      info.ctypes.data_as(vp)))
    return prog[:2 * (info[0] + 1)].copy(), info      # with the padding pair


class Rule:
    """weight_ups of one rule() call (flsim_rule): k entries (the mean's divisor); either the
    reference order [S_t] * c + arrays, or a general order given as events [(position, array
    index)] whose program is built on the host and staged to the device (`stager`).  arrays:
    device tensors or None (a zero entry, torch-1.x)."""

    def __init__(self, k, arrays=(), c=None, events=None, stager=None):
        arrays = list(arrays)
        if len(arrays) > MAX_ARRAYS:
            raise NotImplementedError(f"{len(arrays)} distinct weight_ups arrays in one step "
                                      f"(max {MAX_ARRAYS})")
        r = FlsimRule()
        r.k = int(k)
        r.n_arrays = len(arrays)
        for q, a in enumerate(arrays):
            r.arrays[q] = a.data_ptr() if a is not None else None
        self.arrays = arrays            # keep the tensors alive with the rule
        self.k, self.c, self.events = int(k), c, events
        if events is None:
            r.c = int(c)
            r.prog = None
            self.prog_dev = None
        else:
            words, info = cascade_program(k, events)
            self.prog_dev = stager.upload(words)
            r.c = -1
            r.prog = self.prog_dev.data_ptr()
            for j in range(4):
                r.info[j] = int(info[j])
        self.c_rule = r


class ProgramStager:
    """Pinned host -> device staging of rule programs, double-buffered.  The host waits only for
    the copy out of a pinned buffer two uploads ago; the device buffer is rewritten two uploads
    later, behind (stream order) the launch that reads it now."""

    def __init__(self, device):
        self.device = torch.device(device)
        self.cap = 0
        self.i = 0

    def upload(self, words):
        n = int(words.size)
        if n > self.cap:
            self.cap = max(1024, 2 * n)
            pin = self.device.type == "cuda"
            self.host = [torch.empty(self.cap, dtype=torch.int32, pin_memory=pin) for _ in range(2)]
            self.dev = [torch.empty(self.cap, dtype=torch.int32, device=self.device)
                        for _ in range(2)]
            self.ev = [None, None]
        j = self.i = self.i ^ 1
        if self.ev[j] is not None:
            self.ev[j].synchronize()
        self.host[j][:n].numpy()[:] = words
        self.dev[j][:n].copy_(self.host[j][:n], non_blocking=True)
        if self.device.type == "cuda":
            ev = torch.cuda.Event()
            ev.record()
            self.ev[j] = ev
        return self.dev[j]


def aggregate_rule(S, rule, theta, m, v, step, sizes, lr=1e-3, betas=(0.9, 0.999), eps=1e-8,
                   S_out=None):
    """rule() + Adam from S_t in a buffer (flsim_aggregate_adam_rule_push; S_out may be None)."""
    csz = (ctypes.c_long * len(sizes))(*[int(n) for n in sizes])
    check(lib().flsim_aggregate_adam_rule_push(
        ptr(S), ptr(S_out), ctypes.byref(rule.c_rule), ptr(theta), ptr(m), ptr(v),
        sum(int(n) for n in sizes), csz, len(sizes), int(step), float(lr), float(betas[0]),
        float(betas[1]), float(eps), stream_ptr()))


def worker_table(recs, device):
    """recs: sequence of (t, i, k) -> device tensor of WorkerRec (uint32 x4)."""
    a = np.zeros((len(recs), 4), np.uint32)
    if len(recs):
        a[:, :3] = np.asarray(recs, np.int64).astype(np.uint32)
    return torch.from_numpy(a).to(device, non_blocking=True)
