"""The networks + Worker.fwd_bkwd + the server step, restated on torch-CPU -- TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.

  PerformantNet1Ref    models.py:11-25 (layer construction order => identical default init under
                       torch.manual_seed) and models.py:27-47 (forward) with dropout masks injected
                       from the build's Philox spec instead of torch's RNG
  VGG11Ref             models.py:101-103 vgg11(): make_layers(cfg 'A') then the classifier, then
                       the He-normal conv init of models.py:67-71 (same RNG draw order); forward
                       models.py:73-77; the classifier's two Dropouts use Philox sites 6 and 7
  VGG11BNRef           models.py:106-108 vgg11_bn(): make_layers(cfg 'A', batch_norm=True) -- Conv2d,
                       BatchNorm2d, ReLU per conv (models.py:88-89); BatchNorm in train mode uses
                       the batch statistics of each fwd_bkwd call (one worker's 128 samples) and
                       updates running_mean / running_var (momentum 0.1, unbiased var) on every
                       call, in worker order; eval mode (util.py:31-45) normalises with them
  fwd_bkwd             agents.py:32-40 (forward, CrossEntropyLoss mean, backward accumulating into
                       the shared .grad, returns the loss)
  OracleSim            main.py:126-188: per-epoch worker loop (schedule from oracle.schedule),
                       aggregation rule main.py:23-25 (oracle.cascade_mean == torch stack-mean),
                       Central.update_model agents.py:9-21 (oracle.adam_step == torch Adam); the
                       model is PerformantNet1 (main.py:97) or vgg11 (configs[4])
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import oracle as O

PARAM_NAMES = [
    "conv1.weight", "conv1.bias", "conv2.weight", "conv2.bias", "conv3.weight", "conv3.bias",
    "conv4.weight", "conv4.bias", "conv5.weight", "conv5.bias", "conv6.weight", "conv6.bias",
    "linear1.weight", "linear1.bias", "linear2.weight", "linear2.bias", "linear3.weight",
    "linear3.bias",
]

# NCHW shapes (per sample) at the five dropout sites, models.py:32,36,40,43,45
DROPOUT_SHAPES = [(48, 18, 18), (96, 11, 11), (192, 7, 7), (512,), (256,)]

# models.py:96-98 cfg 'A'; the classifier's Dropout() x2 (models.py:58,61): (site, p, shape)
VGG_CFG = (64, "M", 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M")
VGG_DROPOUT = tuple((site, 0.5, (512,)) for site in O.SITE_VGG_DROPOUT)


class PerformantNet1Ref(nn.Module):
    """Same parameter set and construction order as models.py:13-25."""

    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 48, 3, padding=(2, 2))
        self.conv2 = nn.Conv2d(48, 48, 3, padding=(2, 2))
        self.conv3 = nn.Conv2d(48, 96, 3, padding=(2, 2))
        self.conv4 = nn.Conv2d(96, 96, 3, padding=(2, 2))
        self.conv5 = nn.Conv2d(96, 192, 3, padding=(2, 2))
        self.conv6 = nn.Conv2d(192, 192, 3, padding=(2, 2))
        self.linear1 = nn.Linear(9408, 512)
        self.linear2 = nn.Linear(512, 256)
        self.linear3 = nn.Linear(256, 10)


class VGG11Ref(nn.Module):
    """vgg11() of models.py:101-103: the feature layers are built first (models.py:80-93; each
    Conv2d's default init draws from the RNG), then the classifier's Linears (models.py:57-65),
    then every conv weight is redrawn N(0, sqrt(2 / (9 * out_channels))) and its bias zeroed
    (models.py:67-71).  Parameter names match (features.0, ..., classifier.6)."""

    def __init__(self):
        super().__init__()
        layers, c = [], 3
        for v in VGG_CFG:
            if v == "M":
                layers.append(nn.MaxPool2d(kernel_size=2, stride=2))
            else:
                layers += [nn.Conv2d(c, v, kernel_size=3, padding=1), nn.ReLU(inplace=True)]
                c = v
        self.features = nn.Sequential(*layers)
        self.classifier = nn.Sequential(
            nn.Dropout(), nn.Linear(512, 512), nn.ReLU(True),
            nn.Dropout(), nn.Linear(512, 512), nn.ReLU(True), nn.Linear(512, 10))
        for mod in self.modules():
            if isinstance(mod, nn.Conv2d):
                fan = mod.kernel_size[0] * mod.kernel_size[1] * mod.out_channels
                mod.weight.data.normal_(0, math.sqrt(2.0 / fan))
                mod.bias.data.zero_()


class VGG11BNRef(nn.Module):
    """vgg11_bn() of models.py:106-108: as VGG11Ref with a BatchNorm2d(v) after every conv
    (models.py:88-89; weight 1, bias 0, no RNG draw).  Parameter names match (features.0,
    features.1, features.4, ...)."""

    def __init__(self):
        super().__init__()
        layers, c = [], 3
        for v in VGG_CFG:
            if v == "M":
                layers.append(nn.MaxPool2d(kernel_size=2, stride=2))
            else:
                layers += [nn.Conv2d(c, v, kernel_size=3, padding=1), nn.BatchNorm2d(v),
                           nn.ReLU(inplace=True)]
                c = v
        self.features = nn.Sequential(*layers)
        self.classifier = nn.Sequential(
            nn.Dropout(), nn.Linear(512, 512), nn.ReLU(True),
            nn.Dropout(), nn.Linear(512, 512), nn.ReLU(True), nn.Linear(512, 10))
        for mod in self.modules():
            if isinstance(mod, nn.Conv2d):
                fan = mod.kernel_size[0] * mod.kernel_size[1] * mod.out_channels
                mod.weight.data.normal_(0, math.sqrt(2.0 / fan))
                mod.bias.data.zero_()


VGG_BN_CHANNELS = tuple(v for v in VGG_CFG if v != "M")


class BNState:
    """The BatchNorm2d buffers of vgg11_bn (running_mean, running_var per layer, one
    num_batches_tracked counter for all of them) and the module mode (train / eval)."""

    def __init__(self, dtype=torch.float32):
        self.training = True
        self.bufs = [(torch.zeros(c, dtype=dtype), torch.ones(c, dtype=dtype))
                     for c in VGG_BN_CHANNELS]
        self.num_batches_tracked = 0

    def flat(self):
        """[rm_0, rv_0, rm_1, rv_1, ...] (the engine's running-buffer layout) as float64 numpy."""
        return torch.cat([torch.cat([rm, rv]) for rm, rv in self.bufs]).double().numpy()

    def load_flat(self, a, dtype=torch.float32):
        a = torch.as_tensor(np.asarray(a)).to(dtype)
        off = 0
        for j, c in enumerate(VGG_BN_CHANNELS):
            self.bufs[j] = (a[off:off + c].clone(), a[off + c:off + 2 * c].clone())
            off += 2 * c


def forward(params, x, noise):
    """models.py:27-47 with dropout = x * noise (noise None -> eval mode / dropout off)."""
    (w1, b1, w2, b2, w3, b3, w4, b4, w5, b5, w6, b6, l1w, l1b, l2w, l2b, l3w, l3b) = params
    bs = x.shape[0]
    d = (lambda h, i: h) if noise is None else (lambda h, i: h * noise[i])
    h = F.relu(F.conv2d(x, w1, b1, padding=2))
    h = F.relu(F.conv2d(h, w2, b2, padding=2))
    h = d(F.max_pool2d(h, 2, 2), 0)
    h = F.relu(F.conv2d(h, w3, b3, padding=2))
    h = F.relu(F.conv2d(h, w4, b4, padding=2))
    h = d(F.max_pool2d(h, 2, 2), 1)
    h = F.relu(F.conv2d(h, w5, b5, padding=2))
    h = F.relu(F.conv2d(h, w6, b6, padding=2))
    h = d(F.max_pool2d(h, 2, 2), 2)
    h = h.reshape(bs, -1)
    h = d(F.relu(F.linear(h, l1w, l1b)), 3)
    h = d(F.relu(F.linear(h, l2w, l2b)), 4)
    return F.linear(h, l3w, l3b)


def vgg_forward(params, x, noise):
    """models.py:73-77: make_layers' conv3x3 (padding 1) + ReLU and 2x2 max-pools
    (models.py:80-93), flatten, classifier Dropout -> Linear -> ReLU -> Dropout -> Linear -> ReLU
    -> Linear (models.py:57-65); dropout = x * noise (noise None -> eval mode)."""
    convs = params[:16]
    l1w, l1b, l2w, l2b, l3w, l3b = params[16:]
    d = (lambda h, i: h) if noise is None else (lambda h, i: h * noise[i])
    h, j = x, 0
    for v in VGG_CFG:
        if v == "M":
            h = F.max_pool2d(h, 2, 2)
        else:
            h = F.relu(F.conv2d(h, convs[2 * j], convs[2 * j + 1], padding=1))
            j += 1
    h = h.reshape(x.shape[0], -1)
    h = F.relu(F.linear(d(h, 0), l1w, l1b))
    h = F.relu(F.linear(d(h, 1), l2w, l2b))
    return F.linear(h, l3w, l3b)


def vgg_bn_forward(params, x, noise, bn=None):
    """models.py:73-77 for vgg11_bn: conv3x3 -> BatchNorm2d -> ReLU (models.py:88-89), pools and
    the classifier as vgg_forward.  bn: BNState (train mode: batch statistics of x, running
    buffers updated in place, counter += 1; eval mode: normalise with the running buffers);
    None = train mode without running buffers (gradient-only probes)."""
    convs = params[:32]
    l1w, l1b, l2w, l2b, l3w, l3b = params[32:]
    d = (lambda h, i: h) if noise is None else (lambda h, i: h * noise[i])
    training = bn is None or bn.training
    h, j = x, 0
    for v in VGG_CFG:
        if v == "M":
            h = F.max_pool2d(h, 2, 2)
        else:
            cw, cb, gw, gb = convs[4 * j:4 * j + 4]
            h = F.conv2d(h, cw, cb, padding=1)
            rm, rv = bn.bufs[j] if bn is not None else (None, None)
            h = F.relu(F.batch_norm(h, rm, rv, gw, gb, training, 0.1, 1e-5))
            j += 1
    if bn is not None and training:
        bn.num_batches_tracked += 1
    h = h.reshape(x.shape[0], -1)
    h = F.relu(F.linear(d(h, 0), l1w, l1b))
    h = F.relu(F.linear(d(h, 1), l2w, l2b))
    return F.linear(h, l3w, l3b)


class _Net:
    """One models.py network: module (parameter set + init), forward, and its dropout sites in
    call order as (Philox site, p, per-sample shape)."""

    def __init__(self, module, fwd, dropout):
        self.module, self.forward, self.dropout = module, fwd, dropout
        self._shapes = None

    def shapes(self):
        if self._shapes is None:
            state = torch.random.get_rng_state()     # a shape probe must not move the RNG
            self._shapes = [(n, tuple(p.shape)) for n, p in self.module().named_parameters()]
            torch.random.set_rng_state(state)
        return self._shapes


NETS = {
    "PerformantNet1": _Net(PerformantNet1Ref, forward,
                           tuple(zip(O.SITE_DROPOUT, O.DROPOUT_P, DROPOUT_SHAPES))),
    "vgg11": _Net(VGG11Ref, vgg_forward, VGG_DROPOUT),
    "vgg11_bn": _Net(VGG11BNRef, vgg_bn_forward, VGG_DROPOUT),
}
HAS_BN = {"vgg11_bn"}


def init_params(seed=0, model="PerformantNet1"):
    """torch default init of the model under torch.manual_seed(seed) -> flat fp32 numpy."""
    torch.manual_seed(seed)
    m = NETS[model].module()
    return torch.cat([p.detach().reshape(-1) for _, p in m.named_parameters()]).numpy().copy()


def param_shapes(model="PerformantNet1"):
    return list(NETS[model].shapes())


def _shapes(model="PerformantNet1"):
    return NETS[model].shapes()


def split_flat(flat, model="PerformantNet1"):
    """flat numpy/torch vector -> list of per-tensor views (named_parameters order)."""
    out, off = [], 0
    for _, shp in _shapes(model):
        n = int(np.prod(shp))
        out.append(flat[off:off + n].reshape(shp))
        off += n
    return out


def dropout_noise(seed, t, worker, nsamples, dtype=torch.float32, model="PerformantNet1"):
    """The model's dropout noise tensors (keep * fp32(1/(1-p))) for one worker-step, NCHW."""
    res = []
    for site, p, shp in NETS[model].dropout:
        numel = nsamples * int(np.prod(shp))
        keep = O.dropout_keep(seed, t, worker, site, p, numel)
        noise = torch.from_numpy(keep).reshape((nsamples,) + shp).to(torch.float32).div_(1 - p)
        res.append(noise.to(dtype))
    return res


GROUP_KEY_STRIDE = 1 << 20


def batch_noise(seed, t, worker, nsamples, dtype=torch.float32, model="PerformantNet1"):
    """Dropout noise of a worker's batch of any size: 128-sample group g keyed (t, worker +
    g * 2^20) (the build's spec for --batch_size != 128), the groups'
    samples concatenated and cut to nsamples.  nsamples = 128: dropout_noise itself."""
    if nsamples == 128:
        return dropout_noise(seed, t, worker, 128, dtype, model)
    groups = -(-nsamples // 128)
    per = [dropout_noise(seed, t, worker + g * GROUP_KEY_STRIDE, 128, dtype, model)
           for g in range(groups)]
    return [torch.cat([p[s] for p in per])[:nsamples] for s in range(len(per[0]))]


def fwd_bkwd(params, x, y, noise, fwd=forward):
    """agents.py:32-40: loss = CE(mean) ; backward() accumulates into p.grad ; returns loss."""
    pred = fwd(params, x, noise)
    loss = F.cross_entropy(pred, y)
    loss.backward()
    return loss.detach()


class OracleSim:
    """main.py:126-188 restated on CPU, reference (torch>=2 aliasing), torch1 (stale = zeros) or
    independent semantics (every weight_ups entry a distinct per-worker gradient; a slow worker's
    FIFO holds its own gradient; rule() is the same per-tensor stack-mean, main.py:23-25)."""

    def __init__(self, n, delay=None, delays=None, throttle=False, seed=0, dtype=torch.float32,
                 semantics="reference", dropout=True, pool=None, lr=1e-3, theta0=None,
                 max_throttle=32, model="PerformantNet1", batch_size=128):
        self.n = n
        self.batch_size = int(batch_size)      # main.py:43-44 --batch_size
        self.delays = np.asarray(delays if delays is not None else O.reference_delays(n, delay),
                                 np.int32)
        self.throttle = bool(throttle)
        self.seed = seed
        self.dtype = dtype
        self.semantics = semantics
        self.dropout = dropout
        self.lr = lr
        self.max_throttle = max_throttle
        self.model = model
        self.net = NETS[model]
        self.bn = BNState(dtype) if model in HAS_BN else None
        imgs, labels = pool if pool is not None else O.make_pool(seed)
        self.imgs, self.labels = imgs, labels
        self.lists = O.class_lists(labels)
        self.lut = O.normalize_lut()
        theta0 = init_params(seed, model) if theta0 is None else theta0
        self.theta = np.ascontiguousarray(theta0, np.float32).copy()
        self.m = np.zeros_like(self.theta)
        self.v = np.zeros_like(self.theta)
        self.step_count = 0
        self.rs = np.random.RandomState(seed)   # main.py:138 global numpy RNG stream
        self.t = 0
        self.ring = {}                           # epoch -> S (stale entries kept alive)
        self.window = 0
        self.gone = False
        self.fifo = {i: [] for i in range(n) if self.delays[i] != 0}
        self.trace = []

    # ---- data (main.py:138-142) ----
    def batch(self, t, i, k, dtype=None):
        idx = O.batch_indices(self.seed, t, i, k, self.n, self.lists, self.batch_size)
        x = self.lut[self.imgs[idx]]                      # [B,3,32,32] fp32
        y = self.labels[idx]
        dt = dtype or self.dtype
        return torch.from_numpy(x).to(dt), torch.from_numpy(y)

    def grad_of(self, theta_np, items, dtype=None, bn=None):
        """Sum over `items` [(t, i, k)] of per-worker mean-CE gradients at theta (in order).
        BatchNorm models: bn = a BNState to run the forwards against (train mode, buffers
        updated), False = batch statistics only, None = the simulation's own buffers (when dtype
        is the simulation's)."""
        dt = dtype or self.dtype
        if self.bn is not None and bn is None:
            bn = self.bn if dt == self.dtype else False
        fwd = self.net.forward
        if self.bn is not None:
            st = bn if bn else None
            fwd = lambda p, x, noise: vgg_bn_forward(p, x, noise, st)   # noqa: E731
        params = [torch.tensor(a, dtype=dt, requires_grad=True)
                  for a in split_flat(theta_np.astype(np.float64 if dt == torch.float64
                                                      else np.float32), self.model)]
        losses = []
        for (t, i, k) in items:
            x, y = self.batch(t, i, k, dt)
            noise = batch_noise(self.seed, t, i, x.shape[0], dt, self.model) \
                if self.dropout else None
            losses.append(float(fwd_bkwd(params, x, y, noise, fwd)))
        g = torch.cat([p.grad.reshape(-1) for p in params]).numpy()
        return g, losses

    # ---- one epoch (main.py:126-188) ----
    def epoch(self):
        t, n = self.t, self.n
        ks = self.rs.randint(0, n, size=n)
        items, fast_losses_idx, appended = [], [], []
        ent_src = []                  # independent: ("item", j) or ("own", worker, source epoch)
        pushed_own = {}               # independent: (worker, t) -> item index
        for i in range(n):
            if self.delays[i] != 0:
                self.gone = False
                d = abs(int(self.delays[i]))
                popped = None
                if t == 0:
                    items.append((t, i, int(ks[i])))
                    self.fifo[i].append(t)
                    pushed_own[(i, t)] = len(items) - 1
                elif t % d == 0:
                    items.append((t, i, int(ks[i])))
                    self.fifo[i].append(t)
                    pushed_own[(i, t)] = len(items) - 1
                    popped = self.fifo[i].pop(0)
                if popped is not None:
                    appended.append(("stale", popped))
                    ent_src.append(("own", i, popped))
                    self.gone = True
            else:
                if self.window <= 0:
                    fast_losses_idx.append(len(items))
                    ent_src.append(("item", len(items)))
                    items.append((t, i, int(ks[i])))
                    appended.append(("fast", t))
                    if self.throttle:
                        self.window = 1
                        if not self.gone:
                            self.window = min(self.window * 2, self.max_throttle)
            if self.window > 0:
                self.window -= 1
        if not appended:
            raise IndexError("list index out of range")   # rule(): ups_list[0] (main.py:25)
        if self.semantics == "independent":
            per = [self.grad_of(self.theta, [it]) for it in items]
            gi = [g.astype(np.float32) for g, _ in per]
            losses = [ls[0] for _, ls in per]
            if not hasattr(self, "own"):
                self.own = {}
            for key, j in pushed_own.items():
                self.own[key] = gi[j]
            entries = [gi[e[1]] if e[0] == "item" else self.own.pop((e[1], e[2])) for e in ent_src]
            S = np.sum(np.stack(gi), 0).astype(np.float32) if gi else None
            return self._finish(t, entries, S, losses, fast_losses_idx, items, appended)
        S, losses = self.grad_of(self.theta, items)
        S = S.astype(np.float32)
        entries = []
        for kind, src in appended:
            if kind == "fast":
                entries.append(S)
            else:
                entries.append(self.ring[src] if self.semantics == "reference"
                               else np.zeros_like(S))
        if any(self.delays[i] != 0 and (t == 0 or t % abs(int(self.delays[i])) == 0)
               for i in range(n)):
            self.ring[t] = S
        live = {src for q in self.fifo.values() for src in q}     # entries a FIFO still holds
        self.ring = {src: a for src, a in self.ring.items() if src in live}
        return self._finish(t, entries, S, losses, fast_losses_idx, items, appended)

    def _finish(self, t, entries, S, losses, fast_losses_idx, items, appended):
        """rule() over the weight_ups entries + Adam + loss logging (main.py:184-188)."""
        g = np.empty_like(entries[0])
        off = 0
        for _, shp in _shapes(self.model):                # rule() is per parameter tensor
            nel = int(np.prod(shp))
            g[off:off + nel] = O.cascade_mean([e[off:off + nel] for e in entries])
            off += nel
        self.step_count += 1
        O.adam_step(self.theta, self.m, self.v, g, self.step_count, lr=self.lr)
        mean_loss = float(np.mean(np.asarray([losses[j] for j in fast_losses_idx], np.float32)))\
            if fast_losses_idx else float("nan")
        self.trace.append(dict(t=t, items=items, appended=appended, loss=mean_loss))
        self.t += 1
        self.last_S, self.last_g = S, g
        return mean_loss


def O_init(seed):
    return init_params(seed)


def predict(theta_np, imgs_u8, batch=500, model="PerformantNet1", bn=None):
    """util.py:31-45 forward in eval mode (no dropout): argmax of the logits per image (torch.max
    -> first maximum), fp32 torch CPU.  imgs_u8: [n, 3, 32, 32] uint8 pool images."""
    params = [torch.from_numpy(a) for a in split_flat(theta_np.astype(np.float32), model)]
    lut = O.normalize_lut()
    fwd = NETS[model].forward
    if model in HAS_BN:              # eval mode: the running buffers (bn: BNState or flat array)
        st = bn if isinstance(bn, BNState) else BNState()
        if not isinstance(bn, BNState) and bn is not None:
            st.load_flat(bn)
        was, st.training = st.training, False
        fwd = lambda p, x, noise: vgg_bn_forward(p, x, noise, st)   # noqa: E731
    out = []
    with torch.no_grad():
        for s in range(0, len(imgs_u8), batch):
            x = torch.from_numpy(lut[imgs_u8[s:s + batch]])
            out.append(torch.max(fwd(params, x, None), 1)[1].numpy())
    if model in HAS_BN:
        st.training = was
    return np.concatenate(out).astype(np.int32)
