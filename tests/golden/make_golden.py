"""Generate golden fixtures by running the REFERENCE itself (build container only).

Run:  python tests/golden/make_golden.py   (needs /root/reference; never runs on the GPU box)

What is executed from the reference (read-only, imported/exec'd, never copied):
  * FL/agents.py  Central / Worker / Agg          (real classes)
  * FL/models.py  PerformantNet1, vgg11, vgg11_bn (real modules, their own init)
  * main.py:23-25 rule()                          (exec'd from the parsed AST)
  * main.py:126-203 the training loop `for t in tqdm(range(n_epochs)):` (exec'd from the AST)
with stubs for the I/O the container cannot provide (main.py:8,15,70-73,141 -- torchvision,
tensorboard, CIFAR10 download, DataLoader.next()):
  * trainloaders: n stub loaders whose iterators expose .next() and return batches drawn by the
    build's data spec (oracle.batch_indices) -- the k index comes from the reference's own
    np.random.randint (main.py:138) under np.random.seed(seed)
  * torch.nn.functional.dropout patched to use the build's Philox keep-masks with torch's own
    noise arithmetic (bernoulli -> div_(1-p) -> input * noise)
  * writer.add_scalar recorder, tqdm = identity, print_test_accuracy -> 10 zeros

Outputs (data only; no reference source is written): tests/golden/*.npz, meta.json
"""
import ast
import hashlib
import json
import os
import sys

sys.dont_write_bytecode = True
REF = os.environ.get("FLSIM_REFERENCE", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REF)
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from FL.agents import Agg, Central, Worker  # noqa: E402  (reference)
from FL.models import PerformantNet1  # noqa: E402  (reference)
from oracle import oracle as O  # noqa: E402

torch.set_num_threads(8)

_SRC = open(os.path.join(REF, "main.py")).read()
_TREE = ast.parse(_SRC)


def _rule_fn():
    node = [n for n in _TREE.body if isinstance(n, ast.FunctionDef) and n.name == "rule"][0]
    ns = {"torch": torch}
    exec(compile(ast.Module(body=[node], type_ignores=[]), "main.py", "exec"), ns)
    return ns["rule"]


def _loop_code():
    main_if = [n for n in _TREE.body if isinstance(n, ast.If)][0]
    loop = [n for n in main_if.body if isinstance(n, ast.For) and n.lineno == 126][0]
    assert loop.lineno == 126, loop.lineno
    return compile(ast.Module(body=[loop], type_ignores=[]), "main.py", "exec")


RULE = _rule_fn()
LOOP = _loop_code()


class _Args:
    def __init__(self, delay, throttle):
        self.delay, self.throttle = delay, throttle


class _Writer:
    def __init__(self):
        self.scalars = []

    def add_scalar(self, tag, val, t):
        self.scalars.append((tag, float(val), int(t)))


class _Ctx:
    """Tracks which (t, i) is being computed; set by the stub iterator's next()."""
    t = 0
    i = 0
    calls = 0
    n = 0
    draws = 0


def _run_loop(ns):
    exec(LOOP, ns)


# ---------------------------------------------------------------------------------------------
# (1) schedule traces: real control flow, stubbed compute
# ---------------------------------------------------------------------------------------------
def schedule_trace(n, delay, throttle, n_epochs, seed=0):
    np.random.seed(seed)
    ctx = _Ctx()
    ctx.n = n
    kseq = []

    class It:
        def __init__(self, k):
            self.k = k

        def __iter__(self):
            return self

        def __next__(self):
            return self.next()

        def next(self):
            kseq.append(self.k)
            ctx.i = ctx.draws % n
            ctx.t = ctx.draws // n
            ctx.draws += 1
            return torch.zeros(1), torch.zeros(1)

    class Loader:
        def __init__(self, k):
            self.k = k

        def __iter__(self):
            return It(self.k)

    computes = np.zeros((n_epochs, n), np.uint8)
    tokens = {}

    class StubWorker:
        def __init__(self):
            self.model = None

        def fwd_bkwd(self, inp, outp):
            computes[ctx.t, ctx.i] = 1
            tok = tokens.setdefault(ctx.t, ("G", ctx.t))   # aliased per-epoch grad (agents.py:37-39)
            return tok, np.float32(0.0)

    comp_src = []

    def rec_rule(ups):
        comp_src.append([u[1] for u in ups])
        return None

    class StubCentral:
        model = type("M", (), {"train": lambda s: None, "eval": lambda s: None})()

        def update_model(self, ups):
            pass

    ns = dict(
        tqdm=lambda x: x, range=range, np=np, time=__import__("time"), torch=torch,
        trainloaders=[Loader(k) for k in range(n)], device="cpu", central=StubCentral(),
        worker_list=[StubWorker() for _ in range(n)], agg=Agg(rec_rule), writer=_Writer(),
        args=_Args(delay, throttle), n_workers=n, n_epochs=n_epochs, save_model=False,
        model=None, testloader=None, print_test_accuracy=lambda m, l: [0.0] * 10,
        epochs=[], accuracies=[], pesky_worker_grads=[], throttle_window=0, max_throttle=32,
        slow_guy_gone=False,
    )
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        _run_loop(ns)
    # stale source per epoch: entries of weight_ups whose epoch != t
    c_t = np.array([sum(1 for s in src if s == t) for t, src in enumerate(comp_src)], np.int32)
    stale = np.array([[s for s in src if s != t][0] if any(s != t for s in src) else -1
                      for t, src in enumerate(comp_src)], np.int64)
    kseq = np.asarray(kseq, np.int64).reshape(n_epochs, n)
    return computes, c_t, stale, kseq, int(ns["throttle_window"]), bool(ns["slow_guy_gone"])


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def make_schedule_fixtures():
    out = {}
    configs = []
    for n in (2, 3, 10, 20, 1024):
        for d in (1, 3, 50, 500):
            for thr in (False, True):
                ep = 1500 if n <= 20 else 600
                configs.append((n, d, thr, ep))
    for (n, d, thr, ep) in configs:
        comp, c_t, stale, kseq, w, g = schedule_trace(n, d, thr, ep)
        key = f"n{n}_d{d}_thr{int(thr)}_e{ep}"
        out[key + "_computes"] = np.packbits(comp, axis=1)
        out[key + "_c_t"] = c_t
        out[key + "_stale"] = stale
        out[key + "_k_sha"] = np.frombuffer(bytes.fromhex(_sha(kseq.astype(np.int64))), np.uint8)
        out[key + "_k_head"] = kseq[:3].astype(np.int32)
        out[key + "_final"] = np.array([w, int(g)], np.int64)
        print("schedule", key, "executed fwd_bkwd", int(comp.sum()))
    np.savez_compressed(os.path.join(HERE, "schedule.npz"), **out)


# ---------------------------------------------------------------------------------------------
# (2) cascade-mean known answers through the reference's rule() (main.py:23-25)
# ---------------------------------------------------------------------------------------------
def make_cascade_fixtures():
    out = {}
    sizes = [10, 48, 1296, 2560, 4096]
    for k in (1, 2, 5, 9, 17, 33, 100, 257, 513, 1024, 1025):
        for P in sizes:
            rs = np.random.RandomState(1000 * k + P)
            S = rs.standard_normal(P).astype(np.float32)
            st = rs.standard_normal(P).astype(np.float32)
            # weight_ups shape at a tick: (k-1) aliased copies of S_t then the stale entry
            ups = [[torch.from_numpy(S)]] * (k - 1) + [[torch.from_numpy(st)]]
            res = RULE(ups)[0].numpy()
            out[f"rep_k{k}_P{P}"] = res
            if k <= 257:
                ent = rs.standard_normal((k, P)).astype(np.float32)
                res2 = RULE([[torch.from_numpy(ent[j])] for j in range(k)])[0].numpy()
                out[f"rnd_k{k}_P{P}"] = res2
    np.savez_compressed(os.path.join(HERE, "cascade.npz"), **out)
    print("cascade fixtures", len(out))


# ---------------------------------------------------------------------------------------------
# (3) Adam through Central.update_model (agents.py:9-21) with optim.Adam(lr) (main.py:106)
# ---------------------------------------------------------------------------------------------
def make_adam_fixtures():
    sizes = [10, 300, 5000]
    rs = np.random.RandomState(7)
    p0 = [rs.standard_normal(s).astype(np.float32) for s in sizes]

    class M(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.a = torch.nn.Parameter(torch.from_numpy(p0[0].copy()))
            self.b = torch.nn.Parameter(torch.from_numpy(p0[1].copy()))
            self.c = torch.nn.Parameter(torch.from_numpy(p0[2].copy()))

    model = M()
    opt = torch.optim.Adam(model.parameters(), lr=0.001)
    central = Central(model, opt)
    out = {f"p0_{j}": p0[j] for j in range(3)}
    for step in range(1, 11):
        scale = 10.0 ** rs.uniform(-6, 0)
        grads = [(rs.standard_normal(s) * scale).astype(np.float32) for s in sizes]
        for j in range(3):
            out[f"g{step}_{j}"] = grads[j]
        central.update_model([torch.from_numpy(g.copy()) for g in grads])
        for j, p in enumerate(model.parameters()):
            st = opt.state[p]
            out[f"p{step}_{j}"] = p.detach().numpy().copy()
            out[f"m{step}_{j}"] = st["exp_avg"].numpy().copy()
            out[f"v{step}_{j}"] = st["exp_avg_sq"].numpy().copy()
    np.savez_compressed(os.path.join(HERE, "adam.npz"), **out)
    print("adam fixtures", len(out))


# ---------------------------------------------------------------------------------------------
# (4) real PerformantNet1 training, verbatim loop, build data + dropout spec
# ---------------------------------------------------------------------------------------------
SAMPLE_PER_TENSOR = 256


def sample_index(numel, seed=123):
    rs = np.random.RandomState(seed + numel)
    if numel <= SAMPLE_PER_TENSOR:
        return np.arange(numel)
    return np.sort(rs.choice(numel, SAMPLE_PER_TENSOR, replace=False))


def tensor_stats(ts):
    """per tensor: [sum, sum of squares, min, max] (float64) + sampled values."""
    st, samp = [], []
    for t in ts:
        a = t.detach().double().reshape(-1).numpy()
        st.append([a.sum(), (a * a).sum(), a.min(), a.max()])
        samp.append(a[sample_index(a.size)])
    return np.asarray(st), np.concatenate(samp)


def train_run(n, delay, throttle, n_epochs, seed=0, dtype=torch.float32, dropout=True,
              pool=None, model_fn=PerformantNet1, sites=O.SITE_DROPOUT, keep=None):
    imgs, labels = pool
    lists = O.class_lists(labels)
    lut = O.normalize_lut()
    np.random.seed(seed)
    torch.manual_seed(seed)
    model = model_fn()
    theta0 = torch.cat([p.detach().reshape(-1) for p in model.parameters()]).numpy().copy()
    if dtype == torch.float64:
        model = model.double()
    optimizer = torch.optim.Adam(model.parameters(), lr=0.001)
    loss = torch.nn.CrossEntropyLoss()
    central = Central(model, optimizer)
    ctx = _Ctx()

    class It:
        def __init__(self, k):
            self.k = k

        def __iter__(self):
            return self

        def __next__(self):
            return self.next()

        def next(self):
            t, i = ctx.draws // n, ctx.draws % n
            ctx.t, ctx.i, ctx.calls = t, i, 0
            ctx.draws += 1
            idx = O.batch_indices(seed, t, i, self.k, n, lists)
            x = torch.from_numpy(lut[imgs[idx]]).to(dtype)
            y = torch.from_numpy(labels[idx])
            return x, y

    class Loader:
        def __init__(self, k):
            self.k = k

        def __iter__(self):
            return It(self.k)

    real_dropout = F.dropout

    def spec_dropout(input, p=0.5, training=True, inplace=False):
        if not training or not dropout:
            return input
        site = sites[ctx.calls]
        ctx.calls += 1
        keep = O.dropout_keep(seed, ctx.t, ctx.i, site, p, input.numel())
        noise = torch.from_numpy(keep).reshape(input.shape).to(input.dtype).div_(1 - p)
        return input * noise

    agg_log = []

    def rec_rule(ups):
        fin = RULE(ups)
        # composition by identity (aliasing, agents.py:37-39)
        ids = [id(u[0]) for u in ups]
        agg_log.append(dict(S=tensor_stats(ups[0]) if ups else None,
                            fin=tensor_stats(fin), n_entries=len(ups),
                            n_distinct=len(set(ids))))
        return fin

    writer = _Writer()
    theta_log = []

    class LoggingCentral(Central):
        def update_model(self, ups):
            super().update_model(ups)
            theta_log.append(tensor_stats(list(self.model.parameters())))

    central = LoggingCentral(model, optimizer)
    ns = dict(
        tqdm=lambda x: x, range=range, np=np, time=__import__("time"), torch=torch,
        trainloaders=[Loader(k) for k in range(n)], device="cpu", central=central,
        worker_list=[Worker(loss) for _ in range(n)], agg=Agg(rec_rule), writer=writer,
        args=_Args(delay, throttle), n_workers=n, n_epochs=n_epochs, save_model=False,
        model=model, testloader=None, print_test_accuracy=lambda m, l: [0.0] * 10,
        epochs=[], accuracies=[], pesky_worker_grads=[], throttle_window=0, max_throttle=32,
        slow_guy_gone=False,
    )
    F.dropout = spec_dropout
    torch.nn.functional.dropout = spec_dropout
    try:
        _run_loop(ns)
    finally:
        F.dropout = real_dropout
        torch.nn.functional.dropout = real_dropout
    losses = np.array([v for (tag, v, t) in writer.scalars if tag == "Avg. Loss"], np.float64)
    if keep is not None:
        keep["model"] = model
    return theta0, losses, agg_log, theta_log


def make_train_fixtures(pool):
    out = {}
    configs = [(4, 2, False, 5), (4, 2, True, 5)]
    for (n, d, thr, ep) in configs:
        for dt, tag in ((torch.float32, "f32"), (torch.float64, "f64")):
            theta0, losses, agg_log, theta_log = train_run(n, d, thr, ep, dtype=dt, pool=pool)
            key = f"n{n}_d{d}_thr{int(thr)}_{tag}"
            out[key + "_theta0_sha"] = np.frombuffer(bytes.fromhex(_sha(theta0)), np.uint8)
            out[key + "_losses"] = losses
            for t, a in enumerate(agg_log):
                out[f"{key}_S{t}_stats"], out[f"{key}_S{t}_samp"] = a["S"]
                out[f"{key}_fin{t}_stats"], out[f"{key}_fin{t}_samp"] = a["fin"]
                out[f"{key}_comp{t}"] = np.array([a["n_entries"], a["n_distinct"]])
            for t, th in enumerate(theta_log):
                out[f"{key}_theta{t}_stats"], out[f"{key}_theta{t}_samp"] = th
            print("train", key, "losses", losses)
    np.savez_compressed(os.path.join(HERE, "train.npz"), **out)


def make_grad_fixture(pool):
    """Teacher-forced single worker-step gradient at theta0 (agents.py:32-40), f32 and f64,
    for worker (t=0, i=0, k=0) with dropout masks of the spec.  Sampled + stats."""
    imgs, labels = pool
    lists = O.class_lists(labels)
    lut = O.normalize_lut()
    out = {}
    for dt, tag in ((torch.float32, "f32"), (torch.float64, "f64")):
        torch.manual_seed(0)
        model = PerformantNet1()
        if dt == torch.float64:
            model = model.double()
        model.train()
        idx = O.batch_indices(0, 0, 0, 0, 4, lists)
        x = torch.from_numpy(lut[imgs[idx]]).to(dt)
        y = torch.from_numpy(labels[idx])
        real = F.dropout
        calls = [0]

        def spec(input, p=0.5, training=True, inplace=False):
            site = O.SITE_DROPOUT[calls[0]]
            calls[0] += 1
            keep = O.dropout_keep(0, 0, 0, site, p, input.numel())
            return input * torch.from_numpy(keep).reshape(input.shape).to(input.dtype).div_(1 - p)

        torch.nn.functional.dropout = spec
        try:
            w = Worker(torch.nn.CrossEntropyLoss())
            w.model = model
            grads, lossval = w.fwd_bkwd(x, y)
        finally:
            torch.nn.functional.dropout = real
        out[f"{tag}_loss"] = np.asarray(lossval, np.float64)
        out[f"{tag}_stats"], out[f"{tag}_samp"] = tensor_stats(grads)
        out[f"{tag}_x_sha"] = np.frombuffer(bytes.fromhex(_sha(x.float().numpy())), np.uint8)
    np.savez_compressed(os.path.join(HERE, "grad.npz"), **out)
    print("grad fixture loss", out["f32_loss"], out["f64_loss"])


def make_vgg_fixtures(pool):
    """configs[4]'s vgg11 (models.py:101-103), the reference's own module: init under
    torch.manual_seed(0) (sha), one worker-step gradient through the reference Worker.fwd_bkwd
    (f32 and f64; the classifier's two Dropouts get the spec's masks, sites 6 and 7), and a 3-epoch
    run of the verbatim loop main.py:126-203 with the model swapped for vgg11 (f32)."""
    from FL.models import vgg11  # noqa: E402  (reference)
    imgs, labels = pool
    lists = O.class_lists(labels)
    lut = O.normalize_lut()
    out = {}
    for dt, tag in ((torch.float32, "f32"), (torch.float64, "f64")):
        torch.manual_seed(0)
        model = vgg11()
        if dt == torch.float32:
            theta0 = torch.cat([p.detach().reshape(-1) for p in model.parameters()]).numpy()
            out["theta0_sha"] = np.frombuffer(bytes.fromhex(_sha(theta0)), np.uint8)
        else:
            model = model.double()
        model.train()
        idx = O.batch_indices(0, 0, 0, 0, 4, lists)
        x = torch.from_numpy(lut[imgs[idx]]).to(dt)
        y = torch.from_numpy(labels[idx])
        real = F.dropout
        calls = [0]

        def spec(input, p=0.5, training=True, inplace=False):
            site = O.SITE_VGG_DROPOUT[calls[0]]
            calls[0] += 1
            keep = O.dropout_keep(0, 0, 0, site, p, input.numel())
            return input * torch.from_numpy(keep).reshape(input.shape).to(input.dtype).div_(1 - p)

        torch.nn.functional.dropout = spec
        try:
            w = Worker(torch.nn.CrossEntropyLoss())
            w.model = model
            grads, lossval = w.fwd_bkwd(x, y)
        finally:
            torch.nn.functional.dropout = real
        assert calls[0] == 2
        out[f"{tag}_loss"] = np.asarray(lossval, np.float64)
        out[f"{tag}_stats"], out[f"{tag}_samp"] = tensor_stats(grads)
    theta0, losses, agg_log, theta_log = train_run(3, 2, True, 3, pool=pool, model_fn=vgg11,
                                                   sites=O.SITE_VGG_DROPOUT)
    out["train_losses"] = losses
    for t, th in enumerate(theta_log):
        out[f"train_theta{t}_stats"] = th[0]
    np.savez_compressed(os.path.join(HERE, "vgg.npz"), **out)
    print("vgg fixtures: loss", out["f32_loss"], out["f64_loss"], "train", losses)


def _bn_buffers(model):
    """running_mean, running_var of every BatchNorm2d in order, concatenated per layer
    [rm_0, rv_0, rm_1, rv_1, ...] (float64), and the layers' num_batches_tracked."""
    flat, nbt = [], []
    for mod in model.modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            flat += [mod.running_mean.double(), mod.running_var.double()]
            nbt.append(int(mod.num_batches_tracked))
    return torch.cat(flat).numpy(), np.asarray(nbt, np.int64)


def make_vgg_bn_fixtures(pool):
    """vgg11_bn (models.py:106-108), the reference's own module: init sha; one worker-step
    through the reference Worker.fwd_bkwd in train mode (f32 and f64: gradient stats + samples,
    the BatchNorm running buffers after the call); a 3-epoch run of the verbatim loop
    main.py:126-203 with the model swapped for vgg11_bn (losses, per-epoch parameter stats, the
    final running buffers) and the final model's eval-mode logits on 64 test images (util.py:31-45
    after central.model.eval(), main.py:190)."""
    from FL.models import vgg11_bn  # noqa: E402  (reference)
    imgs, labels = pool
    lists = O.class_lists(labels)
    lut = O.normalize_lut()
    out = {}
    for dt, tag in ((torch.float32, "f32"), (torch.float64, "f64")):
        torch.manual_seed(0)
        model = vgg11_bn()
        if dt == torch.float32:
            theta0 = torch.cat([p.detach().reshape(-1) for p in model.parameters()]).numpy()
            out["theta0_sha"] = np.frombuffer(bytes.fromhex(_sha(theta0)), np.uint8)
        else:
            model = model.double()
        model.train()
        idx = O.batch_indices(0, 0, 0, 0, 4, lists)
        x = torch.from_numpy(lut[imgs[idx]]).to(dt)
        y = torch.from_numpy(labels[idx])
        real = F.dropout
        calls = [0]

        def spec(input, p=0.5, training=True, inplace=False):
            site = O.SITE_VGG_DROPOUT[calls[0]]
            calls[0] += 1
            keep = O.dropout_keep(0, 0, 0, site, p, input.numel())
            return input * torch.from_numpy(keep).reshape(input.shape).to(input.dtype).div_(1 - p)

        torch.nn.functional.dropout = spec
        try:
            w = Worker(torch.nn.CrossEntropyLoss())
            w.model = model
            grads, lossval = w.fwd_bkwd(x, y)
        finally:
            torch.nn.functional.dropout = real
        assert calls[0] == 2
        out[f"{tag}_loss"] = np.asarray(lossval, np.float64)
        out[f"{tag}_stats"], out[f"{tag}_samp"] = tensor_stats(grads)
        out[f"{tag}_running"], _ = _bn_buffers(model)
    keep = {}
    theta0, losses, agg_log, theta_log = train_run(3, 2, True, 3, pool=pool, model_fn=vgg11_bn,
                                                   sites=O.SITE_VGG_DROPOUT, keep=keep)
    model = keep["model"]
    out["train_losses"] = losses
    for t, th in enumerate(theta_log):
        out[f"train_theta{t}_stats"] = th[0]
    out["train_theta_stats"], out["train_theta_samp"] = tensor_stats(list(model.parameters()))
    out["train_running"], out["train_nbt"] = _bn_buffers(model)
    timgs, _ = O.make_test_pool(0)
    model.eval()
    with torch.no_grad():
        out["eval_logits"] = model(torch.from_numpy(lut[timgs[:64]])).double().numpy()
    np.savez_compressed(os.path.join(HERE, "vgg_bn.npz"), **out)
    print("vgg_bn fixtures: loss", out["f32_loss"], out["f64_loss"], "train", losses,
          "nbt", out["train_nbt"])


def main():
    what = sys.argv[1:] or ["schedule", "cascade", "adam", "train", "grad", "vgg", "vgg_bn"]
    pool = None
    if "train" in what or "grad" in what or "vgg" in what or "vgg_bn" in what:
        pool = O.make_pool(0)
    if "schedule" in what:
        make_schedule_fixtures()
    if "cascade" in what:
        make_cascade_fixtures()
    if "adam" in what:
        make_adam_fixtures()
    if "grad" in what:
        make_grad_fixture(pool)
    if "train" in what:
        make_train_fixtures(pool)
    if "vgg" in what:
        make_vgg_fixtures(pool)
    if "vgg_bn" in what:
        make_vgg_bn_fixtures(pool)
    meta = dict(torch=torch.__version__, threads=torch.get_num_threads(),
                cpu_capability=torch.backends.cpu.get_cpu_capability(),
                numpy=np.__version__, pool_sha=_sha(pool[0]) if pool is not None else None,
                sample_per_tensor=SAMPLE_PER_TENSOR)
    mp = os.path.join(HERE, "meta.json")
    old = json.load(open(mp)) if os.path.exists(mp) else {}
    old.update({k: v for k, v in meta.items() if v is not None})
    json.dump(old, open(mp, "w"), indent=1)


if __name__ == "__main__":
    main()
