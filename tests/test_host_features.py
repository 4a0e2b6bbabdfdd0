"""CPU tests of the host-side features around the hot path: checkpoint / resume (replayed
schedule + numpy k-draws), the CIFAR-10 binary reader (main.py:70-73 data from a local copy), the
test-split spec (independent implementations in flsim.data and the oracle agree)."""
import os

import numpy as np
import pytest
import torch

from test_dist_cpu import P, StandInEngine


def _sim(n, d, thr):
    from flsim.sim import FLSimulation
    return FLSimulation(n, delay=d, throttle=thr, device="cpu", engine=StandInEngine(),
                        device_pool=object(), theta0=torch.zeros(P))


@pytest.mark.parametrize("thr", [False, True])
def test_checkpoint_resume_continues_bit_for_bit(tmp_path, thr):
    n, d, total, cut = 11, 3, 9, 4          # the cut leaves a stale gradient in the FIFO
    ref = _sim(n, d, thr)
    ref_losses = [ref.epoch() for _ in range(total)]
    a = _sim(n, d, thr)
    for _ in range(cut):
        a.epoch()
    path = str(tmp_path / "ck.pt")
    a.save_checkpoint(path)
    assert a.checkpoint()["stale"], "the cut should hold a FIFO entry"
    b = _sim(n, d, thr)
    b.restore(path)                          # torch.load(weights_only=True) inside
    for _ in range(total - cut):
        b.epoch()
    assert np.array_equal(b.theta.numpy().view(np.uint32), ref.theta.numpy().view(np.uint32))
    assert [(p.t, p.computes.tobytes(), p.stale) for p in b.trace] == \
           [(p.t, p.computes.tobytes(), p.stale) for p in ref.trace]
    assert b.losses() == ref_losses


def test_restore_rejects_a_different_run(tmp_path):
    a = _sim(11, 3, False)
    a.epoch()
    ck = a.checkpoint()
    with pytest.raises(ValueError):
        _sim(11, 4, False).restore(ck)
    with pytest.raises(ValueError):
        _sim(12, 3, False).restore(ck)


def test_cifar10_binary_reader(tmp_path):
    from flsim.data import load_cifar10_bin
    rs = np.random.RandomState(0)
    want = {}
    for name, nrec in [(f"data_batch_{i}.bin", 3) for i in range(1, 6)] + [("test_batch.bin", 4)]:
        lab = rs.randint(0, 10, nrec).astype(np.uint8)
        img = rs.randint(0, 256, (nrec, 3072)).astype(np.uint8)
        (tmp_path / name).write_bytes(np.concatenate([lab[:, None], img], 1).tobytes())
        want[name] = (lab, img)
    (tr_x, tr_y), (te_x, te_y) = load_cifar10_bin(str(tmp_path))
    assert tr_x.shape == (15, 3, 32, 32) and tr_x.dtype == np.uint8 and te_x.shape == (4, 3, 32, 32)
    assert np.array_equal(tr_y[:3], want["data_batch_1.bin"][0])
    assert np.array_equal(tr_x[3].reshape(-1), want["data_batch_2.bin"][1][0])
    assert np.array_equal(te_y, want["test_batch.bin"][0])
    (tmp_path / "test_batch.bin").write_bytes(b"\0" * 100)
    with pytest.raises(ValueError):
        load_cifar10_bin(str(tmp_path))


def test_test_split_spec_matches_oracle():
    from flsim.data import make_test_pool
    from oracle import oracle as O
    a, la = make_test_pool(3, size=2000)
    b, lb = O.make_test_pool(3, size=2000)
    assert np.array_equal(a, b) and np.array_equal(la, lb)
    tr, _ = O.make_pool(3, size=2000)
    assert not np.array_equal(a, tr)         # independent noise from the train split
    assert np.bincount(la, minlength=10).tolist() == [200] * 10


@pytest.mark.parametrize("model", ["PerformantNet1", "vgg11_bn"])
def test_model_file_warm_start_loads_state_dict(tmp_path, model):
    """--model_file (main.py:98-100): a torch.save'd models.py state_dict becomes theta0 in
    named_parameters order plus the module buffers; a wrong key set fails like load_state_dict."""
    from FL import models
    from flsim.sim import load_model_file
    torch.manual_seed(3)
    m = getattr(models, model)()
    with torch.no_grad():
        for b in m.buffers():
            if b.is_floating_point():
                b.uniform_(0.5, 1.5)
    path = str(tmp_path / "warm_start.pt")
    torch.save(m.state_dict(), path)
    theta0, bufs = load_model_file(path, model)
    want = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
    assert torch.equal(theta0, want)
    assert set(bufs) == {k for k, _ in m.named_buffers()}
    for k, b in m.named_buffers():
        assert torch.equal(bufs[k], b)
    sd = m.state_dict()
    sd.pop(next(iter(sd)))
    torch.save(sd, path)
    with pytest.raises(RuntimeError):
        load_model_file(path, model)


def test_restore_rejects_other_hyperparameters():
    """lr, betas, eps and max_throttle are part of the checkpoint's config."""
    from flsim.sim import FLSimulation
    a = _sim(11, 3, True)
    a.epoch()
    ck = a.checkpoint()
    for kw in (dict(lr=2e-3), dict(betas=(0.8, 0.999)), dict(eps=1e-7), dict(max_throttle=8)):
        b = FLSimulation(11, delay=3, throttle=True, device="cpu", engine=StandInEngine(),
                         device_pool=object(), theta0=torch.zeros(P), **kw)
        with pytest.raises(ValueError):
            b.restore(ck)


def test_restore_migrates_format_1_checkpoints():
    """A round-1 checkpoint (format 1: no model / optimizer / throttle-cap keys, the --delay 0
    slow worker stored as delay 0) restores into a run with the defaults, with a warning."""
    a = _sim(11, 3, True)
    for _ in range(4):
        a.epoch()
    ck = a.checkpoint()
    assert ck["format"] == "flsim-checkpoint-2"
    old = dict(ck, format="flsim-checkpoint-1")
    old["config"] = {k: v for k, v in ck["config"].items()
                     if k not in ("model", "lr", "betas", "eps", "max_throttle")}
    b = _sim(11, 3, True)
    with pytest.warns(UserWarning, match="format-1"):
        b.restore(old)
    a.epoch()
    b.epoch()
    assert np.array_equal(a.theta.numpy().view(np.uint32), b.theta.numpy().view(np.uint32))
    z = _sim(5, 0, False)
    z.epoch()
    ck0 = z.checkpoint()
    old0 = dict(ck0, format="flsim-checkpoint-1")
    old0["config"] = dict(ck0["config"], delays=torch.zeros(5, dtype=torch.int32))
    _sim(5, 0, False).restore(old0)          # delay 0 maps onto DELAY_ZERO
    with pytest.raises(ValueError):
        _sim(5, 0, False).restore(dict(ck0, format="something-else"))


def test_delay_zero_is_the_reference_slow_worker():
    """--delay 0 (main.py:150-158): worker n-1 is still the slow one -- it computes and pushes
    at t = 0 without an entry or a logged loss -- and t = 1 raises ZeroDivisionError (t % 0)."""
    from flsim.schedule import Schedule, reference_delays
    n = 5
    s = Schedule(n, reference_delays(n, 0), False)
    p = s.next_epoch()
    assert p.computes.tolist() == [1] * n
    assert p.fast.tolist() == [1] * (n - 1) + [0]
    assert p.c_t == n - 1 and p.s_t == 0 and p.pushed
    with pytest.raises(ZeroDivisionError):
        s.next_epoch()
    sim = _sim(n, 0, False)
    sim.epoch()
    with pytest.raises(ZeroDivisionError):
        sim.epoch()


def test_fl_util_drop_in_names():
    """main.py:19 `from FL.util import *` resolves to the package with the reference's names."""
    ns = {}
    exec("from FL.util import *", ns)
    for name in ("save_data", "plot_data", "imshow", "print_test_accuracy", "check_mem"):
        assert callable(ns[name]), name


def test_print_test_accuracy_refuses_train_mode():
    """The device evaluation is eval-mode only (main.py:190 calls model.eval() first)."""
    from FL.models import PerformantNet1
    from FL.util import print_test_accuracy
    m = PerformantNet1()
    m.train()
    with pytest.raises(NotImplementedError):
        print_test_accuracy(m, [])


def test_worker_index_reuse_is_refused():
    """Two Worker objects with one index in one epoch would share dropout keys: refused."""
    from FL.agents import Worker, _ModelContext

    class Ctx:
        users = {}
    claim = _ModelContext.claim
    a, b = Worker(torch.nn.CrossEntropyLoss()), Worker(torch.nn.CrossEntropyLoss())
    b.index = a.index
    ctx = Ctx()
    claim(ctx, a)
    claim(ctx, a)                 # the same worker again is not a reuse
    with pytest.raises(ValueError):
        claim(ctx, b)
