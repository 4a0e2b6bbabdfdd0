"""The oracle (CPU restatement) against golden vectors produced by the reference itself.

tests/golden/make_golden.py ran the reference's own main.py loop / rule() / Central.update_model /
Worker.fwd_bkwd in the build container; these tests pin oracle/ to those outputs.
"""
import hashlib
import json
import os
import re

import numpy as np
import pytest
import torch

from oracle import oracle as O
from oracle import model_ref as MR

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).digest()


def _schedule_keys(g):
    return sorted({re.match(r"(n\d+_d\d+_thr\d_e\d+)_", k).group(1) for k in g.files})


def _parse(key):
    n, d, thr, ep = re.match(r"n(\d+)_d(\d+)_thr(\d)_e(\d+)", key).groups()
    return int(n), int(d), int(thr), int(ep)


def test_schedule_bit_exact(golden):
    g = golden.schedule
    keys = _schedule_keys(g)
    assert len(keys) == 40
    for key in keys:
        n, d, thr, ep = _parse(key)
        s = O.schedule(n, O.reference_delays(n, d), thr, ep)
        assert s.rc == 0
        assert np.array_equal(np.packbits(s.computes, axis=1), g[key + "_computes"]), key
        assert np.array_equal(s.c_t, g[key + "_c_t"]), key
        stale = s.stale_src[:, n - 1]
        assert np.array_equal(stale, g[key + "_stale"]), key
        assert np.array_equal(s.s_t, (g[key + "_stale"] >= 0).astype(np.int32)), key
        fw, fg = g[key + "_final"]
        assert s.window_end[-1] == fw and s.gone_end[-1] == fg, key


def test_worker_k_sequence(golden):
    g = golden.schedule
    for key in _schedule_keys(g):
        n, _, _, ep = _parse(key)
        ks = O.worker_k_sequence(0, n, ep)
        assert np.array_equal(ks[:3], g[key + "_k_head"]), key
        assert _sha(ks.astype(np.int64)) == g[key + "_k_sha"].tobytes(), key


def test_cascade_mean_bit_exact(golden):
    g = golden.cascade
    n = 0
    for key in g.files:
        kind, k, P = key.split("_")
        k, P = int(k[1:]), int(P[1:])
        rs = np.random.RandomState(1000 * k + P)
        S = rs.standard_normal(P).astype(np.float32)
        st = rs.standard_normal(P).astype(np.float32)
        if kind == "rep":
            out = O.cascade_mean([S] * (k - 1) + [st])
        else:
            ent = rs.standard_normal((k, P)).astype(np.float32)
            out = O.cascade_mean(list(ent))
        assert np.array_equal(out.view(np.uint32), g[key].view(np.uint32)), key
        n += 1
    assert n >= 90


def test_adam_teacher_forced(golden):
    """m, v bit-exact; p within 1 ulp of the update on <0.5% of elements (torch CPU sqrt is
    MKL-VML, not correctly rounded; the oracle's sqrt is, like the GPU kernel's)."""
    g = golden.adam
    for j in range(3):
        p = g[f"p0_{j}"].copy()
        m = np.zeros_like(p)
        v = np.zeros_like(p)
        for step in range(1, 11):
            if step > 1:
                p = g[f"p{step - 1}_{j}"].copy()
                m = g[f"m{step - 1}_{j}"].copy()
                v = g[f"v{step - 1}_{j}"].copy()
            p0 = p.copy()
            O.adam_step(p, m, v, g[f"g{step}_{j}"].copy(), step)
            assert np.array_equal(m.view(np.uint32), g[f"m{step}_{j}"].view(np.uint32))
            assert np.array_equal(v.view(np.uint32), g[f"v{step}_{j}"].view(np.uint32))
            ref = g[f"p{step}_{j}"]
            diff = p != ref
            assert diff.mean() <= 0.005
            upd = np.abs(ref.astype(np.float64) - p0)
            assert np.all(np.abs(p.astype(np.float64) - ref)[diff] <=
                          np.spacing(np.abs(ref[diff])) + 2 ** -22 * upd[diff] + 1e-12)


def test_pool_and_data_spec():
    meta = json.load(open(os.path.join(GOLDEN, "meta.json")))
    imgs, labels = O.make_pool(0)
    assert hashlib.sha256(imgs.tobytes()).hexdigest() == meta["pool_sha"]
    a, b = O.class_lists(labels)
    assert len(a) == 40000 and len(b) == 10000
    assert set(labels[b]) == {1, 9}


def _stats_close(st, ref, rtol, atol=0.0):
    # [sum, sumsq, min, max]
    return np.allclose(st, ref, rtol=rtol, atol=atol)


def test_single_worker_grad(golden):
    g = golden.grad
    imgs, labels = O.make_pool(0)
    lists = O.class_lists(labels)
    sim = MR.OracleSim(4, delay=2, pool=(imgs, labels))
    x, y = sim.batch(0, 0, 0)
    assert _sha(x.numpy()) == g["f32_x_sha"].tobytes()
    grad, losses = sim.grad_of(sim.theta, [(0, 0, 0)])
    assert abs(losses[0] - float(g["f32_loss"])) < 1e-6
    off = 0
    samp = []
    for (_, shp) in MR._shapes():
        n = int(np.prod(shp))
        a = grad[off:off + n].astype(np.float64)
        off += n
        rs = np.random.RandomState(123 + n)
        idx = np.arange(n) if n <= 256 else np.sort(rs.choice(n, 256, replace=False))
        samp.append(a[idx])
    samp = np.concatenate(samp)
    np.testing.assert_allclose(samp, g["f32_samp"], rtol=1e-4, atol=1e-7)


@pytest.mark.slow
@pytest.mark.parametrize("thr", [0, 1])
def test_training_trajectory(golden, thr):
    g = golden.train
    key = f"n4_d2_thr{thr}_f32"
    imgs, labels = O.make_pool(0)
    sim = MR.OracleSim(4, delay=2, throttle=bool(thr), pool=(imgs, labels))
    assert _sha(sim.theta) == g[key + "_theta0_sha"].tobytes()
    ref_losses = g[key + "_losses"]
    for t in range(len(ref_losses)):
        loss = sim.epoch()
        # the first two epochs agree to the last bits; later ones drift with the host CPU's fp32
        # kernels (Adam turns 1-ulp gradient differences into O(lr) moves).  Measured on
        # the build host against the golden f32 losses: thr0 4.8e-7 / 2.6e-5 / 1.2e-4 at epochs
        # 2 / 3 / 4, thr1 0 throughout (the golden f32 run itself is 6.1e-7 / 1.5e-6 / 6.8e-5
        # from the golden f64 one); bounds 8-20x those
        tol = (1e-6, 1e-6, 1e-5, 2e-4, 1e-3)[min(t, 4)]
        assert abs(loss - ref_losses[t]) <= tol, (t, loss, ref_losses[t])
        n_entries, n_distinct = g[f"{key}_comp{t}"]
        assert len(sim.trace[-1]["appended"]) == n_entries
        ts = []
        off = 0
        for (_, shp) in MR._shapes():
            n = int(np.prod(shp))
            a = sim.theta[off:off + n].astype(np.float64)
            off += n
            ts.append([a.sum(), (a * a).sum(), a.min(), a.max()])
        np.testing.assert_allclose(np.asarray(ts)[:, 1], g[f"{key}_theta{t}_stats"][:, 1],
                                   rtol=1e-3)  # Adam amplifies 1-ulp sqrt diffs


def _sampled(grad, model):
    """The golden sampling of make_golden.tensor_stats: <= 256 fixed indices per tensor."""
    off, samp = 0, []
    for (_, shp) in MR._shapes(model):
        n = int(np.prod(shp))
        a = grad[off:off + n].astype(np.float64)
        off += n
        rs = np.random.RandomState(123 + n)
        idx = np.arange(n) if n <= 256 else np.sort(rs.choice(n, 256, replace=False))
        samp.append(a[idx])
    return np.concatenate(samp)


def test_vgg11_oracle_matches_reference(golden):
    """configs[4]: the oracle's VGG11Ref / vgg_forward against the reference's own vgg11()
    (models.py:50-103): identical init under torch.manual_seed(0), one worker-step gradient
    through Worker.fwd_bkwd with the spec's classifier dropout masks (f32 and f64 runs)."""
    g = golden.vgg
    imgs, labels = O.make_pool(0)
    sim = MR.OracleSim(4, delay=2, pool=(imgs, labels), model="vgg11")
    assert _sha(sim.theta) == g["theta0_sha"].tobytes()
    assert sim.theta.size == 9750922
    grad, losses = sim.grad_of(sim.theta, [(0, 0, 0)])
    assert abs(losses[0] - float(g["f32_loss"])) < 1e-6
    np.testing.assert_allclose(_sampled(grad, "vgg11"), g["f32_samp"], rtol=1e-4, atol=1e-7)
    g64, l64 = sim.grad_of(sim.theta, [(0, 0, 0)], dtype=torch.float64)
    assert abs(l64[0] - float(g["f64_loss"])) < 1e-12
    np.testing.assert_allclose(_sampled(g64, "vgg11"), g["f64_samp"], rtol=1e-9, atol=1e-13)


def test_vgg11_oracle_trajectory(golden):
    """3 epochs of the reference's verbatim loop with vgg11 (n=3, d=2, throttle): same losses."""
    g = golden.vgg
    imgs, labels = O.make_pool(0)
    sim = MR.OracleSim(3, delay=2, throttle=True, pool=(imgs, labels), model="vgg11")
    for t, ref in enumerate(g["train_losses"]):
        loss = sim.epoch()
        # host-CPU fp32 drift after the first Adam steps (the fixture was made on a Xeon host):
        # exact at epoch 0, <= 2.4e-7 at epoch 1, 5.94e-5 at epoch 2 measured on both EPYC hosts
        # this test runs on (this container and the GPU box, profiles/r06/r06f/cpu_drift.txt);
        # bound 1.5 x that
        print("MEASURED", json.dumps(dict(test="vgg11_oracle_trajectory", epoch=t,
                                          loss_drift=abs(loss - float(ref)))))
        assert abs(loss - ref) <= (1e-5 if t < 2 else 9e-5), (t, loss, ref)
        np.testing.assert_allclose(
            [float((a.astype(np.float64) ** 2).sum()) for a in MR.split_flat(sim.theta, "vgg11")],
            g[f"train_theta{t}_stats"][:, 1], rtol=1e-3)


def test_vgg11_bn_oracle_matches_reference(golden):
    """vgg11_bn (models.py:106-108): the oracle's VGG11BNRef / vgg_bn_forward against the
    reference's own module -- identical init, one worker-step gradient through Worker.fwd_bkwd in
    train mode (batch statistics of the worker's 128 samples), and the BatchNorm running buffers
    that call leaves behind (momentum 0.1, unbiased variance)."""
    g = golden.vgg_bn
    imgs, labels = O.make_pool(0)
    sim = MR.OracleSim(4, delay=2, pool=(imgs, labels), model="vgg11_bn")
    assert _sha(sim.theta) == g["theta0_sha"].tobytes()
    assert sim.theta.size == 9756426
    grad, losses = sim.grad_of(sim.theta, [(0, 0, 0)])
    assert abs(losses[0] - float(g["f32_loss"])) < 1e-6
    assert sim.bn.num_batches_tracked == 1
    np.testing.assert_allclose(sim.bn.flat(), g["f32_running"], rtol=1e-5, atol=1e-7)
    # conv biases before a BatchNorm get a gradient that is zero up to rounding: compare with
    # an absolute tolerance at the scale of that rounding noise (1.4e-7 on an EPYC build host
    # whose oneDNN paths differ from the golden generator's)
    np.testing.assert_allclose(_sampled(grad, "vgg11_bn"), g["f32_samp"], rtol=1e-3, atol=5e-7)
    bn64 = MR.BNState(torch.float64)
    g64, l64 = sim.grad_of(sim.theta, [(0, 0, 0)], dtype=torch.float64, bn=bn64)
    assert abs(l64[0] - float(g["f64_loss"])) < 1e-12
    np.testing.assert_allclose(_sampled(g64, "vgg11_bn"), g["f64_samp"], rtol=1e-9, atol=1e-13)
    np.testing.assert_allclose(bn64.flat(), g["f64_running"], rtol=1e-12, atol=1e-15)


def _check_running(got, ref, rm_atol=2e-4, rv_rtol=1e-5):
    """running_var within rv_rtol; running_mean within rm_atol absolute.  A conv bias in front of
    a BatchNorm cancels in the normalisation, so its gradient is rounding noise of a zero sum;
    Adam turns that noise into +-lr steps, and the bias enters running_mean directly.  After a
    few epochs two correct implementations differ there by O(lr * epochs * momentum)."""
    off = 0
    for c in MR.VGG_BN_CHANNELS:
        np.testing.assert_allclose(got[off:off + c], ref[off:off + c], rtol=0, atol=rm_atol)
        np.testing.assert_allclose(got[off + c:off + 2 * c], ref[off + c:off + 2 * c],
                                   rtol=rv_rtol, atol=1e-7)
        off += 2 * c


def test_vgg11_bn_oracle_trajectory_and_eval(golden):
    """3 epochs of the reference's verbatim loop with vgg11_bn (n=3, d=2, throttle): losses,
    parameter norms, the running buffers after every computing worker's forward (in worker
    order), num_batches_tracked, and the eval-mode logits of the final model (util.py:31-45)."""
    g = golden.vgg_bn
    imgs, labels = O.make_pool(0)
    sim = MR.OracleSim(3, delay=2, throttle=True, pool=(imgs, labels), model="vgg11_bn")
    for t, ref in enumerate(g["train_losses"]):
        loss = sim.epoch()
        # host-CPU fp32 drift after the first Adam steps: exact at epochs 0-1, 2.09e-5 at epoch 2
        # on both EPYC hosts this test runs on (2.1e-5 on the Xeon host that made the fixture,
        # profiles/r06/r06f/cpu_drift.txt); bound 1.5 x that
        print("MEASURED", json.dumps(dict(test="vgg11_bn_oracle_trajectory", epoch=t,
                                          loss_drift=abs(loss - float(ref)))))
        assert abs(loss - ref) <= (1e-5 if t < 2 else 3.2e-5), (t, loss, ref)
        np.testing.assert_allclose(
            [float((a.astype(np.float64) ** 2).sum())
             for a in MR.split_flat(sim.theta, "vgg11_bn")][2::4],     # BatchNorm weights
            g[f"train_theta{t}_stats"][2::4, 1], rtol=1e-4)
    assert sim.bn.num_batches_tracked == int(g["train_nbt"][0])
    # running_mean: the pre-BatchNorm conv biases' Adam steps of +-lr on rounding noise enter it
    # directly, so two hosts differ by up to lr * epochs (8e-4 and 1.6e-3 seen on EPYC build
    # hosts); running_var within 1e-2 (2.7e-3 seen there in the 512-channel layers)
    _check_running(sim.bn.flat(), g["train_running"], rm_atol=3e-3, rv_rtol=1e-2)
    timgs, _ = O.make_test_pool(0)
    params = [torch.from_numpy(a) for a in MR.split_flat(sim.theta, "vgg11_bn")]
    sim.bn.training = False
    with torch.no_grad():
        logits = MR.vgg_bn_forward(params, torch.from_numpy(O.normalize_lut()[timgs[:64]]), None,
                                   sim.bn)
    # the same 3-epoch host drift reaches the logits (9e-4 absolute on the EPYC build host); the
    # tight pin of the forward is the one-step test above
    np.testing.assert_allclose(logits.double().numpy(), g["eval_logits"], rtol=1e-3, atol=3e-3)


def test_warm_start_fixture_is_pinned():
    """configs[1]'s warm start (tests/golden/make_warm_start_n10.py: a short fp64 oracle
    pre-training, int8 per tensor): its dequantised fp32 vector has the pinned sha256 and the
    models.py parameter count; it is not the default init."""
    import hashlib
    import json
    import os
    import sys
    from oracle import model_ref as MR
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    sys.path.insert(0, here)
    from make_warm_start_n10 import dequantise
    w = np.load(os.path.join(here, "warm_n10.npz"))
    theta = dequantise(w["codes"], w["scales"])
    meta = json.load(open(os.path.join(here, "meta.json")))
    assert hashlib.sha256(theta.tobytes()).hexdigest() == meta["warm_n10"]["sha256"]
    assert theta.size == 5596090
    assert np.abs(theta - MR.init_params(2)).max() > 1e-3
