"""CPU oracle for the FL-simulation hot path -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module, and
only as the checker (never as the thing measured or shipped).  The product path lives in
fl-distributed-delay_amd/ and fails loudly when its HIP library is missing.

Contents (reference file:line each function restates):
  * ctypes bindings to flsim_oracle.c (schedule scan main.py:119-181, cascade mean main.py:23-25,
    Adam agents.py:9-21 + main.py:106, Philox draws replacing main.py:85-88 / models.py:17,23)
  * synthetic data spec (replaces CIFAR10 + non-IID split, main.py:28-34,65-91,138-142)
  * PerformantNet1 restated in torch-CPU fp32/fp64 (models.py:11-47), dropout masks injected
  * Worker.fwd_bkwd restated (agents.py:32-40) and the full server step (main.py:126-188)

Pinning: tests/golden/* were produced by running the reference itself in the build container
(tests/golden/make_golden.py); tests/test_oracle_golden.py checks this module against them.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass, field

import numpy as np

ORACLE_DIR = os.path.dirname(os.path.abspath(__file__))
_LIB = None

# --- constants of the build's data / RNG spec (DESIGN.md "RNG spec") -------------------------
SITE_DATA = 0x10                  # sample-slot draws
SITE_DROPOUT = (1, 2, 3, 4, 5)    # dropout1 x3 (models.py:32,36,40), dropout2 x2 (models.py:43,45)
DROPOUT_P = (0.25, 0.25, 0.25, 0.5, 0.5)
SITE_VGG_DROPOUT = (6, 7)         # vgg11 classifier Dropout() x2, p = 0.5 (models.py:58,61)
POOL_SIZE = 50000
CLASSES_A = (0, 2, 3, 4, 5, 6, 7, 8)   # main.py:78 targets[0]
CLASSES_B = (1, 9)                      # main.py:78 targets[1]
BATCH = 128                             # main.py:43-44 default --batch_size


def build():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(ORACLE_DIR, "_build", "liboracle.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        L.oracle_philox.restype = ctypes.c_uint32
        L.oracle_philox.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                    ctypes.c_uint32, ctypes.c_uint32]
        L.oracle_dropout_keep.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                          ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64,
                                          ctypes.c_uint64, ctypes.c_void_p]
        L.oracle_sample_slots.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                          ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                          ctypes.c_void_p]
        L.oracle_schedule_run.restype = ctypes.c_int
        L.oracle_schedule_run.argtypes = [ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32,
                                          ctypes.c_int32, ctypes.c_int64] + [ctypes.c_void_p] * 8
        L.oracle_cascade_mean.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                          ctypes.c_void_p]
        L.oracle_adam_step.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int64, ctypes.c_int64] + \
            [ctypes.c_double] * 4
        _LIB = L
    return _LIB


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


# ---------------------------------------------------------------------------------------------
# RNG spec
# ---------------------------------------------------------------------------------------------
def philox_word(seed, t, worker, site, e):
    return int(lib().oracle_philox(seed, t, worker, site, e))


def dropout_keep(seed, t, worker, site, p, numel):
    thr = int(round(p * 2 ** 32))
    out = np.empty(numel, np.uint8)
    lib().oracle_dropout_keep(seed, t, worker, site, thr, 0, numel, _p(out))
    return out.astype(bool)


def sample_slots(seed, t, worker, length, n=BATCH):
    out = np.empty(n, np.uint32)
    lib().oracle_sample_slots(seed, t, worker, SITE_DATA, length, n, _p(out))
    return out


# ---------------------------------------------------------------------------------------------
# Synthetic data spec: CIFAR-shaped uint8 pool (3x32x32), labels j % 10.
# ---------------------------------------------------------------------------------------------
def make_pool(seed=0, size=POOL_SIZE, noise_seed=None):
    rs = np.random.RandomState(seed)
    proto = rs.randint(0, 256, size=(10, 3, 32, 32)).astype(np.int16)
    labels = (np.arange(size) % 10).astype(np.int64)
    rs2 = np.random.RandomState(seed + 1 if noise_seed is None else noise_seed)
    imgs = np.empty((size, 3, 32, 32), np.uint8)
    step = 5000
    for s in range(0, size, step):
        e = min(size, s + step)
        noise = rs2.randint(-48, 49, size=(e - s, 3, 32, 32)).astype(np.int16)
        imgs[s:e] = np.clip(proto[labels[s:e]] + noise, 0, 255).astype(np.uint8)
    return imgs, labels


def make_test_pool(seed=0, size=10000):
    """Test split spec (replaces main.py:72-73 CIFAR10(train=False)): same prototypes, noise
    stream seed + 2."""
    return make_pool(seed, size, noise_seed=seed + 2)


def class_lists(labels):
    a = np.where(np.isin(labels, CLASSES_A))[0]      # main.py:30 np.where(np.isin(...))
    b = np.where(np.isin(labels, CLASSES_B))[0]
    return a, b


def normalize_lut():
    """ToTensor (u8 / 255) then Normalize(0.5, 0.5) (main.py:65-67), fp32 op by op."""
    u = np.arange(256, dtype=np.float32)
    x = u / np.float32(255.0)
    x = (x - np.float32(0.5)) / np.float32(0.5)
    return x.astype(np.float32)


def worker_k_sequence(seed, n, n_epochs):
    """np.random.randint(0, n) per worker per epoch from the seeded global RNG (main.py:138)."""
    rs = np.random.RandomState(seed)
    return np.stack([rs.randint(0, n, size=n) for _ in range(n_epochs)]) if n_epochs else \
        np.zeros((0, n), np.int64)


def batch_indices(seed, t, worker, k, n, lists, batch=BATCH):
    """main.py:138-142 draw of worker-step (t, worker): `batch` samples with replacement from
    dataset k's class list; slot e from philox(seed, t, worker, SITE_DATA, e) (e < batch: any
    --batch_size, main.py:43-44)."""
    lst = lists[1] if k == n - 1 else lists[0]
    return lst[sample_slots(seed, t, worker, len(lst), batch)]


# ---------------------------------------------------------------------------------------------
# Schedule
# ---------------------------------------------------------------------------------------------
@dataclass
class Schedule:
    computes: np.ndarray
    appended: np.ndarray
    stale_src: np.ndarray
    c_t: np.ndarray
    s_t: np.ndarray
    window_end: np.ndarray
    gone_end: np.ndarray
    rc: int = 0
    fail_epoch: int = -1


def schedule(n, delays, throttle, n_epochs, max_throttle=32):
    delays = np.ascontiguousarray(delays, np.int32)
    assert delays.shape == (n,)
    comp = np.zeros((n_epochs, n), np.uint8)
    app = np.zeros((n_epochs, n), np.uint8)
    src = np.full((n_epochs, n), -1, np.int64)
    c = np.zeros(n_epochs, np.int32)
    s = np.zeros(n_epochs, np.int32)
    w = np.zeros(n_epochs, np.int32)
    g = np.zeros(n_epochs, np.uint8)
    fe = np.array([-1], np.int64)
    rc = lib().oracle_schedule_run(n, _p(delays), int(bool(throttle)), max_throttle, n_epochs,
                                   _p(comp), _p(app), _p(src), _p(c), _p(s), _p(w), _p(g), _p(fe))
    return Schedule(comp, app, src, c, s, w, g, rc, int(fe[0]))


def reference_delays(n, delay):
    d = np.zeros(n, np.int32)
    d[n - 1] = delay
    return d


# ---------------------------------------------------------------------------------------------
# Cascade mean / Adam
# ---------------------------------------------------------------------------------------------
def cascade_mean(entries):
    entries = [np.ascontiguousarray(e, np.float32).ravel() for e in entries]
    k = len(entries)
    P = entries[0].size
    ptrs = (ctypes.c_void_p * k)(*[e.ctypes.data for e in entries])
    out = np.empty(P, np.float32)
    lib().oracle_cascade_mean(ptrs, k, P, _p(out))
    return out


def adam_step(p, m, v, g, step, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8):
    """In place on float32 contiguous arrays; `step` is the post-increment count."""
    for a in (p, m, v, g):
        assert a.dtype == np.float32 and a.flags.c_contiguous
    lib().oracle_adam_step(_p(p), _p(m), _p(v), _p(g), p.size, step, lr, beta1, beta2, eps)


# ---------------------------------------------------------------------------------------------
# Trajectory drift measure (test infrastructure): a Johnson-Lindenstrauss sketch of a flat
# parameter vector.  ||sketch(a) - sketch(b)|| / sqrt(rows) estimates ||a - b|| (within ~20 % at
# 64 rows) without storing a or b; the Gaussian rows come from torch's CPU generator (the same
# numbers on every machine).
# ---------------------------------------------------------------------------------------------
def theta_sketch(theta, rows=64, seed=1234):
    import torch
    th = torch.as_tensor(np.asarray(theta, np.float32)).to(torch.float64)
    out = np.empty(rows, np.float64)
    g = torch.Generator()
    for r in range(rows):
        g.manual_seed(seed + r)
        out[r] = float(torch.dot(torch.randn(th.numel(), generator=g).to(torch.float64), th))
    return out


def sketch_distance(sa, sb):
    return float(np.linalg.norm(np.asarray(sa) - np.asarray(sb)) / np.sqrt(len(sa)))
