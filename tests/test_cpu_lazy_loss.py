"""CPU: the facade's lazy loss (FL/agents.py _LazyLoss) reads as the reference's loss value,
agents.py:40's `lossval.detach().cpu().numpy()` -- a 0-d float32 ndarray -- wherever main.py and
user code use it (np.mean over the epoch's list, main.py:181; float(); printing; arithmetic), and
its block's value is fetched once, on the first read of any loss in it.  A stand-in block replaces
the engine (no GPU here)."""
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "fl-distributed-delay_amd"))

from FL.agents import _LazyLoss  # noqa: E402


class StandInBlock:
    def __init__(self, values):
        self.values = np.asarray(values, np.float32)
        self.fetches = 0
        self.host = None

    def value(self, g):
        if self.host is None:
            self.fetches += 1
            self.host = self.values.copy()
        return self.host[g]


def test_lazy_loss_reads_like_a_float32_array():
    vals = [2.3025851, 2.2871, 1.75, 0.5]
    blk = StandInBlock(vals)
    lazy = [_LazyLoss(blk, g) for g in range(len(vals))]
    ref = [np.asarray(np.float32(v)) for v in vals]
    assert blk.fetches == 0                      # nothing read yet
    m, mr = np.mean(lazy), np.mean(ref)
    assert blk.fetches == 1                      # one fetch for the whole block
    assert type(m) is type(mr) and m.dtype == np.float32 and m == mr
    a = lazy[0]
    assert float(a) == float(ref[0]) and str(a) == str(ref[0]) and repr(a) == repr(ref[0])
    assert f"{a:.5f}" == f"{ref[0]:.5f}"
    assert a.shape == () and a.dtype == np.float32 and a.ndim == 0 and a.item() == ref[0].item()
    assert np.asarray(a).dtype == np.float32 and np.array(a, np.float64).dtype == np.float64
    assert a + 1 == ref[0] + 1 and 1 - a == 1 - ref[0] and a * 2 == ref[0] * 2
    assert (a / lazy[1]) == (ref[0] / ref[1]) and -a == -ref[0]
    assert a > lazy[2] and lazy[3] < 1 and a == ref[0]
    assert np.exp(a) == np.exp(ref[0]) and np.float32(1) + a == np.float32(1) + ref[0]
    assert bool(a) and int(lazy[2]) == 1
    assert np.isfinite(np.sum(lazy))
    with pytest.raises(TypeError):
        hash(a)                                  # as ndarray


def test_lazy_loss_pickles_as_its_value():
    import pickle
    blk = StandInBlock([1.25])
    b = pickle.loads(pickle.dumps(_LazyLoss(blk, 0)))
    assert isinstance(b, np.ndarray) and b.dtype == np.float32 and b == np.float32(1.25)
