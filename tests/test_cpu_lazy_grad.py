"""CPU: the FL.agents facade's lazy .grad views (FL/agents.py _LazyGrad).

fwd_bkwd leaves a worker's gradient in the engine's split-K slabs and returns views whose first
use by any torch function reduces the slabs into the flat buffer (agents.py:35's accumulated
.grad).  Without a GPU the reduction is a stand-in counter: these tests pin which operations
trigger it (everything that reads or writes values) and which do not (shape / dtype / storage
metadata, which Central.update_model itself inspects to find the stale entries).
"""
import numpy as np
import torch


class _Ctx:
    def __init__(self):
        self.flushes = 0
        self.touched = False

    def flush(self, touched=False):
        self.flushes += 1
        self.touched = self.touched or touched


def _views():
    from FL.agents import _lazy_views
    ctx = _Ctx()
    G = torch.arange(10, dtype=torch.float32)
    return ctx, G, _lazy_views(G, [("w", (2, 3)), ("b", (4,))], ctx)


def test_metadata_reads_do_not_reduce():
    ctx, G, (w, b) = _views()
    assert w.shape == (2, 3) and b.dtype == torch.float32 and w.device.type == "cpu"
    assert w.untyped_storage().data_ptr() == G.untyped_storage().data_ptr()
    assert (b.data_ptr() - G.data_ptr()) // 4 == 6
    assert w.dim() == 2 and w.numel() == 6 and w.stride() == (3, 1)
    assert ctx.flushes == 0 and not ctx.touched


def test_value_reads_and_writes_reduce_first():
    ctx, G, (w, b) = _views()
    assert float(w.sum()) == 15.0 and ctx.flushes == 1 and ctx.touched
    out = torch.stack([b, b])                       # main.py:25's rule over plain tensors
    assert type(out) is torch.Tensor and ctx.flushes == 2
    assert np.array_equal(b.cpu().numpy(), [6, 7, 8, 9])
    b.zero_()                                        # an in-place write lands in the buffer
    assert float(G[6:].abs().sum()) == 0.0
    assert repr(w).startswith("tensor(")


def test_views_alias_the_buffer_and_assign_as_grad():
    ctx, G, (w, b) = _views()
    p = torch.nn.Parameter(torch.zeros(2, 3))
    p.grad = w                                       # agents.py:35 .grad aliasing
    assert p.grad is w
    G[0] = 42.0
    assert float(p.grad[0, 0]) == 42.0


def test_data_and_base_reduce_and_stay_lazy():
    """p.grad.data / p.grad._base hand out another tensor over G: they reduce first, and what they
    return reduces again on its own later reads (they used to be metadata, so the
    common .grad.data idiom read a stale partial sum)."""
    ctx, G, (w, b) = _views()
    d = w.data
    assert ctx.flushes == 1 and ctx.touched
    assert float(d.sum()) == 15.0 and ctx.flushes == 2      # a later read through .data reduces
    base = b._base                       # None for these views (made by _make_subclass)
    assert ctx.flushes == 3
    if base is not None:
        assert base.untyped_storage().data_ptr() == G.untyped_storage().data_ptr()
        assert float(base.sum()) == 45.0 and ctx.flushes == 4
