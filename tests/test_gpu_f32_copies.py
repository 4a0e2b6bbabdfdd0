"""The fp32 copies of the weight gradients' layer inputs (split.h xs_store_f).

The forward writes a1, d1, a3, d2 and a5 in the split-bf16 form for the split-bf16 forward GEMMs,
and, in the same epilogue store, each value as plain fp32 at the same element offset for the fp32
weight gradients of conv2-6 (BufSrc / BufSrcSM loaders: no L loads, no (h + m) + l recombination).
The copy must be exactly the value the split form holds: (h + m) + l is exact (split.h), so the two
are compared bit for bit, over a chunk with dropout on and one with it off.
"""
import pytest
import torch

from conftest import has_gpu

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not has_gpu(), reason="needs an MI355X")]

DEV = "cuda:0"
# (split tensor id, fp32 copy id, NHWC shape[1:]) -- flsim_pn1_workspace_offset's ids
PAIRS = {"a1": (1, 31, (34, 34, 48)), "d1": (3, 32, (18, 18, 48)), "a3": (4, 33, (20, 20, 96)),
         "d2": (6, 34, (11, 11, 96)), "a5": (7, 35, (13, 13, 192))}


@pytest.mark.parametrize("dropout", [True, False])
def test_fp32_copies_equal_the_split_form(dropout):
    import numpy as np
    from flsim.data import DevicePool
    from flsim.engine import PN1Engine, worker_table
    from flsim.sim import default_theta
    from oracle import oracle as O
    eng = PN1Engine(DEV, chunk_workers=2)
    dpool = DevicePool(DEV, 0, O.make_pool(0))
    theta = default_theta(0, "PerformantNet1").to(DEV)
    eng.begin_epoch(theta)
    loss = torch.zeros(2, device=DEV)
    eng.run_chunk(theta, dpool, worker_table([(3, 0, 5), (3, 2, 1023)], DEV), 2, 1024, 0,
                  dropout, loss)
    torch.cuda.synchronize()
    assert torch.isfinite(loss).all()
    n = 256
    for name, (hm_id, f_id, shape) in PAIRS.items():
        full = (eng.max_samples,) + shape
        split_vals = eng.workspace_view(hm_id, full)[:n]
        raw = eng._workspace_bytes_at(f_id, int(np.prod(full)) * 4).view(torch.float32)
        if eng.slice_major(hm_id):
            h, w, c = shape
            copy = raw.view(eng.max_samples, c // 16, h, w, 16).permute(0, 2, 3, 1, 4)
            copy = copy.reshape(full)[:n]
        else:
            copy = raw.view(full)[:n]
        assert (split_vals > 0).any(), name
        assert torch.equal(copy, split_vals), (name, int((copy != split_vals).sum()))
