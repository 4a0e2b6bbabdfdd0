"""CPU-only checks of the product library: it loads, exports every symbol include/flsim.h
declares, and its host-side schedule (C-ABI) is bit-exact with traces of the reference's loop."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import REPO

HEADER = os.path.join(REPO, "include", "flsim.h")


def _declared():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"\b(flsim_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    from flsim import _lib
    L = _lib.lib()
    names = _declared()
    assert len(names) >= 13
    for n in names:
        assert hasattr(L, n), n
    assert set(names) == set(_lib.EXPORTS)
    assert L.flsim_pn1_param_count() == 5596090
    assert L.flsim_vgg11_param_count() == 9750922          # models.py:101-103 vgg11()


def test_workspace_sizes():
    from flsim import _lib
    L = _lib.lib()
    assert L.flsim_pn1_workspace_bytes(4096) > 4096 * 1_500_000
    assert L.flsim_pn1_gradstate_bytes() > 0
    assert L.flsim_vgg11_workspace_bytes(4096) > 4096 * 600_000
    assert L.flsim_vgg11_gradstate_bytes() > 4 * 9750922


def test_engine_layouts_match_models():
    """The engines' flat layouts are the models' named_parameters order (FL/models.py, the
    reference's parameter sets) and the C-ABI's parameter counts."""
    import torch
    from FL.models import PerformantNet1, vgg11
    from flsim import _lib
    from flsim.engine import PN1Engine, VGG11Engine, engine_for_parameters
    for cls, ctor in ((PN1Engine, PerformantNet1), (VGG11Engine, vgg11)):
        m = ctor()
        assert [(n, tuple(p.shape)) for n, p in m.named_parameters()] == \
            [(n, tuple(s)) for n, s in cls.SHAPES]
        assert engine_for_parameters(n for n, _ in m.named_parameters()) is cls
        assert getattr(_lib.lib(), f"flsim_{cls.PREFIX}_param_count")() == \
            sum(p.numel() for p in m.parameters())
    with pytest.raises(NotImplementedError):
        engine_for_parameters(["fc.weight"])
    off = ctypes.c_long()
    assert _lib.lib().flsim_vgg11_workspace_offset(99, 128, ctypes.byref(off)) == 1


def _parse(key):
    n, d, thr, ep = re.match(r"n(\d+)_d(\d+)_thr(\d)_e(\d+)", key).groups()
    return int(n), int(d), int(thr), int(ep)


def test_schedule_abi_matches_reference_traces(golden):
    from flsim.schedule import Schedule, reference_delays
    g = golden.schedule
    keys = sorted({re.match(r"(n\d+_d\d+_thr\d_e\d+)_", k).group(1) for k in g.files})
    for key in keys:
        n, d, thr, ep = _parse(key)      # every epoch the golden trace holds (n = 1024: 600,
                                         # through the d = 500 tick and the epoch after it)
        s = Schedule(n, reference_delays(n, d), thr)
        comp = np.zeros((ep, n), np.uint8)
        c_t = np.zeros(ep, np.int32)
        stale = np.full(ep, -1, np.int64)
        for t in range(ep):
            p = s.next_epoch()
            comp[t] = p.computes
            c_t[t] = p.c_t
            if p.stale:
                assert len(p.stale) == 1 and p.stale[0][0] == n - 1
                stale[t] = p.stale[0][1]
            assert np.array_equal(p.fast, p.computes * (np.arange(n) != n - 1))
        ref = np.unpackbits(g[key + "_computes"], axis=1)[:ep, :n]
        assert np.array_equal(comp, ref), key
        assert np.array_equal(c_t, g[key + "_c_t"][:ep]), key
        assert np.array_equal(stale, g[key + "_stale"][:ep]), key


def test_schedule_heterogeneous_matches_oracle():
    """Config-4 extension: several slow workers with their own delays."""
    from flsim.schedule import Schedule
    from oracle import oracle as O
    rs = np.random.RandomState(3)
    n = 64
    delays = np.where(rs.rand(n) < 0.3, rs.geometric(0.05, n), 0).astype(np.int32)
    ep = 200
    for thr in (0, 1):
        ref = O.schedule(n, delays, thr, ep)
        s = Schedule(n, delays, thr)
        for t in range(ep):
            p = s.next_epoch()
            assert np.array_equal(p.computes, ref.computes[t])
            assert p.c_t == ref.c_t[t] and p.s_t == ref.s_t[t]
            srcs = [src for (_, src) in p.stale]
            assert srcs == [int(x) for x in ref.stale_src[t][ref.stale_src[t] >= 0]]


def test_schedule_empty_epoch_raises_like_rule():
    from flsim.schedule import Schedule
    # n=1: the only worker is the slow one; at t=1 (not a tick for d=5) weight_ups is empty ->
    # the reference raises IndexError in rule() (main.py:25)
    s = Schedule(1, np.array([5], np.int32), False)
    with pytest.raises(IndexError):
        s.next_epoch()      # t=0: slow worker computes and pushes, nothing appended


def test_comm_abi_one_rank_local():
    """flsim_comm_* / flsim_allreduce_sum through the C-ABI: the one-rank local
    communicator (no unique id, never touches RCCL) reduces in place to the identity; bad ranks,
    a multi-rank communicator without a unique id and a null communicator are refused like the
    other entry points (status 1 + flsim_last_error)."""
    import ctypes

    import torch
    from flsim import _lib
    from flsim.comm import Comm
    L = _lib.lib()
    c = Comm()
    assert (c.size, c.rank) == (1, 0)
    buf = torch.arange(7, dtype=torch.float32)
    ref = buf.clone()
    c.all_reduce_sum(buf)
    assert torch.equal(buf, ref)
    c.all_reduce_sum(torch.zeros(0))              # empty buffer: nothing to do
    c.close()
    h = ctypes.c_void_p()
    for nranks, rank in ((1, 1), (0, 0), (2, -1), (2, 0)):   # (2, 0): no unique id
        assert L.flsim_comm_create(nranks, rank, None, ctypes.byref(h)) == 1
        assert not h.value
        assert L.flsim_last_error()
    assert L.flsim_allreduce_sum(None, None, 4, None) == 1
    assert b"null communicator" in L.flsim_last_error()
    assert L.flsim_comm_destroy(None) == 0
    with pytest.raises(ValueError):
        Comm(2, 0, b"short")


@pytest.mark.parametrize("macro", ["FLSIM_X6_FRESH=5", "FLSIM_WGRAD_X6=1", "FLSIM_X6_FLUSH=16",
                                   "FLSIM_ZL1F=4", "FLSIM_DG_FMS=1"])
def test_measurement_overrides_need_a_lab_build(macro, tmp_path):
    """csrc/common.h: a -DFLSIM_<X> measurement override compiles only with -DFLSIM_LAB (make
    LAB=1), so the product library cannot be built off its measured defaults by accident."""
    import shutil
    import subprocess
    cxx = shutil.which("g++") or shutil.which("c++")
    if cxx is None:
        pytest.skip("no host C++ compiler")
    src = tmp_path / "t.cpp"
    # common.h's own preprocessor check, with the HIP runtime header replaced by an empty one
    (tmp_path / "hip").mkdir()
    (tmp_path / "hip" / "hip_runtime.h").write_text("")
    src.write_text('#include "common.h"\nint main() { return 0; }\n')
    inc = ["-I", str(tmp_path), "-I", os.path.join(REPO, "fl-distributed-delay_amd", "csrc")]
    cmd = [cxx, "-std=c++17", "-E", "-D" + macro] + inc + [str(src)]
    bad = subprocess.run(cmd, capture_output=True, text=True)
    assert bad.returncode != 0 and "need a lab build" in bad.stderr, bad.stderr[-400:]
    ok = subprocess.run(cmd + ["-DFLSIM_LAB"], capture_output=True, text=True)
    assert ok.returncode == 0, ok.stderr[-400:]
