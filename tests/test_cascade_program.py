"""CPU checks of rule()'s summation programs (csrc/cascade.h): the host builder + host
interpreter of libflsim.so against the oracle's cascade restatement (oracle/flsim_oracle.c,
pinned to torch 2.10's stack().mean(0) by tests/golden/cascade.npz), bit for bit.

The device kernels (k_agg_stream, k_slab_step) run the same programs with the same fp32 adds,
so a program that is exact here is exact on the GPU (tests/test_gpu_server_step.py)."""
import ctypes

import numpy as np
import pytest

vp = ctypes.c_void_p


def _eval(words, info, S, arrays, tail):
    from flsim import _lib
    n = S.size
    out = np.empty(n, np.float32)
    ys = (vp * max(1, len(arrays)))(*[a.ctypes.data for a in arrays])
    t = tail.astype(np.uint8)
    rc = _lib.lib().flsim_cascade_eval_host(
        words.ctypes.data_as(vp), info.ctypes.data_as(vp), S.ctypes.data_as(vp), ys, len(arrays),
        t.ctypes.data_as(vp), n, out.ctypes.data_as(vp))
    assert rc == 0
    return out


def _values(rs, n):
    v = (rs.standard_normal(n) * 1e-2).astype(np.float32)
    v[::13] = 0.0
    v[1::13] = -0.0
    v[2::13] = np.float32(3e-39)
    v[3::13] = np.float32(1e30)
    v[4::13] = np.float32(-1e30)
    return v


def _check(k, pos, arr, n_arrays, seed):
    from flsim.engine import cascade_program
    from oracle import oracle as O
    rs = np.random.RandomState(seed)
    n = 64 + 7                                 # 64 multi_row_sum columns + 7 row_sum tail columns
    S = _values(rs, n)
    arrays = [_values(rs, n) for _ in range(n_arrays)]
    words, info = cascade_program(k, list(zip(pos, arr)))
    tail = np.arange(n) >= 64
    got = _eval(words, info, S, arrays, tail) / np.float32(k)
    ents = [S] * k
    for p, a in zip(pos, arr):
        ents[p] = arrays[a]
    ref = O.cascade_mean(ents)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), \
        (k, np.nonzero(got.view(np.uint32) != ref.view(np.uint32))[0][:8])
    return words


@pytest.mark.parametrize("k", [1, 2, 3, 4, 5, 15, 16, 17, 31, 255, 256, 257, 513, 1023, 1024,
                               4095, 4096, 4097, 5000, 16383, 70001])
def test_reference_order_programs(k):
    """[S_t] * c + one stale entry (the reference's slow worker), and no stale entry."""
    _check(k, [k - 1], [0], 1, k)
    _check(k, [], [], 0, k + 1)


@pytest.mark.parametrize("k,nev,seed", [(7, 3, 0), (37, 5, 1), (300, 40, 2), (700, 40, 3),
                                        (5000, 3, 4), (8100, 72, 5), (16383, 50, 6),
                                        (12, 12, 7), (4096, 4096 // 64, 8), (70001, 30, 9)])
def test_general_order_programs(k, nev, seed):
    """Heterogeneous-delay extension: stale entries anywhere among the S_t copies, several entries
    sharing an array, every entry stale (k = nev = 12)."""
    rs = np.random.RandomState(seed)
    pos = np.sort(rs.choice(k, nev, replace=False))
    arr = rs.randint(0, 6, nev)
    _check(k, pos.tolist(), arr.tolist(), 6, seed)


def test_program_is_compact():
    """Pure blocks and level groups compress: the reference order at k = 1024 is a handful of
    words, so it fits the kernel arguments (RULE_INL_PROG = 192)."""
    from flsim.engine import cascade_program
    words, info = cascade_program(1024, [(1023, 0)])
    assert 2 * (info[0] + 1) == len(words) and info[0] < 96 - 1   # pairs + the fetch-pad pair
    assert info[3] == 4
    words, info = cascade_program(8100, [(p, p % 6) for p in range(50, 8100, 113)])
    assert info[1] <= 2 * 72           # main part: one or two macro words per stale entry


def test_program_errors():
    from flsim.engine import cascade_program
    with pytest.raises(ValueError):
        cascade_program(10, [(5, 0), (5, 1)])       # positions must increase
    with pytest.raises(ValueError):
        cascade_program(10, [(10, 0)])              # outside [0, k)
    with pytest.raises(ValueError):
        cascade_program(1 << 20, [])                # beyond the lp = 4 range


def test_configs3_schedule_programs():
    """configs[3]'s heterogeneous schedule (16,384 workers): the programs of its first 120 epochs
    are exact, and no epoch needs more distinct arrays than the kernel arguments hold."""
    from flsim._lib import MAX_ARRAYS
    from flsim.engine import cascade_program
    from flsim.schedule import Schedule, heterogeneous_delays
    n = 16384
    s = Schedule(n, heterogeneous_delays(n), True)
    worst = 0
    for t in range(400):
        plan = s.next_epoch()
        if not plan.stale:
            continue
        fast = np.nonzero(plan.fast)[0]
        sw = np.asarray([w for (w, _) in plan.stale])
        pos = np.searchsorted(fast, sw) + np.arange(len(sw))
        srcs = sorted({src for (_, src) in plan.stale})
        arr = [srcs.index(src) for (_, src) in plan.stale]
        worst = max(worst, len(srcs))
        k = plan.c_t + plan.s_t
        if t < 120 and t % 7 == 0:
            _check(k, pos.tolist(), arr, len(srcs), t)
        else:
            cascade_program(k, list(zip(pos.tolist(), arr)))
    assert worst <= MAX_ARRAYS
