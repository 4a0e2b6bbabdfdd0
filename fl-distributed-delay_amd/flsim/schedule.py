"""Host schedule: ctypes wrapper over flsim_sched_* (the integer scan of main.py:119-181)."""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from ._lib import check, lib


@dataclass
class EpochPlan:
    t: int
    computes: np.ndarray        # u8[n]: worker ran fwd_bkwd (its gradient joins S_t)
    fast: np.ndarray            # u8[n]: fast worker that computed (entry = S_t, loss logged)
    stale: list                 # [(worker, source_epoch)] popped FIFO entries, append order
    c_t: int
    s_t: int
    pushed: bool                # a slow worker stored S_t in its FIFO this epoch


DELAY_ZERO = -(1 << 31)     # FLSIM_DELAY_ZERO: the slow worker under --delay 0


def reference_delays(n, delay):
    """main.py: exactly one slow worker, index n-1, with --delay (main.py:150 tests the index,
    not the delay: under --delay 0 worker n-1 is still the slow one, DELAY_ZERO)."""
    d = np.zeros(n, np.int32)
    d[n - 1] = delay if delay != 0 else DELAY_ZERO
    return d


def heterogeneous_delays(n, seed=0, slow_fraction=0.1, mean_delay=100, dmax=1000):
    """configs[3] / SURVEY 8d C4 spec (the build's): each worker is slow with probability
    slow_fraction; a slow worker's delay is 1 + Geometric(1 / mean_delay) truncated to dmax
    (RandomState(seed + 7)); 0 = fast.  The last worker is always slow, as in main.py."""
    rs = np.random.RandomState(seed + 7)
    slow = rs.rand(n) < slow_fraction
    d = np.minimum(rs.geometric(1.0 / mean_delay, size=n), dmax).astype(np.int32)
    out = np.where(slow, d, 0).astype(np.int32)
    out[n - 1] = max(int(out[n - 1]), int(d[n - 1]))
    return out


class Schedule:
    def __init__(self, n, delays, throttle=False, max_throttle=32):
        self.n = int(n)
        self.delays = np.ascontiguousarray(delays, np.int32)
        if self.delays.shape != (self.n,):
            raise ValueError("delays must have n entries")
        h = lib().flsim_sched_create(self.n, self.delays.ctypes.data_as(ctypes.c_void_p),
                                     int(bool(throttle)), int(max_throttle))
        if not h:
            raise ValueError(lib().flsim_last_error().decode())
        self._h = ctypes.c_void_p(h)
        self._comp = np.zeros(self.n, np.uint8)
        self._fast = np.zeros(self.n, np.uint8)
        self._sw = np.zeros(self.n, np.int32)
        self._ss = np.zeros(self.n, np.int64)
        self._info = np.zeros(4, np.int64)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib().flsim_sched_destroy(h)
            self._h = None

    def next_epoch(self) -> EpochPlan:
        rc = lib().flsim_sched_epoch(
            self._h, self._comp.ctypes.data_as(ctypes.c_void_p),
            self._fast.ctypes.data_as(ctypes.c_void_p), self._sw.ctypes.data_as(ctypes.c_void_p),
            self._ss.ctypes.data_as(ctypes.c_void_p), self._info.ctypes.data_as(ctypes.c_void_p))
        c, s, pushed, t = (int(x) for x in self._info)
        plan = EpochPlan(t, self._comp.copy(), self._fast.copy(),
                         [(int(self._sw[j]), int(self._ss[j])) for j in range(s)], c, s,
                         bool(pushed))
        check(rc)
        return plan

    def state(self):
        out = np.zeros(3, np.int64)
        lib().flsim_sched_state(self._h, out.ctypes.data_as(ctypes.c_void_p))
        return dict(t=int(out[0]), throttle_window=int(out[1]), slow_guy_gone=bool(out[2]))
