"""flsim: MI355X-native engine for the FL-simulation hot path of grossmanlev/FL-distributed-delay.

Importing the package does not touch the GPU; the HIP library is loaded on first use and there
is no CPU fallback (flsim._lib.FLSimError when libflsim.so is missing).
"""
from ._lib import FLSimError, lib  # noqa: F401
from .schedule import EpochPlan, Schedule, reference_delays  # noqa: F401
