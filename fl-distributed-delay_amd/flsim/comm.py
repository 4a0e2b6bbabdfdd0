"""The C-ABI's collective (include/flsim.h flsim_comm_*, flsim_allreduce_sum): the all-reduce
(sum, fp32, in place) of each rank's partial [S_t | losses] over RCCL, for callers that do not go
through torch.distributed (the reference has no collective: main.py:137 runs
every worker in one process, and the sharded partial sums meet before main.py:184's rule()).

  uid = Comm.unique_id()            # rank 0; ship the bytes to the other ranks
  comm = Comm(nranks, rank, uid)    # ncclCommInitRank (Comm() = the one-rank local communicator)
  comm.all_reduce_sum(buf)          # on the current stream
"""
from __future__ import annotations

import ctypes

import torch

from ._lib import COMM_ID_BYTES, check, lib, ptr, stream_ptr


class Comm:
    def __init__(self, nranks=1, rank=0, uid=None):
        if uid is not None and len(uid) != COMM_ID_BYTES:
            raise ValueError(f"unique id of {len(uid)} bytes (expected {COMM_ID_BYTES})")
        self._h = ctypes.c_void_p()
        idbuf = None if uid is None else (ctypes.c_ubyte * COMM_ID_BYTES).from_buffer_copy(uid)
        check(lib().flsim_comm_create(int(nranks), int(rank), idbuf, ctypes.byref(self._h)))

    @staticmethod
    def unique_id() -> bytes:
        buf = (ctypes.c_ubyte * COMM_ID_BYTES)()
        check(lib().flsim_comm_unique_id(buf))
        return bytes(buf)

    @property
    def size(self):
        return int(lib().flsim_comm_size(self._h))

    @property
    def rank(self):
        return int(lib().flsim_comm_rank(self._h))

    def all_reduce_sum(self, buf: torch.Tensor):
        """buf (a contiguous fp32 device tensor) = the sum of every rank's buf."""
        if buf.dtype != torch.float32 or not buf.is_contiguous():
            raise ValueError("all_reduce_sum takes a contiguous float32 tensor")
        check(lib().flsim_allreduce_sum(self._h, ptr(buf) if buf.numel() else None,
                                        buf.numel(), stream_ptr() if buf.is_cuda else None))

    def close(self):
        if self._h:
            h, self._h = self._h, ctypes.c_void_p()
            check(lib().flsim_comm_destroy(h))

    def __del__(self):
        try:
            self.close()
        except Exception:      # interpreter teardown
            pass
