"""ctypes binding of libflsim.so (the C-ABI declared in include/flsim.h).

The library is built in-tree by `make -C fl-distributed-delay_amd` (or __graft_entry__.build()).
torch is imported first so that libflsim.so binds to the HIP runtime torch already loaded
(same soname libamdhip64.so.7).  There is no fallback: a missing library raises.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must be loaded before libflsim.so, see module docstring)

LIB_PATH = os.environ.get("FLSIM_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                        "_lib", "libflsim.so")

EXPORTS = [
    "flsim_last_error", "flsim_sched_create", "flsim_sched_destroy", "flsim_sched_epoch",
    "flsim_sched_state", "flsim_pn1_param_count", "flsim_pn1_gradstate_bytes",
    "flsim_pn1_workspace_bytes", "flsim_pn1_workspace_offset", "flsim_pn1_workspace_split_part",
    "flsim_pn1_workspace_slice_major", "flsim_pn1_begin_epoch",
    "flsim_pn1_fwd_bwd_chunk", "flsim_pn1_fwd_bwd_input", "flsim_pn1_end_epoch",
    "flsim_pn1_eval_pool", "flsim_vgg11_param_count", "flsim_vgg11_gradstate_bytes",
    "flsim_vgg11_workspace_bytes", "flsim_vgg11_workspace_offset", "flsim_vgg11_begin_epoch",
    "flsim_vgg11_fwd_bwd_chunk", "flsim_vgg11_fwd_bwd_input", "flsim_vgg11_end_epoch",
    "flsim_vgg11_eval_pool", "flsim_vgg11_bn_param_count", "flsim_vgg11_bn_gradstate_bytes",
    "flsim_vgg11_bn_workspace_bytes", "flsim_vgg11_bn_workspace_offset",
    "flsim_vgg11_bn_stats_per_worker", "flsim_vgg11_bn_begin_epoch",
    "flsim_vgg11_bn_fwd_bwd_chunk", "flsim_vgg11_bn_fwd_bwd_input", "flsim_vgg11_bn_end_epoch",
    "flsim_vgg11_bn_eval_pool", "flsim_vgg11_bn_update_running",
    "flsim_pn1_eval_input", "flsim_vgg11_eval_input", "flsim_vgg11_bn_eval_input",
    "flsim_pn1_server_step", "flsim_vgg11_server_step", "flsim_vgg11_bn_server_step",
    "flsim_aggregate_adam", "flsim_aggregate_adam_rule", "flsim_aggregate_adam_sum",
    "flsim_cascade_program", "flsim_cascade_eval_host",
    "flsim_probe_enable", "flsim_probe_read", "flsim_probe_disable",
    "flsim_probe_kernel_count", "flsim_probe_kernel_name", "flsim_pn1_release",
    "flsim_pn1_fwd_bwd_chunk_async", "flsim_pn1_fwd_bwd_input_async",
    "flsim_aggregate_adam_rule_push", "flsim_pn1_fwd_rows", "flsim_pn1_bwd_rows",
    "flsim_pn1_load_rows", "flsim_pn1_fwd_loaded_rows", "flsim_vgg11_load_rows",
    "flsim_vgg11_fwd_bwd_loaded_rows", "flsim_vgg11_bn_load_rows",
    "flsim_vgg11_bn_fwd_bwd_loaded_rows",
    "flsim_comm_unique_id", "flsim_comm_create", "flsim_comm_size", "flsim_comm_rank",
    "flsim_allreduce_sum", "flsim_comm_destroy",
]
COMM_ID_BYTES = 128      # FLSIM_COMM_ID_BYTES


class FLSimError(RuntimeError):
    pass


MAX_ARRAYS = 64          # FLSIM_MAX_ARRAYS


class FlsimRule(ctypes.Structure):
    """flsim_rule (include/flsim.h): weight_ups of one rule() call."""
    _fields_ = [("k", ctypes.c_int32), ("c", ctypes.c_int32), ("prog", ctypes.c_void_p),
                ("info", ctypes.c_int32 * 4), ("n_arrays", ctypes.c_int32),
                ("arrays", ctypes.c_void_p * MAX_ARRAYS)]


class WorkerRec(ctypes.Structure):
    _fields_ = [("t", ctypes.c_uint32), ("i", ctypes.c_uint32), ("k", ctypes.c_uint32),
                ("pad", ctypes.c_uint32)]


_L = None
vp = ctypes.c_void_p


def lib():
    global _L
    if _L is not None:
        return _L
    if not os.path.exists(LIB_PATH):
        raise FLSimError(f"{LIB_PATH} not built: run `make -C fl-distributed-delay_amd` "
                         "(no CPU fallback exists)")
    L = ctypes.CDLL(LIB_PATH)
    L.flsim_last_error.restype = ctypes.c_char_p
    L.flsim_sched_create.restype = vp
    L.flsim_sched_create.argtypes = [ctypes.c_int32, vp, ctypes.c_int32, ctypes.c_int32]
    L.flsim_sched_destroy.argtypes = [vp]
    L.flsim_sched_epoch.argtypes = [vp] * 6
    L.flsim_sched_state.argtypes = [vp, vp]
    for net in ("pn1", "vgg11", "vgg11_bn"):      # one per-network contract (include/flsim.h)
        bn = [vp] if net == "vgg11_bn" else []    # + bn_stats (chunk) / running (eval)

        def f(name):
            return getattr(L, f"flsim_{net}_{name}")
        f("param_count").restype = ctypes.c_long
        f("gradstate_bytes").restype = ctypes.c_long
        f("workspace_bytes").restype = ctypes.c_long
        f("workspace_bytes").argtypes = [ctypes.c_int]
        f("workspace_offset").argtypes = [ctypes.c_int, ctypes.c_int, vp]
        f("begin_epoch").argtypes = [vp, vp, vp]
        f("fwd_bwd_chunk").argtypes = [
            vp, vp, ctypes.c_int, vp, vp, vp, vp, ctypes.c_int, vp, ctypes.c_int, vp, vp,
            ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_int, ctypes.c_int, vp] + bn + [vp]
        f("fwd_bwd_input").argtypes = [
            vp, vp, ctypes.c_int, vp, vp, vp, ctypes.c_int, vp, ctypes.c_uint64, ctypes.c_int,
            ctypes.c_int, vp] + bn + [vp]
        f("end_epoch").argtypes = [vp, vp, vp]
        f("eval_input").argtypes = [vp, vp, ctypes.c_int, vp, vp, ctypes.c_int] + bn + [vp, vp]
        f("server_step").argtypes = [vp, vp, vp, vp, vp, vp, ctypes.c_long, ctypes.c_double,
                                     ctypes.c_double, ctypes.c_double, ctypes.c_double, vp]
        f("eval_pool").argtypes = [vp, vp, ctypes.c_int, vp, vp, ctypes.c_int, ctypes.c_int,
                                   vp] + bn + [vp, vp]
    L.flsim_pn1_workspace_split_part.argtypes = [ctypes.c_int]
    L.flsim_pn1_workspace_slice_major.argtypes = [ctypes.c_int]
    L.flsim_vgg11_bn_update_running.argtypes = [vp, vp, ctypes.c_int, vp]
    L.flsim_pn1_release.argtypes = [vp]
    L.flsim_pn1_release.restype = None
    L.flsim_pn1_fwd_bwd_chunk_async.argtypes = [
        vp, vp, ctypes.c_int, vp, vp, vp, vp, ctypes.c_int, vp, ctypes.c_int, vp, vp,
        ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_int, vp, vp]
    L.flsim_pn1_fwd_bwd_input_async.argtypes = [
        vp, vp, ctypes.c_int, vp, vp, vp, ctypes.c_int, vp, ctypes.c_uint64, ctypes.c_int, vp, vp]
    L.flsim_pn1_fwd_rows.argtypes = [
        vp, vp, ctypes.c_int, ctypes.c_int, vp, vp, vp, ctypes.c_int, vp, ctypes.c_uint64,
        ctypes.c_int, vp, vp]
    L.flsim_pn1_bwd_rows.argtypes = [vp, vp, ctypes.c_int, ctypes.c_int, vp, ctypes.c_int, vp]
    L.flsim_pn1_load_rows.argtypes = [vp, vp, ctypes.c_int, ctypes.c_int, vp, vp, ctypes.c_int,
                                      vp]
    L.flsim_vgg11_load_rows.argtypes = L.flsim_pn1_load_rows.argtypes
    L.flsim_vgg11_fwd_bwd_loaded_rows.argtypes = [
        vp, vp, ctypes.c_int, ctypes.c_int, vp, vp, ctypes.c_uint64, ctypes.c_int, vp, vp]
    L.flsim_vgg11_bn_load_rows.argtypes = L.flsim_pn1_load_rows.argtypes
    L.flsim_vgg11_bn_fwd_bwd_loaded_rows.argtypes = [
        vp, vp, ctypes.c_int, ctypes.c_int, vp, vp, ctypes.c_uint64, ctypes.c_int, vp, vp, vp]
    L.flsim_pn1_fwd_loaded_rows.argtypes = [
        vp, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, vp, ctypes.c_uint64, ctypes.c_int,
        vp, vp]
    L.flsim_comm_unique_id.argtypes = [vp]
    L.flsim_comm_create.argtypes = [ctypes.c_int, ctypes.c_int, vp, vp]
    L.flsim_comm_size.argtypes = [vp]
    L.flsim_comm_rank.argtypes = [vp]
    L.flsim_allreduce_sum.argtypes = [vp, vp, ctypes.c_size_t, vp]
    L.flsim_comm_destroy.argtypes = [vp]
    L.flsim_aggregate_adam.argtypes = [
        vp, ctypes.c_int, vp, ctypes.c_int, vp, vp, vp, ctypes.c_long, vp, ctypes.c_int,
        ctypes.c_long, ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double, vp]
    L.flsim_aggregate_adam_sum.argtypes = [
        vp, ctypes.c_int, vp, vp, vp, ctypes.c_long, vp, ctypes.c_int,
        ctypes.c_long, ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double, vp]
    L.flsim_aggregate_adam_rule.argtypes = [
        vp, vp, vp, vp, vp, ctypes.c_long, vp, ctypes.c_int,
        ctypes.c_long, ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double, vp]
    L.flsim_aggregate_adam_rule_push.argtypes = [
        vp, vp, vp, vp, vp, vp, ctypes.c_long, vp, ctypes.c_int,
        ctypes.c_long, ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double, vp]
    L.flsim_cascade_program.argtypes = [ctypes.c_int, vp, vp, ctypes.c_int, vp, ctypes.c_int, vp]
    L.flsim_cascade_eval_host.argtypes = [vp, vp, vp, vp, ctypes.c_int, vp, ctypes.c_long, vp]
    L.flsim_probe_enable.argtypes = [ctypes.c_int]
    L.flsim_probe_read.argtypes = [vp, vp, vp]
    L.flsim_probe_kernel_name.restype = ctypes.c_char_p
    L.flsim_probe_kernel_name.argtypes = [ctypes.c_int]
    _L = L
    return L


def check(rc):
    if rc != 0:
        msg = lib().flsim_last_error().decode(errors="replace")
        if rc == 1:
            if "IndexError" in msg:
                raise IndexError(msg)
            if "ZeroDivisionError" in msg:
                raise ZeroDivisionError(msg)
            raise ValueError(msg)
        raise FLSimError(msg)


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def stream_ptr(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


class KernelProbe:
    """HIP events around every worker-batched GEMM launch (recorded by libflsim.so on the launch
    stream).  read() -> {kernel name: (launches, total_ms, total_algorithmic_flops)}."""

    def __init__(self, capacity=20000):
        check(lib().flsim_probe_enable(capacity))

    def read(self):
        import numpy as np
        n = lib().flsim_probe_kernel_count()
        cnt = np.zeros(n, np.int32)
        ms = np.zeros(n, np.float64)
        fl = np.zeros(n, np.float64)
        check(lib().flsim_probe_read(cnt.ctypes.data_as(vp), ms.ctypes.data_as(vp),
                                     fl.ctypes.data_as(vp)))
        return {lib().flsim_probe_kernel_name(k).decode(): (int(cnt[k]), float(ms[k]), float(fl[k]))
                for k in range(n) if cnt[k]}

    def close(self):
        check(lib().flsim_probe_disable())
