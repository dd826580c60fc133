"""ctypes binding of libdtc_amd.so (C ABI: include/dtc.h).

The library is loaded AFTER ``import torch`` so that its DT_NEEDED ``libamdhip64.so.7`` and
``librccl.so.1`` resolve to the copies torch already mapped: one HIP runtime and one RCCL per
process. There is no fallback: if the shared object is missing or does not
export a symbol the package raises at import time.
"""
from __future__ import annotations

import ctypes as C
import os

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DTC_LIB") or os.path.join(_HERE, "_lib", "libdtc_amd.so")  # DTC_LIB: A/B builds


class NativeError(RuntimeError):
    pass


def _load():
    if not os.path.exists(LIB_PATH):
        raise NativeError(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(or `make -C distributed-training-comparison_amd/csrc`)."
        )
    return C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)


lib = _load()

vp = C.c_void_p
i32 = C.c_int
i64 = C.c_int64
f32 = C.c_float
sz = C.c_size_t
P64 = C.POINTER(C.c_int64)
Pi32 = C.POINTER(C.c_int)
cstr = C.c_char_p


class ConvDesc(C.Structure):
    _fields_ = [(n, C.c_int) for n in ("n", "h", "w", "c", "k", "r", "s", "stride", "pad")]


PConv = C.POINTER(ConvDesc)

# name -> (restype, argtypes)
_SIGS = {
    "dtc_abi_version": (i32, []),
    "dtc_last_error": (cstr, []),
    "dtc_install_crash_handler": (i32, []),
    "dtc_set_option": (i32, [cstr, i32]),
    "dtc_get_option": (i32, [cstr]),
    "dtc_conv2d_workspace_size": (sz, [PConv, i32]),
    "dtc_conv2d_fwd": (i32, [PConv, vp, vp, vp, vp, vp, sz, vp]),
    "dtc_conv2d_dgrad": (i32, [PConv, vp, vp, vp, vp, vp, sz, vp]),
    "dtc_conv2d_fwd_sc": (i32, [PConv, vp, vp, vp, vp, vp, vp, vp, vp]),
    "dtc_conv2d_dgrad_sc": (i32, [PConv, vp, vp, vp, vp, vp, vp]),
    "dtc_conv2d_wgrad_sc_workspace_size": (sz, [PConv]),
    "dtc_conv2d_wgrad_sc": (i32, [PConv, vp, vp, vp, vp, vp, f32, vp, sz, vp]),
    "dtc_conv2d_dgrad_bn": (i32, [PConv, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, sz, vp]),
    "dtc_conv2d_wgrad": (i32, [PConv, vp, vp, vp, f32, vp, sz, vp]),
    "dtc_conv2d_wgrad_batch_workspace_size": (sz, [PConv, i32]),
    "dtc_conv2d_wgrad_batch": (i32, [PConv, i32, C.POINTER(vp), C.POINTER(vp), C.POINTER(vp), f32, vp, sz, vp]),
    "dtc_bn_stat_words": (sz, [i32]),
    "dtc_bn_stat_totals": (i32, [vp, i32, vp]),
    "dtc_bn_fwd_finalize": (i32, [vp, i32, i64, vp, vp, vp, vp, vp, f32, f32, vp, vp, vp, vp, vp]),
    "dtc_bn_apply_relu": (i32, [vp, vp, vp, vp, i64, i32, vp]),
    "dtc_bn_apply_add_relu": (i32, [vp, vp, vp, vp, vp, i64, i32, vp]),
    "dtc_bn_apply_dual_relu": (i32, [vp, vp, vp, vp, vp, vp, vp, i64, i32, vp]),
    "dtc_bn_bwd_reduce": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i64, i32, vp]),
    "dtc_bn_bwd_finalize": (i32, [vp, i32, i64, vp, vp, vp, f32, vp, vp, vp, vp]),
    "dtc_bn_bwd_apply": (i32, [vp, vp, vp, vp, vp, vp, vp, i64, i32, vp]),
    "dtc_stem_im2col": (i32, [vp, vp, i32, i32, i32, vp]),
    "dtc_stem_pack_weight": (i32, [vp, vp, i32, vp]),
    "dtc_stem_fwd": (i32, [vp, vp, vp, vp, i32, i32, i32, vp]),
    "dtc_stem_wgrad_workspace_size": (sz, [i32, i32, i32]),
    "dtc_stem_wgrad": (i32, [vp, vp, vp, f32, i32, i32, i32, vp, sz, vp]),
    "dtc_head_fwd": (i32, [vp, i32, i32, i32, vp, vp, i32, vp, vp, vp]),
    "dtc_head_bwd_workspace_size": (sz, [i32, i32, i32]),
    "dtc_head_bwd": (i32, [vp, vp, vp, i32, i32, i32, i32, f32, vp, vp, vp, vp, sz, vp]),
    "dtc_xent_fwd": (i32, [vp, vp, i32, i32, vp, vp, vp]),
    "dtc_xent_fwd_ex": (i32, [vp, vp, i32, i32, vp, vp, vp, vp, vp, vp]),
    "dtc_xent_bwd": (i32, [vp, vp, vp, vp, i32, i32, vp, vp]),
    "dtc_sgd_nesterov_flat": (i32, [vp, vp, vp, vp, i64, f32, f32, f32, vp, vp, vp]),
    "dtc_cast_f32_bf16": (i32, [vp, vp, i64, vp]),
    "dtc_amp_scale": (i32, [vp, vp, vp, i64, vp]),
    "dtc_amp_check_finite": (i32, [vp, i64, vp, vp]),
    "dtc_amp_update_scale": (i32, [vp, vp, vp, vp, f32, f32, i32, vp]),
    "dtc_cifar_augment": (i32, [vp, vp, i64, vp, vp, vp, i32, i32, i32, i32, C.POINTER(f32), C.POINTER(f32), vp, vp,
                                vp, vp]),
    "dtc_comm_unique_id_bytes": (sz, []),
    "dtc_comm_get_unique_id": (i32, [vp]),
    "dtc_comm_init": (i32, [C.POINTER(vp), i32, i32, vp, i32]),
    "dtc_comm_allreduce_sum": (i32, [vp, vp, sz, i32, vp]),
    "dtc_comm_broadcast": (i32, [vp, vp, sz, i32, i32, vp]),
    "dtc_comm_destroy": (i32, [vp]),
    "dtc_barrier": (i32, [vp, vp]),
    "dtc_comm_init_loopback": (i32, [C.POINTER(vp), i32, i32, C.c_float]),
    "dtc_comm_log_size": (i32, [vp]),
    "dtc_comm_log_entry": (i32, [vp, i32, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.POINTER(i32)]),
    "dtc_comm_log_clear": (i32, [vp]),
    "dtc_comm_init_thread_group": (i32, [C.POINTER(vp), i32, i32]),
    "dtc_comm_rank": (i32, [vp]),
    "dtc_comm_world": (i32, [vp]),
    "dtc_dp_create": (i32, [C.POINTER(vp), i32, C.POINTER(i32)]),
    "dtc_dp_destroy": (i32, [vp]),
    "dtc_dp_is_local": (i32, [vp]),
    "dtc_dp_broadcast": (i32, [vp, C.POINTER(vp), sz, i32, C.POINTER(vp)]),
    "dtc_dp_reduce_add": (i32, [vp, C.POINTER(vp), sz, C.POINTER(vp)]),
    "dtc_copy_peer": (i32, [vp, i32, vp, i32, sz, vp]),
    "dtc_rn18_create": (i32, [C.POINTER(vp), i32, i32, i32, i32, f32]),
    "dtc_rn18_destroy": (i32, [vp]),
    "dtc_rn18_num_params": (i32, [vp]),
    "dtc_rn18_param_info": (i32, [vp, i32, C.POINTER(cstr), P64, P64, Pi32, P64, P64]),
    "dtc_rn18_flat_numel": (i64, [vp]),
    "dtc_rn18_num_bn": (i32, [vp]),
    "dtc_rn18_bn_info": (i32, [vp, i32, C.POINTER(cstr), Pi32, P64, P64]),
    "dtc_rn18_bufs_numel": (i64, [vp]),
    "dtc_rn18_workspace_bytes": (sz, [vp]),
    "dtc_rn18_num_buckets": (i32, [vp]),
    "dtc_rn18_bucket_info": (i32, [vp, i32, P64, P64]),
    "dtc_rn18_bind": (i32, [vp, vp, vp, vp, vp, vp, vp, vp]),
    "dtc_rn18_set_precision": (i32, [vp, i32]),
    "dtc_rn18_precision": (i32, [vp]),
    "dtc_rn18_enable_capture": (i32, [vp]),
    "dtc_rn18_num_captures": (i32, [vp]),
    "dtc_rn18_capture_info": (i32, [vp, i32, C.POINTER(cstr), C.POINTER(sz), Pi32]),
    "dtc_rn18_num_activations": (i32, [vp]),
    "dtc_rn18_activation_info": (i32, [vp, i32, C.POINTER(cstr), C.POINTER(sz), Pi32]),
    "dtc_rn18_profile_begin": (i32, [vp, i32]),
    "dtc_rn18_profile_end": (i32, [vp, C.POINTER(C.c_double), C.POINTER(C.c_double), Pi32]),
    "dtc_rn18_profile_end_ex": (i32, [vp, i32, C.POINTER(C.c_double), C.POINTER(C.c_double), Pi32]),
    "dtc_rn18_profile_events": (i32, [vp, i32]),
    "dtc_rn18_profile_events_result": (i32, [vp, i32, C.POINTER(C.c_double), C.POINTER(C.c_double), Pi32]),
    "dtc_rn18_profile_events_dropped": (i32, [vp, P64]),
    "dtc_rn18_comm_timing": (i32, [vp, i32]),
    "dtc_rn18_comm_timing_result": (i32, [vp, i32, C.POINTER(C.c_double), C.POINTER(C.c_double), Pi32]),
    "dtc_rn18_forward": (i32, [vp, vp, vp, i32, vp]),
    "dtc_rn18_backward": (i32, [vp, vp, f32, vp, vp]),
    "dtc_rn18_xent_backward": (i32, [vp, vp, vp, vp, vp, f32, vp, vp]),
    "dtc_rn18_set_sync_bn": (i32, [vp, vp]),
    "dtc_rn18_dlogits_buffer": (i32, [vp, C.POINTER(sz)]),
}

SYMBOLS = tuple(_SIGS)

for _name, (_res, _args) in _SIGS.items():
    _fn = getattr(lib, _name)  # AttributeError here = library does not export the ABI
    _fn.restype = _res
    _fn.argtypes = _args


def last_error() -> str:
    s = lib.dtc_last_error()
    return s.decode() if s else ""


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        raise NativeError(f"{what or 'dtc call'} failed (code {rc}): {last_error()}")


def call(name: str, *args) -> None:
    check(getattr(lib, name)(*args), name)


def ptr(t) -> int | None:
    """Device pointer of a tensor (None passes NULL)."""
    if t is None:
        return None
    return t.data_ptr()


_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)
_GET_DEVICE = getattr(torch._C, "_cuda_getDevice", None)


def stream_ptr(stream=None) -> int:
    """HIP stream handle of `stream`, or of the current device's current stream (read through torch's raw
    getters: torch.cuda.current_stream() builds a Stream object through several Python lookups, a few us
    per call on every per-step launch)."""
    if stream is not None:
        return stream.cuda_stream
    if _RAW_STREAM is not None and _GET_DEVICE is not None:
        return _RAW_STREAM(_GET_DEVICE())
    return torch.cuda.current_stream().cuda_stream


def require_cuda(*tensors) -> None:
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise NativeError("dtc kernels run on the GPU only: got a tensor on " + str(t.device))
