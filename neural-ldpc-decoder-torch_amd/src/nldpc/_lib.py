"""ctypes binding of libnldpc.so, the C ABI declared in include/nldpc.h.

The library is built in-tree (neural-ldpc-decoder-torch_amd/lib/libnldpc.so, by
`make -C neural-ldpc-decoder-torch_amd/csrc` or __graft_entry__.build()).  There is no CPU
fallback: if the library is missing every decode call raises.

torch is imported before the library is loaded so that libnldpc.so's NEEDED libamdhip64.so.7 binds
to the HIP runtime torch already mapped (same SONAME): one runtime, one set of streams.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must be loaded first, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("NLDPC_LIB_PATH") or os.path.normpath(os.path.join(_HERE, "..", "..", "lib", "libnldpc.so"))

NLDPC_OK, NLDPC_EINVAL, NLDPC_EHIP, NLDPC_EUNSUPPORTED = 0, 1, 2, 3
NLDPC_SP, NLDPC_MS, NLDPC_QMS, NLDPC_NEURAL = 0, 1, 2, 3
ABI_VERSION = 4
FLAG_STREAM, FLAG_FUSED, FLAG_NO_STATE, FLAG_CN_TIED = 1, 2, 4, 8

# every symbol include/nldpc.h declares
EXPORTED = (
    "nldpc_abi_version", "nldpc_last_error", "nldpc_graph_create", "nldpc_graph_destroy", "nldpc_graph_dims",
    "nldpc_graph_edges", "nldpc_graph_attach_kernel", "nldpc_graph_kernels", "nldpc_fast_path", "nldpc_saved_bytes", "nldpc_forward", "nldpc_backward_workspace", "nldpc_backward", "nldpc_ber_count",
    "nldpc_awgn_llr", "nldpc_profile_begin", "nldpc_profile_end", "nldpc_bce_workspace", "nldpc_bce_loss",
    "nldpc_bce_grad", "nldpc_bce_loss_grad", "nldpc_bce_grad_unless_unit", "nldpc_forward_count", "nldpc_channel_llr", "nldpc_hbm_probe",
    "nldpc_code_object_sig",
)


# entries added after the ABI 4 structs were fixed (no layout change): optional in older builds
_ADDED_IN_ABI4 = ("nldpc_bce_loss_grad", "nldpc_bce_grad_unless_unit", "nldpc_code_object_sig")


class NldpcCfg(ctypes.Structure):
    _fields_ = [
        ("kind", ctypes.c_int32),
        ("qbit", ctypes.c_int32),
        ("ucn", ctypes.c_int32),
        ("vn_cumulative", ctypes.c_int32),
        ("llr_lo", ctypes.c_float),
        ("llr_hi", ctypes.c_float),
        ("first_iter", ctypes.c_int32),
        ("c2v_in", ctypes.c_int32),
        ("vn_prefix", ctypes.c_int32),
        ("flags", ctypes.c_int32),
    ]


class NldpcError(RuntimeError):
    pass


class NldpcUnsupported(NldpcError, NotImplementedError):
    pass


_lock = threading.Lock()
_lib = None

_vp = ctypes.c_void_p
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_PP = ctypes.POINTER(ctypes.c_void_p)


def _declare(lib):
    sig = {
        "nldpc_abi_version": (_i32, []),
        "nldpc_last_error": (ctypes.c_char_p, []),
        "nldpc_graph_create": (_i32, [_i32, _i32, _i32, ctypes.POINTER(_i32), _i32, ctypes.POINTER(_vp)]),
        "nldpc_graph_destroy": (_i32, [_vp]),
        "nldpc_graph_dims": (_i32, [_vp, ctypes.POINTER(_i32)]),
        "nldpc_graph_edges": (_i32, [_vp, ctypes.POINTER(_i32), ctypes.POINTER(_i32), ctypes.POINTER(_i32)]),
        "nldpc_graph_attach_kernel": (_i32, [_vp, _i32, _i32, _vp, ctypes.c_size_t, _i32, _i32, _i32]),
        "nldpc_graph_kernels": (_i32, [_vp, ctypes.POINTER(ctypes.c_uint32)]),
        "nldpc_code_object_sig": (_i32, [_vp, ctypes.c_size_t, _i32, ctypes.POINTER(ctypes.c_uint32),
                                         ctypes.POINTER(ctypes.c_uint32)]),
        "nldpc_fast_path": (_i32, [_vp, ctypes.POINTER(NldpcCfg), _i64, _i32, _i32, ctypes.POINTER(_i32)]),
        "nldpc_saved_bytes": (_i32, [_vp, ctypes.POINTER(NldpcCfg), _i64, _i32, ctypes.POINTER(ctypes.c_size_t)]),
        "nldpc_forward": (_i32, [_vp, ctypes.POINTER(NldpcCfg), _i64, _i32, _vp, _vp, _vp, _vp, _vp, _PP, _vp, _vp,
                                 _vp, _vp, _vp]),
        "nldpc_backward_workspace": (_i32, [_vp, ctypes.POINTER(NldpcCfg), _i64, _i32, ctypes.POINTER(ctypes.c_size_t)]),
        "nldpc_backward": (_i32, [_vp, ctypes.POINTER(NldpcCfg), _i64, _i32, _vp, _vp, _vp, _vp, _vp, _PP, _PP, _vp,
                                  _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, ctypes.c_size_t, _vp]),
        "nldpc_ber_count": (_i32, [_vp, _vp, _i64, _i64, _i32, _vp, _vp]),
        "nldpc_forward_count": (_i32, [_vp, ctypes.POINTER(NldpcCfg), _i64, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _i32,
                                       _vp, _vp]),
        "nldpc_awgn_llr": (_i32, [_vp, _i64, _i64, ctypes.c_float, ctypes.c_uint64, _i64, _i32, _vp]),
        "nldpc_channel_llr": (_i32, [_vp, _i64, _i64, ctypes.c_float, ctypes.c_uint64, _i64, _i32, _vp, _i64, _i64,
                                     ctypes.c_float, _i64, _i64, ctypes.c_float, _vp]),
        "nldpc_hbm_probe": (_i32, [_i32, _vp, _vp, _i64, _vp]),
        "nldpc_profile_begin": (_i32, [_i32]),
        "nldpc_profile_end": (_i32, [_i32, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(_i32)]),
        "nldpc_bce_workspace": (_i32, [_i64, _i32, ctypes.POINTER(ctypes.c_size_t)]),
        "nldpc_bce_loss": (_i32, [_PP, _i32, ctypes.POINTER(ctypes.c_float), _vp, _i64, _vp, _vp, ctypes.c_size_t, _vp]),
        "nldpc_bce_grad": (_i32, [_PP, _i32, ctypes.POINTER(ctypes.c_float), _vp, _i64, _vp, _PP, _vp]),
        "nldpc_bce_loss_grad": (_i32, [_PP, _i32, ctypes.POINTER(ctypes.c_float), _vp, _i64, _vp, _PP, _vp,
                                       ctypes.c_size_t, _vp]),
        "nldpc_bce_grad_unless_unit": (_i32, [_PP, _i32, ctypes.POINTER(ctypes.c_float), _vp, _i64, _vp, _PP, _vp]),
    }
    for name, (res, args) in sig.items():
        if name in _ADDED_IN_ABI4 and not hasattr(lib, name):
            continue  # an experiment library built before these entries (tools/exp_build.sh): the old pair runs
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args


def lib():
    """Load (once) and return the library; raises NldpcError when it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise NldpcError(
                    f"libnldpc.so not found at {LIB_PATH}: build it with "
                    "`make -C neural-ldpc-decoder-torch_amd/csrc` (or __graft_entry__.build()). "
                    "There is no CPU fallback.")
            h = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
            _declare(h)
            if h.nldpc_abi_version() != ABI_VERSION:
                raise NldpcError("libnldpc.so ABI version mismatch; rebuild the library")
            _lib = h
    return _lib


def check(status: int, what: str = "nldpc"):
    if status == NLDPC_OK:
        return
    msg = lib().nldpc_last_error().decode(errors="replace")
    if status == NLDPC_EINVAL:
        raise ValueError(f"{what}: {msg}")
    if status == NLDPC_EUNSUPPORTED:
        raise NldpcUnsupported(f"{what}: {msg}")
    raise NldpcError(f"{what}: {msg}")


def ptr(t) -> int | None:
    """Device pointer of a tensor (None for None)."""
    return None if t is None else t.data_ptr()


def ptr_array(tensors):
    arr = (ctypes.c_void_p * len(tensors))(*[ptr(t) for t in tensors])
    return ctypes.cast(arr, _PP), arr  # keep `arr` alive while the call runs


def stream_of(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream
