"""ctypes binding of libfks.so (C ABI: include/fks.h).

The library sits next to this file (built in-tree by fate-llm_amd/Makefile).  There
is no CPU fallback: if the library or a HIP device is missing, every codec call
raises.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FKS_LIB_OVERRIDE") or os.path.join(_HERE, "libfks.so")  # override: diagnostics only

F32, BF16, F16 = 0, 1, 2
HAS_WD, FROZEN, STREAM_ROCM, FRESH, LIBM = 1, 2, 4, 8, 16
VALUE_SCALAR, VALUE_TENSOR = 0, 1
CHECK_SQRT_DOMAIN = 1
CHECK_PHILOX_RADIUS = 2
CHECK_PHILOX_BF16_RADIUS = 3
ABI_VERSION = 1

# every symbol include/fks.h declares (checked by tests/test_capi_host.py)
EXPORTED = (
    "fks_workspace_size", "fks_directional_step", "fks_perturb", "fks_normal", "fks_last_error",
    "fks_abi_version", "fks_build_target", "fks_host_jump_window", "fks_host_tables",
    "fks_directional_step_shard", "fks_stream_length", "fks_profile_begin", "fks_profile_end",
    "fks_shard_census", "fks_perturb_step", "fks_delta_workspace_size", "fks_delta_accumulate", "fks_delta_apply",
    "fks_plan_cache_clear", "fks_perturb_step_dev", "fks_device_selfcheck", "fks_build_id",
    "fks_zindex_size", "fks_zindex_attach", "fks_jwin_size", "fks_jwin_size_shard", "fks_jwin_attach",
    "fks_jwin_stats", "fks_cpu_generator_end", "fks_rocm_offset", "fks_rocm_grid_cap", "fks_source_id",
)


class FksTensor(ctypes.Structure):
    """struct fks_tensor (include/fks.h)."""

    _fields_ = [
        ("data", ctypes.c_void_p),
        ("numel", ctypes.c_int64),
        ("dtype", ctypes.c_int32),
        ("flags", ctypes.c_uint32),
        ("lr", ctypes.c_float),
        ("wd", ctypes.c_float),
    ]


class FksError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"libfks error {code}: {msg}")
        self.code = code


_lib = None
_lock = threading.Lock()


def load():
    """Load libfks.so (raises OSError if it has not been built)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise OSError(f"{LIB_PATH} not built; run `make -C fate-llm_amd` (hipcc, gfx950)")
        # torch's HIP runtime first: loading libfks.so (linked against /opt/rocm's) into a
        # process that has not imported torch yet leaves the library with a HIP runtime that
        # sees no device once torch brings in its own ("no ROCm-capable device is detected")
        import torch  # noqa: F401
        L = ctypes.CDLL(LIB_PATH)
        P, c_i32, c_u64, c_sz = ctypes.c_void_p, ctypes.c_int32, ctypes.c_uint64, ctypes.c_size_t
        L.fks_workspace_size.argtypes = [P, c_i32, c_i32, ctypes.POINTER(c_sz)]
        L.fks_directional_step.argtypes = [P, c_i32, P, P, c_i32, c_i32, P, c_sz, P]
        L.fks_perturb.argtypes = [P, c_i32, c_u64, P, P, c_sz, P]
        L.fks_normal.argtypes = [P, c_i32, c_u64, P, c_sz, P]
        L.fks_last_error.restype = ctypes.c_char_p
        L.fks_abi_version.restype = c_i32
        L.fks_build_target.restype = ctypes.c_char_p
        L.fks_build_id.restype = ctypes.c_char_p
        L.fks_source_id.restype = ctypes.c_char_p
        L.fks_host_jump_window.argtypes = [c_u64, ctypes.c_int64, P]
        L.fks_host_tables.argtypes = [c_i32, P, P, P, c_i32]
        L.fks_directional_step_shard.argtypes = [P, c_i32, P, P, c_i32, c_i32, c_i32, c_i32, P, c_sz, P]
        L.fks_stream_length.argtypes = [P, c_i32, ctypes.POINTER(ctypes.c_int64)]
        L.fks_shard_census.argtypes = [P, c_i32, c_i32, c_i32, P, P]
        L.fks_perturb_step.argtypes = [P, c_i32, c_u64, P, ctypes.c_double, c_i32, c_i32, P, c_sz, P]
        L.fks_profile_begin.argtypes = []
        L.fks_profile_end.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64),
                                      ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64)]
        L.fks_delta_workspace_size.argtypes = [P, c_i32, c_i32, ctypes.POINTER(c_sz)]
        L.fks_delta_accumulate.argtypes = [P, c_i32, P, P, c_i32, P, P, c_sz, P]
        L.fks_delta_apply.argtypes = [P, c_i32, P, P, P, c_sz, P]
        L.fks_plan_cache_clear.argtypes = []
        L.fks_perturb_step_dev.argtypes = [P, c_i32, c_u64, P, P, P, c_sz, P]
        L.fks_device_selfcheck.argtypes = [c_i32, ctypes.POINTER(c_u64), P, c_sz, P]
        L.fks_zindex_size.argtypes = [P, c_i32, ctypes.POINTER(c_sz)]
        L.fks_zindex_attach.argtypes = [P, c_sz]
        L.fks_jwin_size.argtypes = [P, c_i32, c_i32, ctypes.POINTER(c_sz)]
        L.fks_jwin_size_shard.argtypes = [P, c_i32, c_i32, c_i32, c_i32, ctypes.POINTER(c_sz)]
        L.fks_jwin_attach.argtypes = [P, c_sz]
        L.fks_jwin_stats.argtypes = [ctypes.POINTER(c_u64), ctypes.POINTER(c_u64)]
        L.fks_cpu_generator_end.argtypes = [P, c_i32, c_u64, P, ctypes.POINTER(c_i32), ctypes.POINTER(ctypes.c_uint32),
                                            ctypes.POINTER(c_i32), ctypes.POINTER(ctypes.c_double)]
        L.fks_rocm_offset.argtypes = [P, c_i32, ctypes.POINTER(c_u64)]
        L.fks_rocm_grid_cap.argtypes = [ctypes.POINTER(ctypes.c_int64)]
        for name in ("fks_workspace_size", "fks_directional_step", "fks_perturb", "fks_normal",
                     "fks_host_jump_window", "fks_host_tables", "fks_directional_step_shard",
                     "fks_stream_length", "fks_profile_begin", "fks_profile_end", "fks_shard_census", "fks_perturb_step",
                     "fks_delta_workspace_size", "fks_delta_accumulate", "fks_delta_apply", "fks_plan_cache_clear",
                     "fks_perturb_step_dev", "fks_device_selfcheck", "fks_zindex_size", "fks_zindex_attach",
                     "fks_jwin_size", "fks_jwin_size_shard", "fks_jwin_attach", "fks_jwin_stats",
                     "fks_cpu_generator_end", "fks_rocm_offset", "fks_rocm_grid_cap"):
            getattr(L, name).restype = ctypes.c_int
        if L.fks_abi_version() != ABI_VERSION:
            raise OSError(f"libfks.so ABI {L.fks_abi_version()} != {ABI_VERSION}")
        _lib = L
        return L


def build_id() -> str:
    """16 hex digits identifying the device code of the loaded libfks.so (fks_build_id)."""
    return load().fks_build_id().decode()


def source_id() -> str:
    """16 hex digits identifying the sources the loaded libfks.so was built from (fks_source_id)."""
    return load().fks_source_id().decode()


def check(rc: int) -> None:
    if rc != 0:
        raise FksError(rc, load().fks_last_error().decode(errors="replace"))
