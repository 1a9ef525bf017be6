"""ctypes front-end of the CPU oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY -- the parity checker for the HIP product path, never the
thing measured or shipped.  Importers allowed: tests/, __graft_entry__.smoke(),
bench.py's cpu_baseline leg.  It restates the arithmetic that
``zo_utils.directional_derivative_step`` (python/fate_llm/algo/fedkseed/zo_utils.py:23-54)
and ``ZerothOrderOptimizer.random_perturb_parameters`` (optimizer.py:152-173) run
through torch's CPU generator; see fks_oracle.c for the torch file:line anchors.

Arrays are numpy: fp32 -> float32, bf16/f16 -> uint16 bit patterns, f64 -> float64.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.environ.get("FKS_ORACLE_LIB") or os.path.join(_HERE, "liboracle.so")  # override: sanitizer builds

F32, BF16, F16, F64 = 0, 1, 2, 3
DTYPE_NAMES = {"float32": F32, "bfloat16": BF16, "float16": F16, "float64": F64}
NP_STORAGE = {F32: np.float32, BF16: np.uint16, F16: np.uint16, F64: np.float64}

CAP_AVX2 = 0     # AVX2/AVX512 dispatch (what any x86-64 host with AVX2 runs)
CAP_DEFAULT = 1  # ATEN_CPU_CAPABILITY=default (libm Box-Muller)


def build() -> str:
    """Compile liboracle.so with the committed Makefile (gcc)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.fko_seed.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
        L.fko_random.argtypes = [ctypes.c_void_p]
        L.fko_random.restype = ctypes.c_uint32
        L.fko_random64.argtypes = [ctypes.c_void_p]
        L.fko_random64.restype = ctypes.c_uint64
        L.fko_fill_u32.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
        L.fko_normal.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int]
        L.fko_update.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int,
                                 ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_int]
        L.fko_perturb.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_double]
        L.fko_reconstruct.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_int32, ctypes.c_int32]
        L.fko_reconstruct.restype = ctypes.c_int
        L.fko_perturb_params.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_uint64, ctypes.c_double,
                                         ctypes.c_int32]
        L.fko_delta_accumulate.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32]
        L.fko_delta_accumulate.restype = ctypes.c_int
        L.fko_delta_apply.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_void_p]
        L.fko_perturb_params.restype = ctypes.c_int
        L.fko_set_contract.argtypes = [ctypes.c_int]
        L.fko_sizeof_gen.restype = ctypes.c_int
        L.fko_sizeof_tensor.restype = ctypes.c_int
        _lib = L
    return _lib


class Generator:
    """The CPU generator state torch.manual_seed(seed) creates (mt19937 + normal cache)."""

    def __init__(self, seed: int):
        self._buf = ctypes.create_string_buffer(lib().fko_sizeof_gen())
        self.seed(seed)

    @property
    def ptr(self):
        return ctypes.addressof(self._buf)

    def seed(self, seed: int):
        lib().fko_seed(self.ptr, int(seed) & 0xFFFFFFFFFFFFFFFF)

    def random(self) -> int:
        return lib().fko_random(self.ptr)

    def random64(self) -> int:
        return lib().fko_random64(self.ptr)

    def u32(self, n: int) -> np.ndarray:
        out = np.empty(n, np.uint32)
        lib().fko_fill_u32(self.ptr, out.ctypes.data, n)
        return out

    def state_words(self) -> np.ndarray:
        return np.frombuffer(self._buf.raw[: 624 * 4], dtype=np.uint32).copy()

    def left_next(self):
        raw = self._buf.raw
        return (int(np.frombuffer(raw[624 * 4: 624 * 4 + 4], np.int32)[0]),
                int(np.frombuffer(raw[624 * 4 + 4: 624 * 4 + 8], np.int32)[0]))

    def normal(self, n: int, dtype: int, capability: int = CAP_AVX2) -> np.ndarray:
        out = np.empty(max(n, 0), NP_STORAGE[dtype])
        lib().fko_normal(self.ptr, out.ctypes.data, n, dtype, capability)
        return out


def update(p: np.ndarray, z: np.ndarray, dtype: int, g: float, lr: float, wd, ) -> None:
    """In place: zo_utils.py:49 (wd not None) / :52 (wd None)."""
    assert p.flags.c_contiguous and z.flags.c_contiguous and p.size == z.size
    has_wd = wd is not None
    lib().fko_update(p.ctypes.data, z.ctypes.data, p.size, dtype, float(g), float(lr),
                     float(wd) if has_wd else 0.0, int(has_wd))


def perturb(p: np.ndarray, z: np.ndarray, dtype: int, scale: float) -> None:
    """In place: optimizer.py:173 with scale = scaling_factor * eps (python double)."""
    lib().fko_perturb(p.ctypes.data, z.ctypes.data, p.size, dtype, float(scale))


class _Tensor(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("numel", ctypes.c_int64), ("dtype", ctypes.c_int32),
                ("has_wd", ctypes.c_int32), ("lr", ctypes.c_double), ("wd", ctypes.c_double)]


def _tensor_array(arrays, dtypes, lrs, wds):
    T = (_Tensor * max(len(arrays), 1))()
    for i, (a, dt, lr, wd) in enumerate(zip(arrays, dtypes, lrs, wds)):
        assert a.flags.c_contiguous
        T[i].data = a.ctypes.data
        T[i].numel = a.size
        T[i].dtype = dt
        T[i].has_wd = int(wd is not None)
        T[i].lr = float(lr)
        T[i].wd = float(wd) if wd is not None else 0.0
    return T


def reconstruct(arrays, dtypes, lrs, wds, seeds, scalars, capability: int = CAP_AVX2) -> None:
    """fedkseed.py:136-141: for (seed, g) in order, skip g == 0.0, apply directional step.

    ``lrs``/``wds`` are per tensor, already resolved by the sticky rule (zo_utils.py:44-45).
    """
    assert lib().fko_sizeof_tensor() == ctypes.sizeof(_Tensor)
    T = _tensor_array(arrays, dtypes, lrs, wds)
    s = np.ascontiguousarray(np.asarray(seeds, dtype=np.uint64))
    g = np.ascontiguousarray(np.asarray(scalars, dtype=np.float64))
    rc = lib().fko_reconstruct(ctypes.addressof(T), len(arrays), s.ctypes.data, g.ctypes.data, len(s), capability)
    if rc != 0:
        raise RuntimeError(f"fko_reconstruct failed: {rc}")


def perturb_params(arrays, dtypes, seed: int, scale: float, capability: int = CAP_AVX2) -> None:
    T = _tensor_array(arrays, dtypes, [0.0] * len(arrays), [None] * len(arrays))
    rc = lib().fko_perturb_params(ctypes.addressof(T), len(arrays), int(seed), float(scale), capability)
    if rc != 0:
        raise RuntimeError(f"fko_perturb_params failed: {rc}")


def set_contract(bits: int) -> None:
    """Select an FMA-contraction variant (-1 = pinned default); for the pinning search only."""
    lib().fko_set_contract(int(bits))


def delta_accumulate(arrays, dtypes, seeds, coefs, delta: np.ndarray, frozen=None,
                     capability: int = CAP_AVX2) -> None:
    """Seed-sharded variant (not a reference routine): delta (f32, the arrays'
    concatenation) += f32(coef_s) * z_s, one fmaf per element and seed, seeds in order."""
    assert delta.dtype == np.float32 and delta.flags.c_contiguous
    assert delta.size == sum(a.size for a in arrays)
    T = _tensor_array(arrays, dtypes, [0.0] * len(arrays), [None] * len(arrays))
    fz = np.ascontiguousarray(np.asarray(frozen if frozen is not None else [0] * len(arrays), dtype=np.int32))
    s = np.ascontiguousarray(np.asarray(seeds, dtype=np.uint64))
    c = np.ascontiguousarray(np.asarray(coefs, dtype=np.float64))
    rc = lib().fko_delta_accumulate(ctypes.addressof(T), len(arrays), fz.ctypes.data, s.ctypes.data, c.ctypes.data,
                                    len(s), delta.ctypes.data, capability)
    if rc != 0:
        raise RuntimeError(f"fko_delta_accumulate failed: {rc}")


def delta_apply(arrays, dtypes, delta: np.ndarray, decays, frozen=None) -> None:
    """p = dtype(fmaf(f32(decay_i), p, -delta)) per tensor, in place."""
    T = _tensor_array(arrays, dtypes, [0.0] * len(arrays), [None] * len(arrays))
    fz = np.ascontiguousarray(np.asarray(frozen if frozen is not None else [0] * len(arrays), dtype=np.int32))
    d = np.ascontiguousarray(np.asarray(decays, dtype=np.float64))
    lib().fko_delta_apply(ctypes.addressof(T), len(arrays), fz.ctypes.data, delta.ctypes.data, d.ctypes.data)
