"""Host side of the MI355X FedKSeed codec: torch tensors in, libfks.so calls out.

Three operations, each replacing one reference routine (include/fks.h has the ABI):

* ``directional_step``  -- K x zo_utils.directional_derivative_step
  (python/fate_llm/algo/fedkseed/zo_utils.py:23-54); K = 1 is the local ZO update
  (optimizer.py:92), K = len(seeds) the reconstruct loop of ClientTrainer.train_once
  (fedkseed.py:136-141) in ONE device pass.
* ``perturb``          -- ZerothOrderOptimizer.random_perturb_parameters
  (optimizer.py:152-173).
* ``normal_``          -- the torch.normal(mean=0, std=1, size, dtype) draws the two
  routines above make after torch.manual_seed(seed) (zo_utils.py:47, optimizer.py:170).

The z stream (``stream_mode``) is the one the reference draws where its parameters live
(zo_utils.py:47 and optimizer.py:170-172 draw on ``param.data.device``):

* ``"torch_rocm"``: torch's HIP-device generator, Philox4x32-10 + rocrand's Box-Muller in
  torch's grid-stride mapping -- a reference client whose model sits on an MI355X, and
  what the default ``"auto"`` resolves to for every tensor the codec accepts;
* ``"torch_cpu"``: torch's CPU generator, mt19937 + normal_fill -- a reference client that
  trains on the CPU (the FedKSeed tutorial's configuration); an explicit choice.  Its fp32
  z has two flavours, as torch's CPU kernel has (``cpu_fp32_flavour``): Cephes under
  ATen's AVX2 / AVX512 capability, glibc's logf / sinf / cosf under DEFAULT.

All parties of one federation must draw the same stream.  The
process-wide setting comes from ``FKS_STREAM_MODE`` and ``set_stream_mode``: one of the
two streams, or ``"auto"`` -- the DEFAULT when ``FKS_STREAM_MODE`` is unset -- which draws
what the reference draws for the call's tensors: ``torch_rocm`` for tensors on a HIP
device (every tensor the codec accepts), so a drop-in client on an MI355X gives the bits
an unmodified reference client on the same device gives.  ``torch_cpu`` (1.8x faster
here) is the explicit choice for a federation whose reference clients train on the CPU,
or whose parties are all drop-in clients; the round payloads carry the stream so that a
drop-in arbiter rejects a mixed federation (payload.py).  Updates are applied in
place (the reference rebinds ``param.data`` to a new tensor of identical values), and
torch's generators are left where the reference's draws leave them (``_leave``).

There is no CPU path: tensors must live on a HIP device and libfks.so must be
loadable, otherwise these functions raise.
"""
from __future__ import annotations

import ctypes
import math
import os
import threading
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np
import torch

from . import _native as N

_DTYPES = {torch.float32: N.F32, torch.bfloat16: N.BF16, torch.float16: N.F16}
STREAM_MODES = ("torch_cpu", "torch_rocm")
STREAM_SETTINGS = STREAM_MODES + ("auto",)
_stream_mode = os.environ.get("FKS_STREAM_MODE") or "auto"
if _stream_mode not in STREAM_SETTINGS:
    raise ValueError(f"FKS_STREAM_MODE must be one of {STREAM_SETTINGS}, not {_stream_mode!r}")


def set_stream_mode(mode: str) -> None:
    """The z stream every codec call draws unless told otherwise (module docstring):
    "torch_cpu", "torch_rocm" or "auto" (the stream of the tensors' device)."""
    global _stream_mode
    if mode not in STREAM_SETTINGS:
        raise ValueError(f"stream_mode must be one of {STREAM_SETTINGS}, not {mode!r}")
    _stream_mode = mode


def get_stream_mode() -> str:
    """The process-wide setting (possibly "auto"); resolve_stream_mode gives the stream."""
    return _stream_mode


# fp32 tensors of >= 16 elements on the torch_cpu stream: torch's CPU kernel fills them with
# normal_fill_16_AVX2 (Cephes log / sincos) when ATen dispatches to its AVX2 or AVX512 build
# and with normal_fill_16<float> (glibc's logf / sinf / cosf) under the DEFAULT capability --
# ATEN_CPU_CAPABILITY=default, or a host without AVX2 (DistributionTemplates.h:139-149,
# 195-205).  The reference draws whichever its own process dispatches to, so the flavour is
# this process's torch's unless FKS_CPU_FP32_FLAVOUR or set_cpu_fp32_flavour names one (a
# drop-in joining reference clients that run another capability).  bf16 / f16 tensors and
# tensors of < 16 elements draw the same z either way.
CPU_FP32_FLAVOURS = ("avx", "libm")
_cpu_fp32_flavour = os.environ.get("FKS_CPU_FP32_FLAVOUR") or None
if _cpu_fp32_flavour is not None and _cpu_fp32_flavour not in CPU_FP32_FLAVOURS:
    raise ValueError(f"FKS_CPU_FP32_FLAVOUR must be one of {CPU_FP32_FLAVOURS}, not {_cpu_fp32_flavour!r}")


def set_cpu_fp32_flavour(flavour: Optional[str]) -> None:
    """"avx", "libm", or None for this process's torch's CPU capability."""
    global _cpu_fp32_flavour
    if flavour is not None and flavour not in CPU_FP32_FLAVOURS:
        raise ValueError(f"cpu fp32 flavour must be one of {CPU_FP32_FLAVOURS} or None, not {flavour!r}")
    _cpu_fp32_flavour = flavour


def cpu_fp32_flavour() -> str:
    """The fp32 z of the torch_cpu stream: "avx" (normal_fill_16_AVX2) or "libm"
    (normal_fill_16<float>), per the setting or torch.backends.cpu.get_cpu_capability()."""
    if _cpu_fp32_flavour is not None:
        return _cpu_fp32_flavour
    return "avx" if torch.backends.cpu.get_cpu_capability() in ("AVX2", "AVX512") else "libm"


def stream_identity(stream_mode: str, params=None) -> str:
    """The stream as parties compare it (payload.py): ``stream_mode``, except that a
    torch_cpu stream whose fp32 z is the libm flavour is "torch_cpu_libm" -- when ``params``
    (an iterable of tensors, None = assume so) hold an fp32 tensor of >= 16 elements, the
    only draws the flavour changes."""
    if stream_mode != "torch_cpu" or cpu_fp32_flavour() != "libm":
        return stream_mode
    if params is not None and not any(p.dtype == torch.float32 and p.numel() >= 16 for p in params):
        return stream_mode
    return "torch_cpu_libm"


def resolve_stream_mode(device=None, stream_mode=None) -> str:
    """The stream a call on tensors of ``device`` draws: ``stream_mode`` if given, else the
    process-wide setting; "auto" is the stream the reference draws on that device
    (zo_utils.py:47, optimizer.py:170-172 draw on ``param.data.device``): torch's HIP
    generator on a HIP device, the CPU generator otherwise (and for ``device=None``, a
    call with no tensors, which draws nothing)."""
    m = _stream_mode if stream_mode is None else stream_mode
    if m not in STREAM_SETTINGS:
        raise ValueError(f"stream_mode must be one of {STREAM_SETTINGS}, not {m!r}")
    if m == "auto":
        return "torch_rocm" if device is not None and torch.device(device).type == "cuda" else "torch_cpu"
    return m


@dataclass
class ParamSpec:
    """One tensor of the z stream, in draw order."""

    tensor: torch.Tensor
    lr: float = 0.0
    weight_decay: Optional[float] = None  # None -> zo_utils.py:52 form (no decay term)
    frozen: bool = False                  # draws its z, is not written
    fresh: bool = False                   # the reference's param.data is a tensor an earlier step allocated (mark_rebound)


def _f32(x: float) -> float:
    return float(np.float32(x))


class _Batch:
    """fks_tensor array for a list of specs (keeps contiguous staging copies alive)."""

    def __init__(self, specs: Sequence[ParamSpec], stream_mode=None):
        self.specs = list(specs)
        self.copies = []  # (original, contiguous staging) pairs to write back
        self.device = None
        for sp in self.specs:
            t = sp.tensor
            if t.dtype not in _DTYPES:
                raise NotImplementedError(f"FedKSeed codec: dtype {t.dtype} is not supported on the MI355X path")
            if t.device.type != "cuda":
                raise ValueError("FedKSeed codec: parameters must be on a HIP device "
                                 f"(got {t.device}); there is no CPU path")
            if self.device is None:
                self.device = t.device
            elif t.device != self.device:
                raise ValueError("FedKSeed codec: all parameters must be on one device")
        self.stream_mode = resolve_stream_mode(self.device, stream_mode)
        stream_flag = N.STREAM_ROCM if self.stream_mode == "torch_rocm" else 0
        # the CPU stream's fp32 flavour travels on every tensor (the library wants one per call)
        cpu_flag = N.LIBM if not stream_flag and cpu_fp32_flavour() == "libm" else 0
        arr = (N.FksTensor * max(1, len(self.specs)))()
        for i, sp in enumerate(self.specs):
            t = sp.tensor
            if not t.is_contiguous():
                c = t.contiguous()
                self.copies.append((t, c))
                t = c
            arr[i].data = t.data_ptr() if t.numel() else None
            arr[i].numel = t.numel()
            arr[i].dtype = _DTYPES[t.dtype]
            flags = stream_flag | cpu_flag
            if sp.weight_decay is not None:
                flags |= N.HAS_WD
            if sp.frozen:
                flags |= N.FROZEN
            if sp.fresh and stream_flag and t.dtype == torch.float16:  # only the torch_rocm f16 chain reads it
                flags |= N.FRESH
            arr[i].flags = flags
            arr[i].lr = _f32(sp.lr)
            arr[i].wd = _f32(sp.weight_decay) if sp.weight_decay is not None else 0.0
        self.arr = arr
        self.n = len(self.specs)

    def workspace(self, k: int, delta: bool = False):
        L = N.load()
        nbytes = ctypes.c_size_t(0)
        size_fn = L.fks_delta_workspace_size if delta else L.fks_workspace_size
        N.check(size_fn(ctypes.addressof(self.arr), self.n, int(k), ctypes.byref(nbytes)))
        ws = torch.empty(max(int(nbytes.value), 1), dtype=torch.uint8, device=self.device)
        return ws, int(nbytes.value)

    def finish(self):
        for orig, c in self.copies:
            orig.copy_(c)


def _stream_handle(device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def _seed_u64(s) -> int:
    s = int(s)
    if s < 0:
        s &= 0xFFFFFFFFFFFFFFFF  # torch.manual_seed accepts negatives as two's complement
    if s >= 1 << 64:
        raise ValueError(f"seed {s} out of range")
    return s


# ---------------------------------------------------------------- torch's global generators
# The reference draws z from torch's generators right after torch.manual_seed(seed)
# (zo_utils.py:42,47; optimizer.py:165,170-172), so once a call returns, the generator of
# the parameters' device stands past the last seed's draws, and whatever the caller draws
# next -- a sampler's permutation, the dropout of the zeroth-order closure -- starts there.
# The codec's kernels draw nothing from torch; every call that stands for the reference's
# draws (leave_generator=True, the default) re-seeds torch with the last seed and moves the
# generator of the call's stream to where the reference's draws leave it:
#   torch_rocm: the device generator's Philox offset (fks_rocm_offset);
#   torch_cpu:  the CPU generator's mt19937 state and its cached normal (fks_cpu_generator_end).
_CPU_STATE_BYTES = 5056  # sizeof(CPUGeneratorImplState) (ATen/CPUGeneratorImpl.h), torch.get_rng_state()
_cpu_state_cache = {}    # (numels, seed) -> state tensor: the zeroth-order step's three calls share one
_cpu_state_lock = threading.Lock()


def cpu_generator_state(arr, n: int, seed: int) -> torch.Tensor:
    """The CPU generator's state (torch.get_rng_state() bytes) after torch.manual_seed(seed)
    and the CPU-stream draws of the ``n`` fks_tensor entries of ``arr`` (host-only: only
    their sizes and dtypes matter): CPUGeneratorImplState = the legacy THGeneratorState
    (the_initial_seed u64 @0, left i32 @8, seeded i32 @12, next u64 @16, state u64[624]
    @24, normal_x / normal_y / normal_rho f64 @5016 / 5024 / 5032, normal_is_valid i32
    @5040) + the float normal cache @5048 (reset by manual_seed)."""
    seed = _seed_u64(seed)
    key = (tuple((int(x.numel), int(x.dtype)) for x in arr[:n]), seed)
    with _cpu_state_lock:
        hit = _cpu_state_cache.get(key)
    if hit is not None:
        return hit
    st = np.zeros(624, dtype=np.uint32)
    left, nxt = ctypes.c_int32(0), ctypes.c_uint32(0)
    valid, normal = ctypes.c_int32(0), ctypes.c_double(0.0)
    N.check(N.load().fks_cpu_generator_end(ctypes.addressof(arr), n, seed, st.ctypes.data, ctypes.byref(left),
                                           ctypes.byref(nxt), ctypes.byref(valid), ctypes.byref(normal)))
    raw = np.zeros(_CPU_STATE_BYTES, dtype=np.uint8)
    raw[0:8].view("<u8")[0] = seed
    raw[8:12].view("<i4")[0] = left.value
    raw[12:16].view("<i4")[0] = 1
    raw[16:24].view("<u8")[0] = nxt.value
    raw[24:24 + 8 * 624].view("<u8")[:] = st
    if valid.value:
        raw[5024:5032].view("<f8")[0] = normal.value
        raw[5040:5044].view("<i4")[0] = 1
    out = torch.from_numpy(raw)
    with _cpu_state_lock:
        if len(_cpu_state_cache) >= 16:
            _cpu_state_cache.pop(next(iter(_cpu_state_cache)))
        _cpu_state_cache[key] = out
    return out


def rocm_offset(b: "_Batch") -> int:
    """The Philox offset one seed's torch_rocm draws of b's tensors advance the device
    generator by (fks_rocm_offset)."""
    off = ctypes.c_uint64(0)
    with torch.cuda.device(b.device):
        N.check(N.load().fks_rocm_offset(ctypes.addressof(b.arr), b.n, ctypes.byref(off)))
    return int(off.value)


def rocm_grid_cap(device=None) -> int:
    """torch's grid cap for draws on ``device`` (fks_rocm_grid_cap): CUs x (max threads per
    CU / 256), 2,048 on an MI355X in SPX mode.  The torch_rocm stream of every tensor of more
    than 256 x cap / 4 elements depends on it (DistributionTemplates.h:50-62), so it is part
    of the stream's identity on the wire (payload.py)."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    cap = ctypes.c_int64(0)
    with torch.cuda.device(dev):
        N.check(N.load().fks_rocm_grid_cap(ctypes.byref(cap)))
    return int(cap.value)


def _leave(b: "_Batch", seed) -> None:
    seed = _seed_u64(seed)
    torch.manual_seed(seed)  # every generator, as the reference's call does
    if b.stream_mode == "torch_rocm":
        idx = b.device.index if b.device.index is not None else torch.cuda.current_device()
        torch.cuda.default_generators[idx].set_offset(rocm_offset(b))
    else:
        torch.set_rng_state(cpu_generator_state(b.arr, b.n, seed))


def leave_generators(specs: Sequence[ParamSpec], seed: int, stream_mode=None) -> None:
    """Leave torch's generators where the reference's torch.manual_seed(seed) and the
    draws of ``specs`` (every tensor, frozen ones included) leave them."""
    b = _Batch(specs, stream_mode)
    if b.device is not None:
        _leave(b, seed)


def directional_step(specs: Sequence[ParamSpec], seeds: Sequence[int], values: Sequence[float],
                     value_is_tensor: bool = False, shard: int = 0, nshards: int = 1, stream_mode=None,
                     cache_windows: bool = False, leave_generator: bool = True) -> None:
    """For each (seed, value) in order: p <- p - lr*(value*z + wd*p) over ``specs``.

    ``shard``/``nshards``: only the shard-th of nshards equal parts of the parameter stream
    is updated (element sharding across ranks; bit-identical): runs of MT19937 blocks
    (torch_cpu) or of whole Philox rows (torch_rocm).  ``cache_windows``: keep the jumped
    generator windows in the reconstruct window cache (jwin_reserve) so that the next
    reconstruct of the same list skips the jumps of the seeds it finds there.
    ``leave_generator``: leave torch's generators where the reference's last
    directional_derivative_step leaves them (see _leave)."""
    if len(seeds) != len(values):
        raise ValueError("seeds and values differ in length")
    if not specs or not len(seeds):
        return
    b = _Batch(specs, stream_mode)
    if b.device is None:
        return
    L = N.load()
    s = np.ascontiguousarray([_seed_u64(x) for x in seeds], dtype=np.uint64)
    v = np.ascontiguousarray([float(x) for x in values], dtype=np.float64)
    with torch.cuda.device(b.device):
        if cache_windows and b.stream_mode == "torch_cpu":
            jwin_reserve(b, len(s), shard, nshards)
        ws, nbytes = b.workspace(len(s))
        N.check(L.fks_directional_step_shard(ctypes.addressof(b.arr), b.n, s.ctypes.data, v.ctypes.data, len(s),
                                             N.VALUE_TENSOR if value_is_tensor else N.VALUE_SCALAR,
                                             int(shard), int(nshards), ws.data_ptr(), nbytes,
                                             _stream_handle(b.device)))
        b.finish()
        if leave_generator:
            _leave(b, s[-1])


# ---------------------------------------------------------------- z-index buffer
# A one-seed bf16 perturb stores its Box-Muller table indices (1 byte per parameter) so
# that the zeroth-order step's second and third calls with the same seed replay them
# (include/fks.h, fks_zindex_attach).  The buffer is a torch tensor -- it counts in
# torch.cuda.memory_allocated and goes back to torch's allocator on release -- and is
# taken only while it stays within ZINDEX_BUDGET_FRAC of the device's memory (the
# parameters' owner keeps the rest for activations); FKS_ZCACHE=0 turns it off.
ZINDEX_BUDGET_FRAC = float(os.environ.get("FKS_ZINDEX_BUDGET_FRAC", "0.05"))
ZINDEX_HEADROOM = 1 << 30  # free device memory the buffer always leaves untouched
_zindex = {}  # device index -> attached uint8 tensor
_zindex_lock = threading.Lock()


def _alloc_zindex(nbytes: int, device) -> torch.Tensor:
    return torch.empty(nbytes, dtype=torch.uint8, device=device)


def zindex_reserve(b: "_Batch") -> bool:
    """Attach a z-index buffer big enough for one-seed calls over ``b`` on its device, if
    the budget allows; returns whether one is attached."""
    if os.environ.get("FKS_ZCACHE", "1").startswith("0") or ZINDEX_BUDGET_FRAC <= 0:
        return False
    L = N.load()
    need = ctypes.c_size_t(0)
    N.check(L.fks_zindex_size(ctypes.addressof(b.arr), b.n, ctypes.byref(need)))
    need = int(need.value)
    if need == 0:
        return False
    idx = b.device.index if b.device.index is not None else torch.cuda.current_device()
    with _zindex_lock:
        cur = _zindex.get(idx)
        if cur is not None and cur.numel() >= need:
            return True
        if need > ZINDEX_BUDGET_FRAC * torch.cuda.get_device_properties(idx).total_memory:
            return False
        # a speed cache only: never take the last of the device's memory for it (free memory
        # as the driver sees it plus what torch holds cached and could hand out), and a
        # failed allocation means "generate the z values", not an error
        free, _ = torch.cuda.mem_get_info(idx)
        reclaimable = torch.cuda.memory_reserved(idx) - torch.cuda.memory_allocated(idx)
        if need > free + reclaimable - ZINDEX_HEADROOM:
            return False
        try:
            buf = _alloc_zindex(need, b.device)
        except torch.cuda.OutOfMemoryError:
            return False
        N.check(L.fks_zindex_attach(buf.data_ptr(), need))  # waits for the old buffer's last user
        _zindex[idx] = buf
        return True


def zindex_release(device=None) -> None:
    """Detach and free the z-index buffer of ``device`` (all devices if None)."""
    L = N.load()
    with _zindex_lock:
        for idx in [d for d in _zindex if device is None or d == torch.device(device).index]:
            with torch.cuda.device(idx):
                N.check(L.fks_zindex_attach(None, 0))
            del _zindex[idx]


# ---------------------------------------------------------------- reconstruct window cache
# The generator windows a multi-seed bf16 reconstruct jumps to, one set per seed (include/
# fks.h, fks_jwin_attach): a client reconstructs the same seed list from model_0 every
# round, so from the second round on the jumps are skipped.  A torch tensor taken under
# JWIN_BUDGET_FRAC of the device's memory and never past its free memory (less
# ZINDEX_HEADROOM); an allocation failure only means "jump"; FKS_NO_JWIN=1 (or true / yes)
# turns it off, as FKS_NO_JWIN does in the library (fks_capi.cpp env_on).
JWIN_BUDGET_FRAC = float(os.environ.get("FKS_JWIN_BUDGET_FRAC", "0.05"))
_jwin = {}  # device index -> attached uint8 tensor


def _env_on(name: str) -> bool:
    """A boolean switch: set to 1 / true / yes (any case); unset, empty, 0, false, no: off."""
    return os.environ.get(name, "").strip().lower() in ("1", "true", "yes", "on")


def _alloc_jwin(nbytes: int, device) -> torch.Tensor:
    return torch.empty(nbytes, dtype=torch.uint8, device=device)


def jwin_reserve(b: "_Batch", k: int, shard: int = 0, nshards: int = 1) -> bool:
    """Attach a window cache that holds ``k`` seeds' window sets for the tensor list of
    ``b`` (element shard ``shard`` of ``nshards``: sets sized from that shard's plan) on
    its device, if the budget allows; returns whether one is attached."""
    if _env_on("FKS_NO_JWIN") or JWIN_BUDGET_FRAC <= 0:
        return False
    L = N.load()
    need = ctypes.c_size_t(0)
    N.check(L.fks_jwin_size_shard(ctypes.addressof(b.arr), b.n, int(k), int(shard), int(nshards), ctypes.byref(need)))
    need = int(need.value)
    if need == 0:
        return False
    idx = b.device.index if b.device.index is not None else torch.cuda.current_device()
    with _zindex_lock:
        cur = _jwin.get(idx)
        if cur is not None and cur.numel() >= need:
            return True
        if need > JWIN_BUDGET_FRAC * torch.cuda.get_device_properties(idx).total_memory:
            return False
        free, _ = torch.cuda.mem_get_info(idx)
        reclaimable = torch.cuda.memory_reserved(idx) - torch.cuda.memory_allocated(idx)
        if need > free + reclaimable - ZINDEX_HEADROOM:
            return False
        try:
            buf = _alloc_jwin(need, b.device)
        except torch.cuda.OutOfMemoryError:
            return False
        N.check(L.fks_jwin_attach(buf.data_ptr(), need))  # waits for the old buffer's last user
        _jwin[idx] = buf
        return True


def jwin_release(device=None) -> None:
    """Detach and free the reconstruct window cache of ``device`` (all devices if None)."""
    L = N.load()
    with _zindex_lock:
        for idx in [d for d in _jwin if device is None or d == torch.device(device).index]:
            with torch.cuda.device(idx):
                N.check(L.fks_jwin_attach(None, 0))
            del _jwin[idx]


def jwin_stats():
    """(seeds found in the window cache, seeds jumped into it) since the library loaded."""
    h, m = ctypes.c_uint64(0), ctypes.c_uint64(0)
    N.check(N.load().fks_jwin_stats(ctypes.byref(h), ctypes.byref(m)))
    return int(h.value), int(m.value)


def perturb(tensors: Sequence[torch.Tensor], seed: int, scales, stream_mode=None, leave_generator: bool = True,
            fresh: Optional[Sequence[bool]] = None) -> None:
    """p <- p + scale_i*z for every tensor i (scale = scaling_factor*eps of its group, a
    python double); ``scales`` is one number for all tensors or one per tensor; ``fresh``:
    ParamSpec.fresh per tensor."""
    specs = [ParamSpec(t, fresh=bool(fresh[i]) if fresh else False) for i, t in enumerate(tensors)]
    if not specs:
        return
    if isinstance(scales, (int, float)):
        scales = [float(scales)] * len(specs)
    if len(scales) != len(specs):
        raise ValueError("one scale per tensor")
    b = _Batch(specs, stream_mode)
    if b.device is None:
        return
    L = N.load()
    sc = np.ascontiguousarray([float(x) for x in scales], dtype=np.float64)
    with torch.cuda.device(b.device):
        if b.stream_mode == "torch_cpu":
            zindex_reserve(b)
        ws, nbytes = b.workspace(1)
        N.check(L.fks_perturb(ctypes.addressof(b.arr), b.n, _seed_u64(seed), sc.ctypes.data, ws.data_ptr(), nbytes,
                              _stream_handle(b.device)))
        b.finish()
        if leave_generator:
            _leave(b, seed)


def perturb_step(specs: Sequence[ParamSpec], seed: int, scales: Sequence[float], value: float,
                 value_is_tensor: bool = True, update: bool = True, stream_mode=None,
                 leave_generator: bool = True) -> None:
    """zeroth_order_step's restore perturbation fused with its directional step, in one
    device pass: p <- p + scale_i*z, then (``update``) p <- p - lr*(value*z + wd*p) with
    the same z.  Equal, bit for bit, to ``perturb`` followed by ``directional_step``
    over the same tensor list."""
    specs = list(specs)
    if not specs:
        return
    if len(scales) != len(specs):
        raise ValueError("one scale per tensor")
    b = _Batch(specs, stream_mode)
    if b.device is None:
        return
    L = N.load()
    sc = np.ascontiguousarray([float(x) for x in scales], dtype=np.float64)
    with torch.cuda.device(b.device):
        ws, nbytes = b.workspace(1)
        N.check(L.fks_perturb_step(ctypes.addressof(b.arr), b.n, _seed_u64(seed), sc.ctypes.data, float(value),
                                   N.VALUE_TENSOR if value_is_tensor else N.VALUE_SCALAR, 1 if update else 0,
                                   ws.data_ptr(), nbytes, _stream_handle(b.device)))
        b.finish()
        if leave_generator:
            _leave(b, seed)


def perturb_step_device(specs: Sequence[ParamSpec], seed: int, scales: Sequence[float], value: torch.Tensor,
                        apply: torch.Tensor, stream_mode=None, leave_generator: bool = True) -> None:
    """``perturb_step`` with ``value`` (g) and ``apply`` (bool) as device tensors read by the
    kernels when they run: the restore perturbation always, the update iff ``apply`` --
    no host synchronisation on the losses.  g is rounded to each tensor's dtype like a
    tensor value of ``perturb_step``."""
    specs = list(specs)
    if not specs:
        return
    if len(scales) != len(specs):
        raise ValueError("one scale per tensor")
    b = _Batch(specs, stream_mode)
    if b.device is None:
        return
    if value.device != b.device or apply.device != b.device:
        raise ValueError("value and apply must live on the parameters' device")
    L = N.load()
    sc = np.ascontiguousarray([float(x) for x in scales], dtype=np.float64)
    with torch.cuda.device(b.device):
        dv = torch.stack([value.detach().reshape(()).float(), apply.detach().reshape(()).float()])
        ws, nbytes = b.workspace(1)
        N.check(L.fks_perturb_step_dev(ctypes.addressof(b.arr), b.n, _seed_u64(seed), sc.ctypes.data, dv.data_ptr(),
                                       ws.data_ptr(), nbytes, _stream_handle(b.device)))
        b.finish()
        if leave_generator:
            _leave(b, seed)


def normal_(tensors: Sequence[torch.Tensor], seed: int, frozen: Optional[Sequence[bool]] = None,
            stream_mode=None, leave_generator: bool = True) -> None:
    """Overwrite every tensor with the z the reference draws for it after manual_seed(seed)."""
    specs = [ParamSpec(t, frozen=bool(frozen[i]) if frozen else False) for i, t in enumerate(tensors)]
    if not specs:
        return
    b = _Batch(specs, stream_mode)
    if b.device is None:
        return
    L = N.load()
    with torch.cuda.device(b.device):
        ws, nbytes = b.workspace(1)
        N.check(L.fks_normal(ctypes.addressof(b.arr), b.n, _seed_u64(seed), ws.data_ptr(), nbytes,
                             _stream_handle(b.device)))
        b.finish()
        if leave_generator:
            _leave(b, seed)


def _check_delta(b: _Batch, delta: torch.Tensor) -> None:
    total = sum(sp.tensor.numel() for sp in b.specs)
    if delta.dtype != torch.float32 or not delta.is_contiguous() or delta.numel() != total:
        raise ValueError(f"delta must be a contiguous float32 tensor of {total} elements (the tensors' concatenation)")
    if delta.device != b.device:
        raise ValueError("delta must live on the parameters' device")


def delta_accumulate(specs: Sequence[ParamSpec], seeds: Sequence[int], coefs: Sequence[float],
                     delta: torch.Tensor, stream_mode=None) -> None:
    """Seed-sharded variant (include/fks.h): delta += f32(coef_s) * z_s for every seed in
    order, z_s the reference's stream for the spec list (the call's stream_mode, either
    stream; frozen specs draw, are not accumulated); delta is the f32 concatenation of the
    specs' elements.  Draws nothing from torch's generators (the caller leaves them,
    leave_generators, once the whole list is applied)."""
    if len(seeds) != len(coefs):
        raise ValueError("seeds and coefs differ in length")
    specs = list(specs)
    if not specs or not len(seeds):
        return
    b = _Batch(specs, stream_mode)
    if b.device is None:
        return
    _check_delta(b, delta)
    L = N.load()
    s = np.ascontiguousarray([_seed_u64(x) for x in seeds], dtype=np.uint64)
    c = np.ascontiguousarray([float(x) for x in coefs], dtype=np.float64)
    with torch.cuda.device(b.device):
        ws, nbytes = b.workspace(len(s), delta=True)
        N.check(L.fks_delta_accumulate(ctypes.addressof(b.arr), b.n, s.ctypes.data, c.ctypes.data, len(s),
                                       delta.data_ptr(), ws.data_ptr(), nbytes, _stream_handle(b.device)))


def delta_apply(specs: Sequence[ParamSpec], delta: torch.Tensor, decays: Sequence[float]) -> None:
    """p = dtype(f32(decay_i) * p - delta) per non-frozen spec (one fma, one rounding)."""
    specs = list(specs)
    if not specs:
        return
    if len(decays) != len(specs):
        raise ValueError("one decay per spec")
    b = _Batch(specs, "torch_cpu")  # draws nothing: the stream flag is irrelevant
    if b.device is None:
        return
    _check_delta(b, delta)
    L = N.load()
    d = np.ascontiguousarray([float(x) for x in decays], dtype=np.float64)
    with torch.cuda.device(b.device):
        ws, nbytes = b.workspace(1, delta=True)
        N.check(L.fks_delta_apply(ctypes.addressof(b.arr), b.n, delta.data_ptr(), d.ctypes.data, ws.data_ptr(),
                                  nbytes, _stream_handle(b.device)))
        b.finish()


def shard_range(specs: Sequence[ParamSpec], shard: int, nshards: int, stream_mode=None):
    """What element shard ``shard`` of ``nshards`` owns (fks_shard_census: the clipping
    fks_directional_step_shard launches with).  torch_cpu: the stream words [lo, hi); for
    a list of contiguous tensors laid end to end whose sizes are multiples of 16 (no tail
    recompute words) the words are the elements of their concatenation.  torch_rocm: the
    elements [lo, hi) of the tensors' concatenation (runs of whole Philox rows)."""
    b = _Batch(specs, stream_mode)
    rng = (ctypes.c_int64 * 2)()
    with torch.cuda.device(b.device):
        N.check(N.load().fks_shard_census(ctypes.addressof(b.arr), b.n, int(shard), int(nshards), rng, None))
    return int(rng[0]), int(rng[1])


def stream_length(tensors: Sequence[torch.Tensor]) -> int:
    """32-bit MT19937 words the tensors consume per seed (their z-stream length)."""
    b = _Batch([ParamSpec(t) for t in tensors], "torch_cpu")
    out = ctypes.c_int64(0)
    N.check(N.load().fks_stream_length(ctypes.addressof(b.arr), b.n, ctypes.byref(out)))
    return int(out.value)


class profile:
    """Context manager: device time of every codec kernel launched inside (HIP events)."""

    def __enter__(self):
        N.check(N.load().fks_profile_begin())
        return self

    def __exit__(self, *exc):
        a, j = ctypes.c_double(0), ctypes.c_double(0)
        na, nj = ctypes.c_int64(0), ctypes.c_int64(0)
        N.check(N.load().fks_profile_end(ctypes.byref(a), ctypes.byref(na), ctypes.byref(j), ctypes.byref(nj)))
        self.apply_ms, self.n_apply, self.jump_ms, self.n_jump = a.value, na.value, j.value, nj.value
        return False


def mark_rebound(params) -> None:
    """Record that the reference would have rebound each parameter's ``param.data`` to a
    tensor torch allocated (zo_utils.py:49, optimizer.py:173: every update and perturbation
    assigns a new tensor), which the drop-in's in-place update does not do: the next call's
    first ``wd * p`` then reads that fresh, 16-byte-aligned tensor in the reference, whatever
    the alignment of the buffer here (ParamSpec.fresh, FKS_FRESH; it decides an f16 rounding
    on the torch_rocm stream).  Keyed on the buffer's address: a parameter whose .data the
    caller rebinds starts over."""
    for p in params:
        try:
            p._fks_rebound_ptr = p.data_ptr()
        except (AttributeError, RuntimeError):  # an object that takes no attributes: no record
            pass


def is_rebound(p) -> bool:
    return getattr(p, "_fks_rebound_ptr", None) == p.data_ptr()


def resolve_groups(param_groups: List[dict], lr=None, weight_decay=None) -> List[ParamSpec]:
    """zo_utils.py:43-46: walk the groups in order; lr / weight_decay are re-bound from
    each group only while still None -- so the first group's values stick for all
    later groups ("sticky" semantics)."""
    specs = []
    for group in param_groups:
        weight_decay = group["weight_decay"] if weight_decay is None else weight_decay
        lr = group["lr"] if lr is None else lr
        for p in group["params"]:
            specs.append(ParamSpec(p.data, lr=float(lr) if lr is not None else 0.0,
                                   weight_decay=None if weight_decay is None else float(weight_decay),
                                   fresh=is_rebound(p)))
    return specs


def is_finite_number(x) -> bool:
    try:
        return math.isfinite(float(x))
    except (TypeError, ValueError):
        return False
