"""Compact wire format for the FedKSeed round payloads.

The reference moves two Python objects per round through the FATE federation
(pickled by the transport):

* arbiter -> client, key ``"train_once"`` (fedkseed.py:57-68):
  ``(should_exit, {"seed_candidates": LongTensor[K], "seed_probabilities": f32[K],
  "direction_derivative_sum": dict[int, float] | None})``.  The sums dict is created
  from ``seed_candidates`` in order (fedkseed.py:73-74) and updated in place, so it
  carries all K keys every round, even the zero ones;
* client -> arbiter, key ``"direction_derivative_history"`` (fedkseed.py:128,
  trainer.py:59-66, optimizer.py:189,233): ``dict[int, list[float]]`` with all K seeds
  as keys and one ``g.item()`` per local step appended to the sampled seed's list.

This module encodes both as flat little-endian binary records and decodes them back
to objects equal to the originals -- same key order, same float bits, the same torch
dtypes -- so the receiving ``Trainer``/``ClientTrainer`` code runs unchanged:

* seeds: u32 when every seed is in [0, 2**32) (``build_seed_candidates`` draws there),
  else i64;
* probabilities: the f32 tensor's bytes;
* sums: f64 values only, when the dict's keys are exactly ``seed_candidates`` in order
  (always, for the reference's arbiter); otherwise explicit keys as well;
* history: CSR -- keys, u32 counts, values -- as f32 when every value round-trips
  through f32 bit-exactly (``g.item()`` of a 0-dim f32 tensor always does), else f64.
  When both ends know the round's seed candidates and the history's keys are exactly
  those candidates in order (always, for the reference's optimizer: optimizer.py:189),
  only the seeds with values travel, as (candidate index, count) pairs: S local steps
  cost 8 bytes per distinct sampled seed + 4 per value instead of 8 K + 4 S.  The
  decoder restores the empty lists, so the object is equal to the original.

``WireContext`` wraps a federation context (the duck-typed ``ctxs_range`` / ``guest``
/ ``hosts`` / ``arbiter`` surface fedkseed.py uses) so those two keys travel encoded
and every other key passes through untouched: opt-in, with no change to the trainers.

**The z stream travels with the round.**  The reference draws z where the parameters
live (zo_utils.py:47, optimizer.py:170-172: ``device=param.data.device``), so a party on
a GPU and a party on the CPU apply the same (seed, scalar) list along different
directions -- silently.  A record can carry the stream its
sender draws (``stream_mode``: "torch_cpu" or "torch_rocm", two flag bits) and, for
torch_rocm, the grid cap of the sender's device (``stream_grid``: CUs x (max threads per CU
/ 256), a u32 after the header).  torch draws a tensor of n elements in a grid of
min(ceil(n / 256), cap) blocks and thread idx of it takes elements idx + 256 x grid x (4 j
+ i) (DistributionTemplates.h:50-89), so two GPUs with different caps -- an MI355X in SPX
mode (2,048) and one in a CPX partition (256), or an MI300X (2,432) -- draw different z for
every tensor above 256 x cap / 4 elements: the cap is part of the stream.  The drop-in
``ClientTrainer`` declares its stream into its ``WireContext``, the arbiter's ``Trainer``
rejects a history whose stream differs from the others' (``StreamMismatchError``) and
declares the federation's stream into its own records, and a client rejects a
"train_once" whose declared stream differs from its own.  Untagged records (a reference
party) decode as before.

Host-side logic only; it touches no parameters and no device.
"""
import struct
from typing import Dict, List, Mapping, Optional, Sequence, Tuple

import numpy as np
import torch

MAGIC = b"FKSW"
VERSION = 1
KIND_TRAIN_ONCE = 1
KIND_HISTORY = 2

# train_once flags
_F_EXIT = 1 << 0
_F_SEEDS_I64 = 1 << 1
_F_HAS_SUMS = 1 << 2
_F_SUM_KEYS = 1 << 3      # sums carry explicit keys (order or key set differs from the seeds)
_F_HAS_PROBS = 1 << 4
# history flags
_F_KEYS_I64 = 1 << 1
_F_VALUES_F64 = 1 << 2
_F_SPARSE = 1 << 3        # keys = the candidates: only (index, count) of non-empty lists
# both kinds: the sender's z stream (bits 8-9, clear of every other flag)
_F_STREAM_TAGGED = 1 << 8
_F_STREAM_ROCM = 1 << 9
_F_STREAM_GRID = 1 << 10  # a u32 grid cap follows the header (torch_rocm only)
_F_STREAM_LIBM = 1 << 11  # torch_cpu with the libm flavour of fp32 z (codec.stream_identity)
STREAMS = ("torch_cpu", "torch_cpu_libm", "torch_rocm")
_GRID = struct.Struct("<I")

_HEADER = struct.Struct("<4sBBHQ")  # magic, version, kind, flags, count
_U32_MAX = 2 ** 32


class WireFormatError(ValueError):
    """A buffer that is not a valid FedKSeed wire record."""


class StreamMismatchError(RuntimeError):
    """Two parties of one federation draw different z streams (module docstring)."""


class History(dict):
    """A decoded ``direction_derivative_history``: the dict itself (equal to the
    original), plus the ``stream_mode`` its sender declared (None if untagged)."""

    stream_mode: Optional[str] = None
    stream_grid: Optional[int] = None


def _stream_flags(stream_mode: Optional[str], stream_grid: Optional[int] = None) -> int:
    if stream_mode is None:
        if stream_grid is not None:
            raise WireFormatError("a stream_grid needs a stream_mode")
        return 0
    if stream_mode not in STREAMS:
        raise WireFormatError(f"stream_mode must be one of {STREAMS} or None, not {stream_mode!r}")
    if stream_grid is not None:
        if stream_mode != "torch_rocm":
            raise WireFormatError("stream_grid belongs to the torch_rocm stream only")
        if not 0 < int(stream_grid) < 2 ** 32:
            raise WireFormatError(f"stream_grid must be a positive u32, not {stream_grid!r}")
    return (_F_STREAM_TAGGED | (_F_STREAM_ROCM if stream_mode == "torch_rocm" else 0)
            | (_F_STREAM_LIBM if stream_mode == "torch_cpu_libm" else 0)
            | (_F_STREAM_GRID if stream_grid is not None else 0))


def _stream_of(flags: int) -> Optional[str]:
    if not flags & _F_STREAM_TAGGED:
        if flags & (_F_STREAM_ROCM | _F_STREAM_LIBM | _F_STREAM_GRID):
            raise WireFormatError("stream bits on an untagged record")
        return None
    if flags & _F_STREAM_ROCM:
        if flags & _F_STREAM_LIBM:
            raise WireFormatError("the libm flavour belongs to the torch_cpu stream only")
        return "torch_rocm"
    return "torch_cpu_libm" if flags & _F_STREAM_LIBM else "torch_cpu"


def _grid_bytes(stream_grid: Optional[int]) -> bytes:
    return b"" if stream_grid is None else _GRID.pack(int(stream_grid))


def _read_grid(buf: memoryview, flags: int, off: int) -> Tuple[Optional[int], int]:
    if not flags & _F_STREAM_GRID:
        return None, off
    if not flags & _F_STREAM_ROCM:
        raise WireFormatError("grid cap on a record that is not torch_rocm")
    (g,), off = _read(buf, off, "<u4", 1)
    return int(g), off


def describe_stream(mode: Optional[str], grid: Optional[int] = None) -> str:
    return f"{mode} (grid cap {grid})" if mode == "torch_rocm" and grid is not None else str(mode)


def check_stream(expected: Optional[str], got: Optional[str], what: str, expected_grid: Optional[int] = None,
                 got_grid: Optional[int] = None) -> None:
    """Raise StreamMismatchError when both streams are known and differ: another generator,
    or torch_rocm on devices of different grid caps (when both caps are known)."""
    if expected is None or got is None:
        return
    if expected != got or (expected == "torch_rocm" and expected_grid is not None and got_grid is not None
                           and int(expected_grid) != int(got_grid)):
        raise StreamMismatchError(
            f"{what} draws the {describe_stream(got, got_grid)} z stream, this federation draws "
            f"{describe_stream(expected, expected_grid)}: the parties would apply the same (seed, scalar) list "
            "along different directions (zo_utils.py:47 draws on the parameters' device, in a grid of at most "
            "CUs x threads per CU / 256 blocks; on the CPU generator, fp32 z follows ATen's CPU capability: "
            "torch_cpu_libm is ATEN_CPU_CAPABILITY=default); set FKS_STREAM_MODE / codec.set_stream_mode alike on "
            "every party, train every torch_rocm party on devices of one CU count and partition mode, and every "
            "torch_cpu party under one CPU capability (FKS_CPU_FP32_FLAVOUR)")


def _keys_array(keys: Sequence[int]) -> Tuple[np.ndarray, bool]:
    a = np.asarray(keys, dtype=np.int64) if len(keys) else np.zeros(0, np.int64)
    if a.size and (a.min() < 0 or a.max() >= _U32_MAX):
        return a, True
    return a.astype("<u4"), False


def _read(buf: memoryview, off: int, dtype: str, n: int) -> Tuple[np.ndarray, int]:
    dt = np.dtype(dtype)
    end = off + dt.itemsize * n
    if end > len(buf):
        raise WireFormatError(f"truncated record: need {end} bytes, have {len(buf)}")
    return np.frombuffer(buf[off:end], dtype=dt, count=n), end


def _header(buf, kind: int) -> Tuple[memoryview, int, int]:
    buf = memoryview(buf).cast("B")
    if len(buf) < _HEADER.size:
        raise WireFormatError("truncated header")
    magic, version, k, flags, count = _HEADER.unpack_from(buf, 0)
    if magic != MAGIC or version != VERSION:
        raise WireFormatError(f"bad magic/version {magic!r}/{version}")
    if k != kind:
        raise WireFormatError(f"record kind {k}, expected {kind}")
    return buf, flags, count


def encode_train_once(message: Tuple[bool, Mapping], stream_mode: Optional[str] = None,
                      stream_grid: Optional[int] = None) -> bytes:
    """``(should_exit, kwargs)`` of the arbiter's "train_once" put (fedkseed.py:66-68);
    ``stream_mode`` / ``stream_grid``: the federation's z stream, if the arbiter declares one."""
    should_exit, kw = message
    seeds = kw["seed_candidates"]
    seeds_np = seeds.detach().cpu().numpy() if torch.is_tensor(seeds) else np.asarray(seeds)
    seeds_arr, seeds_i64 = _keys_array(seeds_np.reshape(-1).tolist())
    k = seeds_arr.size
    probs = kw.get("seed_probabilities")
    sums: Optional[Mapping[int, float]] = kw.get("direction_derivative_sum")

    flags = ((_F_EXIT if should_exit else 0) | (_F_SEEDS_I64 if seeds_i64 else 0)
             | _stream_flags(stream_mode, stream_grid))
    kdt = "<i8" if seeds_i64 else "<u4"
    parts = [_grid_bytes(stream_grid), seeds_arr.astype(kdt).tobytes()]
    if probs is not None:
        p = probs.detach().cpu() if torch.is_tensor(probs) else torch.as_tensor(probs)
        if p.dtype != torch.float32 or p.numel() != k:
            raise WireFormatError(f"seed_probabilities must be float32[{k}], got {p.dtype}[{p.numel()}]")
        flags |= _F_HAS_PROBS
        parts.append(p.contiguous().numpy().astype("<f4").tobytes())
    if sums is not None:
        flags |= _F_HAS_SUMS
        keys = [int(s) for s in sums.keys()]
        vals = np.fromiter((float(v) for v in sums.values()), dtype="<f8", count=len(keys))
        if keys != seeds_arr.astype(np.int64).tolist():
            flags |= _F_SUM_KEYS
            karr, ki64 = _keys_array(keys)
            if ki64 and not seeds_i64:
                raise WireFormatError("sum keys outside [0, 2**32) with u32 seeds")
            parts.append(struct.pack("<Q", len(keys)))
            parts.append(karr.astype(kdt).tobytes())
        parts.append(vals.tobytes())
    return _HEADER.pack(MAGIC, VERSION, KIND_TRAIN_ONCE, flags, k) + b"".join(parts)


def decode_train_once(buf) -> Tuple[bool, Dict]:
    """Inverse of ``encode_train_once``: seeds as ``torch.long``, probabilities as
    ``torch.float32``, sums as a ``dict[int, float]`` in the encoded key order; a tagged
    record adds ``"stream_mode"`` (and ``"stream_grid"``) to the kwargs (the reference reads
    only its three keys)."""
    buf, flags, k = _header(buf, KIND_TRAIN_ONCE)
    grid, off = _read_grid(buf, flags, _HEADER.size)
    kdt = "<i8" if flags & _F_SEEDS_I64 else "<u4"
    seeds, off = _read(buf, off, kdt, k)
    seed_t = torch.from_numpy(seeds.astype(np.int64))
    probs = None
    if flags & _F_HAS_PROBS:
        p, off = _read(buf, off, "<f4", k)
        probs = torch.from_numpy(p.astype(np.float32))
    sums = None
    if flags & _F_HAS_SUMS:
        if flags & _F_SUM_KEYS:
            (n,), _ = _read(buf, off, "<u8", 1)
            keys, off = _read(buf, off + 8, kdt, int(n))
            keys = keys.astype(np.int64).tolist()
        else:
            keys = seed_t.tolist()
        vals, off = _read(buf, off, "<f8", len(keys))
        sums = dict(zip(keys, vals.tolist()))
    if off != len(buf):
        raise WireFormatError(f"{len(buf) - off} trailing bytes")
    kw = {"seed_candidates": seed_t, "seed_probabilities": probs, "direction_derivative_sum": sums}
    if _stream_of(flags) is not None:
        kw["stream_mode"] = _stream_of(flags)
        if grid is not None:
            kw["stream_grid"] = grid
    return bool(flags & _F_EXIT), kw


def _values_block(flat: np.ndarray) -> Tuple[int, bytes]:
    with np.errstate(over="ignore", invalid="ignore"):
        as32 = flat.astype("<f4")
    lossless = np.array_equal(as32.astype("<f8").view("<u8"), flat.view("<u8"))
    return (0 if lossless else _F_VALUES_F64), (as32 if lossless else flat).tobytes()


def encode_history(history: Mapping[int, Sequence[float]], candidates: Optional[Sequence[int]] = None,
                   stream_mode: Optional[str] = None, stream_grid: Optional[int] = None) -> bytes:
    """A client's ``direction_derivative_history`` (dict seed -> list of g values).
    ``candidates``: the round's seed candidates, known to both ends -- enables the
    sparse form when the history's keys are exactly these seeds in order.
    ``stream_mode`` / ``stream_grid``: the z stream the client drew its steps from (tags the
    record)."""
    sflags = _stream_flags(stream_mode, stream_grid)
    gbytes = _grid_bytes(stream_grid)
    keys = [int(s) for s in history.keys()]
    counts = np.fromiter((len(v) for v in history.values()), dtype="<u4", count=len(keys))
    flat = np.fromiter((float(x) for v in history.values() for x in v), dtype="<f8",
                       count=int(counts.sum()))
    vflag, vbytes = _values_block(flat)
    if candidates is not None and keys == [int(c) for c in candidates]:
        nz = np.nonzero(counts)[0]
        return (_HEADER.pack(MAGIC, VERSION, KIND_HISTORY, _F_SPARSE | vflag | sflags, len(nz)) + gbytes
                + nz.astype("<u4").tobytes() + counts[nz].tobytes() + vbytes)
    karr, ki64 = _keys_array(keys)
    flags = (_F_KEYS_I64 if ki64 else 0) | vflag | sflags
    return (_HEADER.pack(MAGIC, VERSION, KIND_HISTORY, flags, len(keys)) + gbytes
            + karr.astype("<i8" if ki64 else "<u4").tobytes() + counts.tobytes() + vbytes)


def decode_history(buf, candidates: Optional[Sequence[int]] = None) -> Dict[int, List[float]]:
    """Inverse of ``encode_history``; a tagged record decodes to a ``History`` carrying
    the sender's ``stream_mode`` and ``stream_grid``."""
    buf, flags, n = _header(buf, KIND_HISTORY)
    grid, off = _read_grid(buf, flags, _HEADER.size)
    if flags & _F_SPARSE:
        if candidates is None:
            raise WireFormatError("sparse history record needs the round's seed candidates")
        idx, off = _read(buf, off, "<u4", n)
    else:
        keys, off = _read(buf, off, "<i8" if flags & _F_KEYS_I64 else "<u4", n)
    counts, off = _read(buf, off, "<u4", n)
    total = int(counts.astype(np.int64).sum())
    vals, off = _read(buf, off, "<f8" if flags & _F_VALUES_F64 else "<f4", total)
    if off != len(buf):
        raise WireFormatError(f"{len(buf) - off} trailing bytes")
    flat = vals.astype(np.float64).tolist()
    stream = _stream_of(flags)
    out: Dict[int, List[float]] = {} if stream is None else History()
    if stream is not None:
        out.stream_mode = stream
        out.stream_grid = grid
    pos = 0
    if flags & _F_SPARSE:
        cand = [int(c) for c in candidates]
        if n and int(idx.max()) >= len(cand):
            raise WireFormatError("candidate index out of range")
        got = {}
        for i, c in zip(idx.tolist(), counts.tolist()):
            got[i] = flat[pos:pos + c]
            pos += c
        out.update((s, got.get(i, [])) for i, s in enumerate(cand))
        return out
    for key, c in zip(keys.astype(np.int64).tolist(), counts.tolist()):
        out[key] = flat[pos:pos + c]
        pos += c
    return out


class _WireParty:
    """One federation party (``ctx.guest`` / a host / ``ctx.arbiter``) whose FedKSeed
    keys are encoded on ``put`` and decoded on ``get``.  The link remembers the seed
    candidates of its last "train_once" (either direction) for the sparse history, and
    tags what it sends with the stream its context declared."""

    def __init__(self, party, state, role):
        self._party, self._state, self._role = party, state, role

    def put(self, key, value):
        stream, grid = self._state.get(_STREAM_KEY), self._state.get(_GRID_KEY)
        if key == "train_once":
            self._state[self._role] = [int(s) for s in value[1]["seed_candidates"]]
            value = encode_train_once(value, stream, grid)
        elif key == "direction_derivative_history":
            value = encode_history(value, self._state.get(self._role), stream, grid)
        return self._party.put(key, value)

    def get(self, key):
        value = self._party.get(key)
        if not isinstance(value, (bytes, bytearray, memoryview)):
            return value
        if key == "train_once":
            value = decode_train_once(value)
            self._state[self._role] = value[1]["seed_candidates"].tolist()
            check_stream(self._state.get(_STREAM_KEY), value[1].get("stream_mode"), "the arbiter",
                         self._state.get(_GRID_KEY), value[1].get("stream_grid"))
        elif key == "direction_derivative_history":
            value = decode_history(value, self._state.get(self._role))
        return value

    def __getattr__(self, name):
        return getattr(self._party, name)


_STREAM_KEY = object()  # WireContext state: the z stream this party declared
_GRID_KEY = object()    # ... and its torch_rocm grid cap


class WireContext:
    """Wraps a federation context: ``ctxs_range`` yields wrapped sub-contexts whose
    ``guest``, ``hosts`` and ``arbiter`` parties move the FedKSeed round payloads in
    the compact format.  Both ends of a link must be wrapped.  ``stream_mode``: the z
    stream this party draws ("torch_cpu" / "torch_rocm"), and ``stream_grid`` its torch_rocm
    grid cap, carried by every record it sends; the drop-in ClientTrainer declares its own
    (``declare_stream_mode``)."""

    def __init__(self, ctx, _state=None, stream_mode: Optional[str] = None, stream_grid: Optional[int] = None):
        self._ctx = ctx
        self._state = {} if _state is None else _state  # role -> seed candidates of the link
        if stream_mode is not None:
            self.declare_stream_mode(stream_mode, stream_grid)

    def declare_stream_mode(self, stream_mode: Optional[str], stream_grid: Optional[int] = None) -> None:
        _stream_flags(stream_mode, stream_grid)  # validates
        check_stream(self._state.get(_STREAM_KEY), stream_mode, "this party", self._state.get(_GRID_KEY), stream_grid)
        self._state[_STREAM_KEY] = stream_mode
        if stream_grid is not None or stream_mode != "torch_rocm":
            self._state[_GRID_KEY] = stream_grid

    @property
    def stream_mode(self) -> Optional[str]:
        return self._state.get(_STREAM_KEY)

    @property
    def stream_grid(self) -> Optional[int]:
        return self._state.get(_GRID_KEY)

    def ctxs_range(self, n):
        for i, sub in self._ctx.ctxs_range(n):
            yield i, WireContext(sub, self._state)

    @property
    def guest(self):
        return _WireParty(self._ctx.guest, self._state, "guest")

    @property
    def hosts(self):
        hosts = getattr(self._ctx, "hosts", None)
        return [_WireParty(h, self._state, f"host{i}") for i, h in enumerate(hosts)] if hosts else hosts

    @property
    def arbiter(self):
        return _WireParty(self._ctx.arbiter, self._state, "arbiter")

    def __getattr__(self, name):
        return getattr(self._ctx, name)
