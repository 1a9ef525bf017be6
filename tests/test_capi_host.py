"""CPU-side checks of the product library (no device needed).

* libfks.so loads and exports every symbol include/fks.h declares;
* the host GF(2) jump-ahead reproduces the oracle's sequential MT19937 state at
  arbitrary stream blocks (the math every device jump depends on);
* the bf16 Box-Muller tables are exactly the reduced-precision values torch's
  normal_fill_16<BFloat16> computes (checked through the pinned oracle streams);
* the stream layout (words consumed per tensor, tail recompute, serial path with
  its cached sample) matches the oracle generator's consumption.
"""
import ctypes
import os
import re

import numpy as np
import pytest

from oracle import fks_oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _lib():
    from fate_llm.algo.fedkseed import _native
    return _native, _native.load()


def test_header_symbols_exported():
    N, L = _lib()
    with open(os.path.join(ROOT, "include", "fks.h")) as f:
        hdr = f.read()
    declared = set(re.findall(r"^\s*(?:int|int32_t|const char\*)\s+(fks_\w+)\s*\(", hdr, re.M))
    assert declared, "no declarations parsed"
    assert declared == set(N.EXPORTED), (declared ^ set(N.EXPORTED))
    for name in declared:
        assert hasattr(L, name), name
    assert L.fks_abi_version() == N.ABI_VERSION
    assert L.fks_build_target() == b"gfx950"
    assert re.fullmatch(r"[0-9a-f]{16}", N.build_id())
    # the library in the tree was built from the sources beside it (__graft_entry__.ensure_built)
    import __graft_entry__
    assert N.source_id() == __graft_entry__.source_id()


def test_fks_tensor_layout_matches_header():
    N, _ = _lib()
    assert ctypes.sizeof(N.FksTensor) == 32
    assert N.FksTensor.lr.offset == 24 and N.FksTensor.wd.offset == 28


@pytest.mark.parametrize("seed,block", [(0, 1), (1, 2), (42, 17), (2**32 - 1, 1000), (12345, 31337),
                                        (2**40 + 7, 5), (3141592653, 4096)])
def test_host_jump_window_matches_sequential_mt(seed, block):
    _, L = _lib()
    out = np.zeros(624, np.uint32)
    assert L.fks_host_jump_window(seed, block, out.ctypes.data) == 0
    g = O.Generator(seed)
    g.u32(624 * block)  # after drawing `block` whole blocks the state array is the window
    assert np.array_equal(out, g.state_words())


def test_bf16_tables_reproduce_pinned_stream(golden):
    """z = round_bf16(R[a] * C[b]) (+0) over the whole pinned 2^20 bf16 stream."""
    _, L = _lib()
    r = np.zeros(256, np.float32)
    c = np.zeros(256, np.float32)
    s = np.zeros(256, np.float32)
    assert L.fks_host_tables(1, r.ctypes.data, c.ctypes.data, s.ctypes.data, 256) == 0
    ref = golden("normal_streams.npz")["long_bfloat16"]
    u = O.Generator(2024).u32(ref.size) & 0xFF
    blk = u.reshape(-1, 16)
    a, b = blk[:, :8].reshape(-1), blk[:, 8:].reshape(-1)

    def rne(x):
        bits = x.astype(np.float32).view(np.uint32).astype(np.uint64)
        return ((bits + 0x7FFF + ((bits >> 16) & 1)) >> 16).astype(np.uint16)

    zc = rne((r[a] * c[b]) + np.float32(0.0))
    zs = rne((r[a] * s[b]) + np.float32(0.0))
    got = np.empty((blk.shape[0], 16), np.uint16)
    got[:, :8] = zc.reshape(-1, 8)
    got[:, 8:] = zs.reshape(-1, 8)
    assert np.array_equal(got.reshape(-1), ref)


def test_f16_tables_reproduce_pinned_stream(golden):
    """z = round_f16(R[a] * C[b]) (+0) over the pinned 2^18 f16 stream (11-bit uniforms)."""
    _, L = _lib()
    r = np.zeros(2048, np.float32)
    c = np.zeros(2048, np.float32)
    s = np.zeros(2048, np.float32)
    assert L.fks_host_tables(2, r.ctypes.data, c.ctypes.data, s.ctypes.data, 2048) == 0
    ref = golden("normal_streams.npz")["long_float16"]
    u = O.Generator(2024).u32(ref.size) & 0x7FF
    blk = u.reshape(-1, 16)
    a, b = blk[:, :8].reshape(-1), blk[:, 8:].reshape(-1)
    zc = ((r[a] * c[b]) + np.float32(0.0)).astype(np.float16).view(np.uint16)
    zs = ((r[a] * s[b]) + np.float32(0.0)).astype(np.float16).view(np.uint16)
    got = np.empty((blk.shape[0], 16), np.uint16)
    got[:, :8] = zc.reshape(-1, 8)
    got[:, 8:] = zs.reshape(-1, 8)
    assert np.array_equal(got.reshape(-1), ref)


def test_tables_reject_bad_args():
    _, L = _lib()
    buf = np.zeros(16, np.float32)
    assert L.fks_host_tables(0, buf.ctypes.data, buf.ctypes.data, buf.ctypes.data, 16) < 0
    assert L.fks_last_error()


@pytest.mark.parametrize("shapes", [[16, 32, 624], [37, 5, 3, 16], [5, 3, 1, 7, 100], [1, 1, 1, 15, 17]])
def test_stream_length_matches_oracle(shapes):
    N, L = _lib()
    arr = (N.FksTensor * len(shapes))()
    for i, n in enumerate(shapes):
        arr[i].data = 16 if n else None  # never dereferenced
        arr[i].numel = n
        arr[i].dtype = N.BF16
    words = ctypes.c_int64(0)
    assert L.fks_stream_length(ctypes.addressof(arr), len(shapes), ctypes.byref(words)) == 0
    # oracle: count draws by running the same sequence on an instrumented generator
    g = O.Generator(11)
    for n in shapes:
        g.normal(n, O.BF16)
    h = O.Generator(11)
    h.u32(words.value)
    assert np.array_equal(g.state_words(), h.state_words()) and g.left_next() == h.left_next()


def test_invalid_inputs_rejected():
    N, L = _lib()
    arr = (N.FksTensor * 1)()
    arr[0].data = 3  # misaligned for bf16
    arr[0].numel = 32
    arr[0].dtype = N.BF16
    nbytes = ctypes.c_size_t(0)
    assert L.fks_workspace_size(ctypes.addressof(arr), 1, 1, ctypes.byref(nbytes)) < 0
    assert b"misaligned" in L.fks_last_error()
    arr[0].data = 16
    arr[0].dtype = 7
    assert L.fks_workspace_size(ctypes.addressof(arr), 1, 1, ctypes.byref(nbytes)) < 0
    # FKS_LIBM is a flavour of the CPU generator's stream, one per call
    arr[0].dtype = N.F32
    arr[0].flags = N.LIBM | N.STREAM_ROCM
    assert L.fks_workspace_size(ctypes.addressof(arr), 1, 1, ctypes.byref(nbytes)) < 0
    assert b"flavour" in L.fks_last_error()
    two = (N.FksTensor * 2)()
    for i in range(2):
        two[i].data = 16
        two[i].numel = 32
        two[i].dtype = N.F32
    two[0].flags = N.LIBM
    assert L.fks_workspace_size(ctypes.addressof(two), 2, 1, ctypes.byref(nbytes)) < 0
    assert b"same z stream" in L.fks_last_error()


_TORCH_DT = {0: "float32", 1: "bfloat16", 2: "float16"}


@pytest.mark.parametrize("layout", [
    [(3, 0), (20, 0)],                         # serial pair cached, then a tail recompute
    [(5, 1), (7, 2), (1000, 1), (1, 0)],       # caches consumed and refilled across tensors
    [(4096, 0), (5, 0)],
    [(16, 1)],                                 # no serial draw: no cached value
    [(100000, 0), (3, 1), (17, 2)],
    [(0, 0)],                                  # draws nothing: the freshly seeded state
    [(624 * 3, 1)],                            # ends exactly on a block boundary
    [(3 * 10**7 + 5, 0), (2, 1)],              # many blocks (a jump far into the stream)
])
@pytest.mark.parametrize("seed", [0, 12345, 2**40 + 7])
def test_cpu_generator_end_matches_torch(layout, seed):
    """fks_cpu_generator_end, assembled into torch's CPU generator state by
    codec.cpu_generator_state, equals torch's own CPU generator after torch.manual_seed(seed)
    and torch.normal draws of the same sizes and dtypes (zo_utils.py:42,47 on CPU tensors):
    byte for byte, and the next draws agree."""
    import torch

    from fate_llm.algo.fedkseed import codec
    N, _ = _lib()
    arr = (N.FksTensor * len(layout))()
    for i, (n, d) in enumerate(layout):
        arr[i].data = 16 if n else None  # never dereferenced
        arr[i].numel = n
        arr[i].dtype = d
    ours = codec.cpu_generator_state(arr, len(layout), seed)
    torch.manual_seed(seed)
    for n, d in layout:
        torch.normal(mean=0, std=1, size=(n,), dtype=getattr(torch, _TORCH_DT[d]))
    ref = torch.get_rng_state()
    assert torch.equal(ours, ref)
    follow = torch.randn(7, dtype=torch.float64), torch.randint(0, 2**31, (5,)), torch.normal(0, 1, (3,))
    torch.set_rng_state(ours)
    again = torch.randn(7, dtype=torch.float64), torch.randint(0, 2**31, (5,)), torch.normal(0, 1, (3,))
    assert all(torch.equal(a, b) for a, b in zip(follow, again))


@pytest.mark.parametrize("shapes", [[(600_000_000, 0)], [(1_100_000_003, 0), (5, 1)], [(2**30 + 4099, 2), (2**29, 0)]])
@pytest.mark.parametrize("nshards", [1, 3, 8])
def test_torch_rocm_pieces_tile_the_tensors(shapes, nshards):
    """Host geometry of the torch_rocm stream (fks_shard_census, no device: the grid cap
    falls back to an MI355X's 2,048) for tensors past 2^31 bytes, drawn by torch in
    32-bit-indexable pieces (phx_geometry): element shards are contiguous runs that tile the
    concatenation, and every element of every tensor is written exactly once."""
    N, L = _lib()
    arr = (N.FksTensor * len(shapes))()
    for i, (n, d) in enumerate(shapes):
        arr[i].data = 4096
        arr[i].numel = n
        arr[i].dtype = d
        arr[i].flags = N.STREAM_ROCM
    total = [0] * len(shapes)
    lo_expected = 0
    for r in range(nshards):
        rng = (ctypes.c_int64 * 2)()
        wr = (ctypes.c_int64 * len(shapes))()
        assert L.fks_shard_census(ctypes.addressof(arr), len(shapes), r, nshards, rng, wr) == 0, L.fks_last_error()
        assert rng[0] == lo_expected and rng[1] >= rng[0]
        lo_expected = rng[1]
        total = [a + b for a, b in zip(total, wr)]
    assert lo_expected == sum(n for n, _ in shapes)
    assert total == [n for n, _ in shapes]
