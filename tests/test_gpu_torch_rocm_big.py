"""torch_rocm draws of tensors past 2^31 bytes, and the seed-sharded variant on that stream.

**Past 2^31 bytes.** torch's distribution_nullary_kernel (ATen/native/cuda/
DistributionTemplates.h:111-133) first reserves the whole tensor's Philox offset
increment, then -- when the iterator cannot use 32-bit indexing (largest byte offset past
INT32_MAX) -- draws each piece TensorIterator::with_32bit_indexing yields (halves split until
they fit: first floor(n / 2) elements then the rest, recursively) as a call of its own, with
its own launch geometry and its own reservation; the intermediate halves reserve nothing
(the 4.4 GB case, four pieces, pins that).  fks_capi.cpp phx_geometry restates that: each piece is a table
entry of its own.  Oracle: torch.normal(device="cuda") itself, and the reference's update
expression as torch ops on the device (oracle/torch_replica.py).  Bar: bit-exact, and the
device generator's offset after the call equal to torch's.

**Seed-sharded (C3) on the default stream.** fks_delta_accumulate draws the torch_rocm
stream: delta = fmaf(f32(c_k), z_k, delta) per seed in order, against the same f32
operation order applied to torch.normal(device="cuda") draws (fmaf emulated exactly with
numpy: the f32 x f32 product is exact in f64, and the f64 sum is corrected where it lands
on an f32 rounding midpoint).  And reconstruct_seed_sharded_ with FKS_STREAM_MODE unset
(the drop-in default "auto": torch_rocm on the GPU)."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from oracle import torch_replica as R
from test_gpu_parity import _dev

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bits(t):
    return t.view(torch.int16) if t.element_size() == 2 else t.view(torch.int32)


def _assert_same(got, want, what):
    if not torch.equal(_bits(got), _bits(want)):
        bad = (_bits(got) != _bits(want)).nonzero()
        raise AssertionError(f"{what}: {bad.shape[0]} of {got.numel()} elements differ, first at {bad[0].tolist()}")


def _pieces(n, es):
    """The 32-bit-indexable pieces torch draws a tensor of n elements of es bytes in."""
    if n <= 2**31 - 1 and 1 + (n - 1) * es <= 2**31 - 1:
        return [n]
    return _pieces(n // 2, es) + _pieces(n - n // 2, es)


# fp32: 2.4 GB (two pieces) and 4.4 GB (four pieces of unequal sizes); f16: 2.1 GB
BIG = [("float32", 600_000_000), ("float32", 1_100_000_003), ("float16", 2**30 + 4099)]


@pytest.mark.parametrize("dtype,n", BIG)
def test_normal_past_2gb_matches_torch(dtype, n):
    from fate_llm.algo.fedkseed import codec
    dev = _dev()
    dt = getattr(torch, dtype)
    es = torch.empty((), dtype=dt).element_size()
    assert len(_pieces(n, es)) >= 2
    shapes = [(1000,), (n,), (5000,)]  # the tensor after the big one checks its offset accounting
    for seed in (7, 2**40 + 3):
        torch.manual_seed(seed)
        want = [torch.normal(mean=0, std=1, size=s, device=dev, dtype=dt) for s in shapes]
        want_state = torch.cuda.get_rng_state(dev)
        got = [torch.empty(s, device=dev, dtype=dt) for s in shapes]
        torch.manual_seed(0)
        codec.normal_(got, seed, stream_mode="torch_rocm")
        torch.cuda.synchronize()
        assert torch.equal(torch.cuda.get_rng_state(dev), want_state), "device generator offset"
        for s, g, w in zip(shapes, got, want):
            _assert_same(g, w, f"{dtype} seed {seed} shape {s}")
        del want, got
        torch.cuda.empty_cache()


@pytest.mark.parametrize("dtype,n", [BIG[0], BIG[2]])
def test_reconstruct_past_2gb_matches_torch_ops(dtype, n):
    """K = 3 through the torch_rocm update chain on a list with one >2^31-byte tensor, vs
    the reference's loop (zo_utils.py:42-52) as torch ops on the device; f16 includes the
    per-piece vectorized / unrolled rounding rule of torch's elementwise kernels (each
    32-bit piece is its own launch), at wd 0.01."""
    from fate_llm.algo.fedkseed import codec
    dev = _dev()
    dt = getattr(torch, dtype)
    g = torch.Generator().manual_seed(1)
    small = (torch.randn(3000, generator=g) * 0.02).to(torch.bfloat16).to(dev)
    big = torch.empty(n, dtype=dt, device=dev)
    big.normal_(0.0, 0.02, generator=torch.Generator(device=dev).manual_seed(2))
    ref = [big.clone(), small.clone()]
    seeds, vals = [11, 2**33 + 1, 5], [3.5, -12.0, 0.75]
    R.reconstruct(ref, seeds, vals, 1e-3, 0.01)
    want_state = torch.cuda.get_rng_state(dev)
    specs = [codec.ParamSpec(big, lr=1e-3, weight_decay=0.01), codec.ParamSpec(small, lr=1e-3, weight_decay=0.01)]
    codec.directional_step(specs, seeds, vals, stream_mode="torch_rocm")
    torch.cuda.synchronize()
    assert torch.equal(torch.cuda.get_rng_state(dev), want_state)
    _assert_same(big, ref[0], f"{dtype} big")
    _assert_same(small, ref[1], "bf16 small")


def _fma32(c, z, d):
    """Exact fmaf(c, z, d) over f32 numpy arrays (c a scalar): p = c z is exact in f64, s =
    RN64(p + d) with its TwoSum error e (p + d = s + e exactly); RN32(s) is RN32(p + d)
    unless s is an f32 rounding midpoint and e != 0, where the exact sum lies on e's side."""
    p = np.float64(np.float32(c)) * np.asarray(z, np.float32).astype(np.float64)
    d64 = np.asarray(d, np.float32).astype(np.float64)
    s = p + d64
    bb = s - p
    e = (p - (s - bb)) + (d64 - bb)
    r = s.astype(np.float32)
    r64 = r.astype(np.float64)
    up = np.nextafter(r, np.float32(np.inf))
    dn = np.nextafter(r, np.float32(-np.inf))
    out = r.copy()
    fix_up = (s == (r64 + up.astype(np.float64)) / 2) & (e > 0)  # s midway above r, exact sum beyond it
    fix_dn = (s == (r64 + dn.astype(np.float64)) / 2) & (e < 0)
    out[fix_up] = up[fix_up]
    out[fix_dn] = dn[fix_dn]
    return out


def test_fma32_emulation_is_exact():
    """The checker itself: equal to libm's fmaf on crafted midpoint cases and random data."""
    import ctypes
    libm = ctypes.CDLL("libm.so.6")
    libm.fmaf.restype = ctypes.c_float
    libm.fmaf.argtypes = [ctypes.c_float] * 3
    rng = np.random.default_rng(0)
    z = rng.standard_normal(20000).astype(np.float32)
    d = (rng.standard_normal(20000) * 1e-3).astype(np.float32)
    d[:5000] = (rng.standard_normal(5000) * 1e6).astype(np.float32)
    c = np.float32(1.2345e-4)
    # midpoints: d = 1 and c z = 2^-24 +- tiny
    z[-4:] = np.float32(1.0)
    d[-4:] = np.float32(1.0)
    for c_ in (c, np.float32(2.0 ** -24), np.float32(2.0 ** -24 * (1 + 2.0 ** -20)), np.float32(-(2.0 ** -25))):
        got = _fma32(c_, z, d)
        want = np.array([libm.fmaf(float(c_), float(a), float(b)) for a, b in zip(z, d)], dtype=np.float32)
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


@pytest.mark.parametrize("dtype", ["float32", "bfloat16", "float16"])
@pytest.mark.parametrize("k", [1, 33])
def test_delta_accumulate_torch_rocm_matches_device_draws(dtype, k):
    from fate_llm.algo.fedkseed import codec
    dev = _dev()
    dt = getattr(torch, dtype)
    shapes = [4096, 1000, 3, 700_001, 7, 65536]
    g = torch.Generator().manual_seed(9)
    ts = [torch.zeros(n, dtype=dt, device=dev) for n in shapes]
    frozen = [i == 2 for i in range(len(ts))]  # draws, not accumulated
    seeds = torch.randint(0, 2**32, (k,), generator=g).tolist()
    coefs = (torch.randn(k, generator=g, dtype=torch.float64) * 1e-4).tolist()
    total = sum(shapes)
    delta = torch.zeros(total, dtype=torch.float32, device=dev)
    delta[::5] = 0.125
    ref = delta.cpu().numpy().copy()
    codec.delta_accumulate([codec.ParamSpec(t, frozen=f) for t, f in zip(ts, frozen)], seeds, coefs, delta,
                           stream_mode="torch_rocm")
    torch.cuda.synchronize()
    for s, c in zip(seeds, coefs):
        torch.manual_seed(s)
        off = 0
        for n, f in zip(shapes, frozen):
            z = torch.normal(mean=0, std=1, size=(n,), device=dev, dtype=dt).float().cpu().numpy()
            if not f:
                ref[off:off + n] = _fma32(np.float32(c), z, ref[off:off + n])
            off += n
    got = delta.cpu().numpy()
    bad = got.view(np.uint32) != ref.view(np.uint32)
    assert not bad.any(), f"{int(bad.sum())} of {bad.size} delta elements differ (first {int(np.argmax(bad))})"


def test_seed_sharded_reconstruct_with_the_default_stream():
    """reconstruct_seed_sharded_ (the north star's C3 form, zo_utils.py) in a subprocess
    with FKS_STREAM_MODE unset: "auto" resolves to torch_rocm on the GPU, the delta is
    accumulated from the device stream, and the result equals delta_accumulate +
    delta_apply built from torch.normal(device="cuda") draws (fp32, wd 0.01)."""
    env = {k: v for k, v in os.environ.items() if k != "FKS_STREAM_MODE"}
    code = r'''
import sys
sys.path.insert(0, "fate-llm_amd/python"); sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import numpy as np, torch
from fate_llm.algo.fedkseed import codec, zo_utils
from test_gpu_torch_rocm_big import _fma32
assert codec.get_stream_mode() == "auto"
dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(4)
init = [(torch.randn(n, generator=g) * 0.02) for n in (4096, 300_001, 5)]
params = [torch.nn.Parameter(t.to(dev)) for t in init]
seeds = [101, 202, 303, 404]
vals = [2.0, -1.0, 0.0, 0.5]
lr, wd = 1e-3, 0.01
n = zo_utils.reconstruct_seed_sharded_([{"params": params, "lr": 0.0, "weight_decay": 0.0}], seeds, vals, lr, wd)
assert n == 3
keep = [(s, v) for s, v in zip(seeds, vals) if v != 0.0]
first, last, coefs, decay = zo_utils.seed_shard_coefficients([v for _, v in keep], lr, wd)
tot = sum(t.numel() for t in init)
delta = np.zeros(tot, np.float32)
for (s, _), c in zip(keep, coefs):
    torch.manual_seed(s)
    off = 0
    for t in init:
        z = torch.normal(0, 1, size=t.shape, device=dev).cpu().numpy()
        delta[off:off + t.numel()] = _fma32(np.float32(c), z, delta[off:off + t.numel()])
        off += t.numel()
off = 0
for p, t in zip(params, init):
    want = _fma32(np.float32(decay), t.numpy(), -delta[off:off + t.numel()])
    off += t.numel()
    assert np.array_equal(p.detach().cpu().numpy().view(np.uint32), want.view(np.uint32))
print("ok")
'''
    out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0 and out.stdout.strip().endswith("ok"), out.stderr[-3000:]
