"""Randomised parity of the drop-in against the CPU oracle: 48 seeded random calls, each a
random tensor list (1..10 tensors; numel from the serial path's < 16 through ragged sizes
to 2^17, with every dtype, mixed in one call), random per-tensor lr / weight decay (None,
+0.0, -0.0, 0.01, 0.3), K in 1..80 (the small-K kernel, the 19-seed fp32 and the 32/64-seed
bf16 slice passes with their remainders), seeds past 2^32, scalars with zeros and edge
values, applied whole or as 2 or 3 element shards, with the reconstruct window cache on
or off.  Bit-exact (NaN matches NaN) against oracle.fks_oracle.reconstruct of the whole.
With the window cache on, the same call runs twice, cold then warm on a fresh copy of the
parameters (a client's next round), half the time with a seed repeated inside the first
64-seed pass: both results must match the oracle, and where the call uses the cache
(fks_jwin_size_shard > 0) the warm call must find seeds in it."""
import ctypes

import numpy as np
import pytest
import torch

from conftest import assert_bitwise
from oracle import fks_oracle as O
from test_gpu_parity import DTC, TD, _dev, from_np, to_np

pytestmark = pytest.mark.gpu
DTYPES = ["float32", "bfloat16", "float16"]


@pytest.fixture(scope="module", autouse=True)
def _release_window_cache():
    """The sweep attaches reconstruct window caches (cache_windows=True); the tests after
    this module start from none, as they would without it."""
    yield
    if torch.cuda.is_available():
        from fate_llm.algo.fedkseed import codec
        codec.jwin_release()


def _config(rng):
    nt = int(rng.integers(1, 11))
    sizes = []
    for _ in range(nt):
        kind = rng.integers(0, 4)
        if kind == 0:
            sizes.append(int(rng.integers(1, 16)))                # serial path
        elif kind == 1:
            sizes.append(int(rng.integers(16, 2000)))             # ragged
        elif kind == 2:
            sizes.append(16 * int(rng.integers(1, 4096)))         # whole 16-blocks
        else:
            sizes.append(int(rng.integers(2000, 1 << 17)))
    dtypes = [DTYPES[int(rng.integers(0, 3))] for _ in range(nt)]
    if rng.random() < 0.5:  # the common case: one dtype
        dtypes = [dtypes[0]] * nt
    lrs = [float(rng.choice([1e-5, 1e-3, 0.5])) for _ in range(nt)]
    wds = [[None, 0.0, -0.0, 0.01, 0.3][int(rng.integers(0, 5))] for _ in range(nt)]
    k = int(rng.choice([1, 2, 3, int(rng.integers(4, 20)), 19, 23, 32, 33, 40, 64, int(rng.integers(65, 81))]))
    seeds = [int(s) for s in rng.integers(0, 2**40, k)]
    vals = (rng.normal(0.0, 20.0, k)).tolist()
    for i in range(k):
        r = rng.random()
        if r < 0.05:
            vals[i] = 0.0
        elif r < 0.08:
            vals[i] = float(rng.choice([1e-40, -3e38, 1e30, -0.0]))
    nshards = int(rng.choice([1, 1, 2, 3]))
    jwin = bool(rng.random() < 0.5)
    if jwin and k >= 2 and rng.random() < 0.5:  # a seed twice inside one 64-seed pass
        seeds[int(rng.integers(1, min(k, 64)))] = seeds[0]
    return sizes, dtypes, lrs, wds, seeds, vals, nshards, jwin


@pytest.mark.parametrize("case", range(48))
def test_random_call_matches_oracle(case):
    from fate_llm.algo.fedkseed import codec
    dev = _dev()
    rng = np.random.default_rng(1000 + case)
    sizes, dtypes, lrs, wds, seeds, vals, nshards, jwin = _config(rng)
    from fate_llm.algo.fedkseed import _native as N
    g = torch.Generator().manual_seed(case)
    base = [to_np((torch.randn(n, generator=g) * 0.02).to(TD[d])) for n, d in zip(sizes, dtypes)]
    # train_once drops g == 0.0 entries (fedkseed.py:137; zo_utils.reconstruct_), the oracle too
    ks = [s for s, v in zip(seeds, vals) if v != 0.0]
    kv = [v for v in vals if v != 0.0]
    ref = [a.copy() for a in base]
    O.reconstruct(ref, [DTC[d] for d in dtypes], lrs, wds, seeds, vals)
    what = f"case {case}: sizes {sizes} dtypes {dtypes} wds {wds} k {len(seeds)} shards {nshards} jwin {jwin}"

    def run(label):
        ts = [from_np(a, d, dev) for a, d in zip(base, dtypes)]
        specs = [codec.ParamSpec(t, lr=lr, weight_decay=wd) for t, lr, wd in zip(ts, lrs, wds)]
        if ks:
            for r in range(nshards):
                codec.directional_step(specs, ks, kv, shard=r, nshards=nshards, cache_windows=jwin)
        torch.cuda.synchronize()
        for t, r_, d in zip(ts, ref, dtypes):
            assert_bitwise(to_np(t), r_, d, f"{what} ({label})")
        return specs

    specs = run("cold")
    if jwin and ks:
        used = False  # does any shard's call use the window cache?
        b = codec._Batch(specs)
        for r in range(nshards):
            need = ctypes.c_size_t(0)
            N.check(N.load().fks_jwin_size_shard(ctypes.addressof(b.arr), b.n, len(ks), r, nshards, ctypes.byref(need)))
            used |= need.value > 0
        hits0, _ = codec.jwin_stats()
        run("warm")
        hits1, _ = codec.jwin_stats()
        if used:
            assert hits1 > hits0, f"{what}: the warm call found no seed in the window cache"


@pytest.mark.parametrize("case", range(16))
def test_random_call_libm_flavour_matches_oracle(case):
    """The same sweep on the CPU stream's libm flavour (ATen's DEFAULT capability: glibc's
    logf / sinf / cosf for fp32), fp32-heavy layouts, against the oracle's
    CAP_DEFAULT path; element shards and the window cache as above."""
    from fate_llm.algo.fedkseed import codec
    dev = _dev()
    rng = np.random.default_rng(7000 + case)
    sizes, dtypes, lrs, wds, seeds, vals, nshards, jwin = _config(rng)
    dtypes = ["float32" if rng.random() < 0.75 else d for d in dtypes]
    g = torch.Generator().manual_seed(case)
    base = [to_np((torch.randn(n, generator=g) * 0.02).to(TD[d])) for n, d in zip(sizes, dtypes)]
    ks = [s for s, v in zip(seeds, vals) if v != 0.0]
    kv = [v for v in vals if v != 0.0]
    ref = [a.copy() for a in base]
    O.reconstruct(ref, [DTC[d] for d in dtypes], lrs, wds, seeds, vals, O.CAP_DEFAULT)
    what = f"libm case {case}: sizes {sizes} dtypes {dtypes} wds {wds} k {len(seeds)} shards {nshards} jwin {jwin}"
    codec.set_cpu_fp32_flavour("libm")
    try:
        for label in (("cold", "warm") if jwin else ("cold",)):
            ts = [from_np(a, d, dev) for a, d in zip(base, dtypes)]
            specs = [codec.ParamSpec(t, lr=lr, weight_decay=wd) for t, lr, wd in zip(ts, lrs, wds)]
            if ks:
                for r in range(nshards):
                    codec.directional_step(specs, ks, kv, shard=r, nshards=nshards, cache_windows=jwin)
            torch.cuda.synchronize()
            for t, r_, d in zip(ts, ref, dtypes):
                assert_bitwise(to_np(t), r_, d, f"{what} ({label})")
    finally:
        codec.set_cpu_fp32_flavour(None)


def _rocm_reference(params, seeds, vals, lrs, wds):
    """zo_utils.directional_derivative_step's torch calls on the device (zo_utils.py:42-52),
    per-tensor lr / wd as the codec's ParamSpecs carry them."""
    for sd, g in zip(seeds, vals):
        torch.manual_seed(sd)
        for p, lr, wd in zip(params, lrs, wds):
            z = torch.normal(mean=0, std=1, size=p.data.size(), device=p.data.device, dtype=p.data.dtype)
            if wd is not None:
                p.data = p.data - lr * (g * z + wd * p.data)
            else:
                p.data = p.data - lr * (g * z)


@pytest.mark.parametrize("case", range(24))
def test_random_call_matches_torch_on_device(case):
    """The torch_rocm stream (the reference's z when its model is on the MI355X) on random
    layouts -- bf16 mostly, where the radius shortcut of phx_z_bf16 applies -- against
    torch.normal(device="cuda") and the reference's update as torch ops."""
    from fate_llm.algo.fedkseed import codec
    dev = _dev()
    rng = np.random.default_rng(5000 + case)
    nt = int(rng.integers(1, 8))
    sizes = [int(rng.choice([int(rng.integers(1, 64)), int(rng.integers(64, 5000)), int(rng.integers(5000, 1 << 20))]))
             for _ in range(nt)]
    dtypes = [str(rng.choice(["bfloat16", "bfloat16", "bfloat16", "float32", "float16"])) for _ in range(nt)]
    lrs = [float(rng.choice([1e-5, 1e-3])) for _ in range(nt)]
    wds = [[None, 0.0, 0.01][int(rng.integers(0, 3))] for _ in range(nt)]
    k = int(rng.integers(1, 9))
    seeds = [int(s) for s in rng.integers(0, 2**40, k)]
    vals = [float(v) for v in rng.normal(0.0, 20.0, k)]
    g = torch.Generator(dev).manual_seed(case)
    base = [torch.empty(n, dtype=TD[d], device=dev).normal_(0.0, 0.02, generator=g) for n, d in zip(sizes, dtypes)]
    got = [b.clone() for b in base]
    specs = [codec.ParamSpec(t, lr=lr, weight_decay=wd) for t, lr, wd in zip(got, lrs, wds)]
    codec.directional_step(specs, seeds, vals, stream_mode="torch_rocm")
    ref = [torch.nn.Parameter(b.clone(), requires_grad=False) for b in base]
    _rocm_reference(ref, seeds, vals, lrs, wds)
    torch.cuda.synchronize()
    what = f"case {case}: sizes {sizes} dtypes {dtypes} wds {wds} k {k}"
    for a, r, d in zip(got, ref, dtypes):
        assert_bitwise(to_np(a), to_np(r.data), d, what)
