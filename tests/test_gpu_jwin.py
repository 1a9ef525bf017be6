"""The reconstruct window cache (include/fks.h fks_jwin_*; codec cache_windows, used by
zo_utils.reconstruct_): a client reconstructs the same (seed, sum) list from model_0
every round (fedkseed.py:57-68, :132-141), so the second round finds every seed's jumped
windows in the cache and skips the jumps.  A speed cache only: every result here is
bit-identical to the uncached reconstruct --

  * cold (filling) and warm (every seed found) calls, whole and element-sharded;
  * a second list sharing part of the first one's seeds, in another order;
  * a cache too small for the list (sets recycled while the call runs);
  * a cache filled by one shard's plan and then used by another's (the key resets it);
  * at full size: the bench's 7B bf16 layout, K=4096, 8 element shards with the cache
    cold and warm against the uncached whole reconstruct.
"""
import ctypes

import pytest
import torch

from test_gpu_parity import _dev

pytestmark = pytest.mark.gpu


def _bits(t):
    return t.view(torch.int16)


def _seeds(k, seed):
    g = torch.Generator().manual_seed(seed)
    return (torch.randint(0, 2**32, (k,), generator=g).tolist(),
            (torch.randn(k, generator=g, dtype=torch.float64) * 20).tolist())


def _specs(buf, sizes, wd):
    from fate_llm.algo.fedkseed import codec
    out, off = [], 0
    for n in sizes:
        out.append(codec.ParamSpec(buf[off:off + n], lr=1e-5, weight_decay=wd))
        off += n
    return out


@pytest.fixture
def fresh_cache():
    from fate_llm.algo.fedkseed import _native as N
    from fate_llm.algo.fedkseed import codec
    codec.jwin_release()
    N.check(N.load().fks_plan_cache_clear())
    yield codec
    codec.jwin_release()


@pytest.mark.parametrize("wd", [0.0, 0.01])
def test_cold_warm_partial_and_sharded_equal_uncached(fresh_cache, wd):
    codec = fresh_cache
    dev = _dev()
    sizes = [4096 * 1000, 48 * 64, 3_000_000 + 16 * 7, 11_008 * 512]
    total = sum(sizes)
    g = torch.Generator(device=dev).manual_seed(3)
    base = (torch.randn(total, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    ks, kv = _seeds(200, 5)
    ks2 = ks[150:] + _seeds(120, 6)[0]  # 50 seeds of the first list (other positions), 120 new
    kv2 = _seeds(170, 7)[1]

    def run(lists, cache, shards=1):
        buf = base.clone()
        sp = _specs(buf, sizes, wd)
        for s, v in lists:
            for r in range(shards):
                codec.directional_step(sp, s, v, shard=r, nshards=shards, cache_windows=cache)
        torch.cuda.synchronize()
        return buf

    lists = [(ks, kv), (ks2, kv2)]
    ref = run(lists, False)
    h0, m0 = codec.jwin_stats()
    cold = run(lists, True)
    h1, m1 = codec.jwin_stats()
    assert torch.equal(_bits(cold), _bits(ref))
    # the first list misses everywhere (its 8-seed remainder pass is not cached); the second
    # finds the shared seeds that sat in two-slice passes (42 of its 50)
    assert m1 - m0 > 0 and h1 - h0 >= 42
    # the same list twice: the second call jumps nothing
    one = run([(ks, kv)], True)
    h2, m2 = codec.jwin_stats()
    again = run([(ks, kv)], True)
    h3, m3 = codec.jwin_stats()
    ref1 = run([(ks, kv)], False)
    assert torch.equal(_bits(one), _bits(ref1)) and torch.equal(_bits(again), _bits(ref1))
    assert m3 - m2 == 0 and h3 - h2 == 192, "the warm call jumped into the cache"
    # element shards: each shard's plan keys the cache afresh
    sh_ref = run(lists, False, shards=3)
    sh_cold = run(lists, True, shards=3)
    sh_warm = run([(ks, kv)] * 2, True, shards=3)
    sh_ref2 = run([(ks, kv)] * 2, False, shards=3)
    assert torch.equal(_bits(sh_cold), _bits(sh_ref)) and torch.equal(_bits(sh_ref), _bits(ref))
    assert torch.equal(_bits(sh_warm), _bits(sh_ref2))


def test_cache_smaller_than_the_list(fresh_cache, monkeypatch):
    """A cache of 70 window sets against a 300-seed list: sets are recycled while the call
    runs (never one the running pass needs); results still equal the uncached ones."""
    codec = fresh_cache
    from fate_llm.algo.fedkseed import _native as N
    dev = _dev()
    n = 1 << 24
    base = (torch.randn(n, device=dev) * 0.02).to(torch.bfloat16)
    ks, kv = _seeds(300, 9)
    a, b = base.clone(), base.clone()
    spa = _specs(a, [n], 0.0)
    codec.directional_step(spa, ks, kv)
    spb = _specs(b, [n], 0.0)
    bt = codec._Batch(spb)
    need = ctypes.c_size_t(0)
    N.check(N.load().fks_jwin_size(ctypes.addressof(bt.arr), bt.n, 70, ctypes.byref(need)))
    small = torch.empty(int(need.value), dtype=torch.uint8, device=dev)
    N.check(N.load().fks_jwin_attach(small.data_ptr(), small.numel()))
    monkeypatch.setattr(codec, "JWIN_BUDGET_FRAC", 0.0)  # keep this buffer: no codec reservation
    try:
        h0, m0 = codec.jwin_stats()
        for _ in range(2):
            c = base.clone()
            codec.directional_step(_specs(c, [n], 0.0), ks, kv, cache_windows=True)
            torch.cuda.synchronize()
            assert torch.equal(_bits(c), _bits(a))
        h1, m1 = codec.jwin_stats()
        # all 300 seeds sit in two-slice passes; 70 sets hold the last ~70 of them, which the
        # second call's early passes evict before reaching them: both calls miss them all
        assert m1 - m0 == 600 and h1 - h0 == 0
    finally:
        N.check(N.load().fks_jwin_attach(None, 0))
        del small


def test_full_size_shards_cold_and_warm(fresh_cache):
    """The bench's 7B bf16 layout at K=4096, 8 element shards (one GPU's share of an 8-GPU
    run each), cache cold then warm, against the uncached whole reconstruct."""
    import os
    import sys
    codec = fresh_cache
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    dev = _dev()
    shapes = bench.llama7b_shapes()
    sizes = [bench.numel(s) for s in shapes]
    total = sum(sizes)
    seeds, scalars = bench.synthetic_seeds(4096)
    keep = [(s, g) for s, g in zip(seeds, scalars) if g != 0.0]
    ks, kv = [s for s, _ in keep], [g for _, g in keep]
    base = torch.empty(total, dtype=torch.bfloat16, device=dev)
    base.normal_(0.0, 0.02, generator=torch.Generator(dev).manual_seed(0))
    whole = base.clone()
    codec.directional_step(_specs(whole, sizes, 0.0), ks, kv)
    # each rank's shard has its own plan (a rank keeps one shard: the cache is per device)
    buf = base.clone()
    sp = _specs(buf, sizes, 0.0)
    for r in range(8):
        codec.directional_step(sp, ks, kv, shard=r, nshards=8, cache_windows=True)
    torch.cuda.synchronize()
    assert torch.equal(_bits(buf), _bits(whole))
    del buf
    # one shard twice in a row: the second call finds all of its two-slice-pass seeds
    buf = base.clone()
    sp = _specs(buf, sizes, 0.0)
    codec.directional_step(sp, ks, kv, shard=3, nshards=8, cache_windows=True)
    h0, m0 = codec.jwin_stats()
    codec.directional_step(sp, ks, kv, shard=3, nshards=8, cache_windows=True)
    h1, m1 = codec.jwin_stats()
    assert m1 - m0 == 0 and h1 - h0 == 64 * (len(ks) // 64)
    # ... with the same bits as the uncached shard applied twice
    ref = base.clone()
    spr = _specs(ref, sizes, 0.0)
    codec.directional_step(spr, ks, kv, shard=3, nshards=8)
    codec.directional_step(spr, ks, kv, shard=3, nshards=8)
    torch.cuda.synchronize()
    assert torch.equal(_bits(buf), _bits(ref))


def test_mixed_layout_cached_equals_uncached(fresh_cache):
    """A list where the slice kernel's bf16 fast segments (cached windows) sit beside
    tensors the other kernels take from the workspace's windows -- an fp32 tensor (19-seed
    kernel), a ragged bf16 tensor and its unaligned successor (irregular kernel), an f16
    tensor and numel < 16 tensors (serial path): cold and warm == uncached, bit for bit."""
    codec = fresh_cache
    dev = _dev()
    g = torch.Generator().manual_seed(17)
    spec = [((624 * 3000,), torch.bfloat16), ((5000, 3), torch.float32), ((1_000_003,), torch.bfloat16),
            ((624 * 1000,), torch.bfloat16), ((7,), torch.bfloat16), ((4096, 4), torch.float16),
            ((3,), torch.float32), ((624 * 2048,), torch.bfloat16)]
    base = [(torch.randn(s, generator=g) * 0.02).to(dt).to(dev) for s, dt in spec]
    ks, kv = _seeds(150, 18)

    def run(cache, reps=1):
        ps = [b.clone() for b in base]
        sp = [codec.ParamSpec(p, lr=1e-3, weight_decay=0.01 if i % 2 else None) for i, p in enumerate(ps)]
        for _ in range(reps):
            codec.directional_step(sp, ks, kv, cache_windows=cache)
        torch.cuda.synchronize()
        return ps

    ref = run(False, 2)
    h0, m0 = codec.jwin_stats()
    got = run(True, 2)  # the first call fills, the second finds every two-slice seed
    h1, m1 = codec.jwin_stats()
    for i, (a, b) in enumerate(zip(got, ref)):
        w = torch.int16 if a.element_size() == 2 else torch.int32
        assert torch.equal(a.view(w), b.view(w)), f"tensor {i}"
    assert m1 - m0 == 128 and h1 - h0 == 128  # 2 two-slice passes of 64 seeds, then a 22-seed split pass
