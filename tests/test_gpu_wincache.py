"""The one-seed caches (fks_capi.cpp): the jumped-window cache (WinCache) and the bf16
z-index cache (ZCache: a perturb stores every block's table indices, later calls with
the same seed replay them without the generator).  A sequence of perturb / perturb_step
/ K=1 update calls that hits, misses (new seed, other tensor list with other chunk
starts, shard), and moves to another stream and back (the buffers pass between streams
through events) gives the same parameters, bit for bit, with either cache or both on as
with both off (FKS_NO_WIN_CACHE, FKS_ZCACHE=0, read per call)."""
import os

import pytest
import torch

from test_gpu_parity import _dev, from_np, rand_params

pytestmark = pytest.mark.gpu


def _sequence(params, side):
    from fate_llm.algo.fedkseed import codec
    specs = [codec.ParamSpec(p, lr=1e-3, weight_decay=0.01 if i % 2 else None) for i, p in enumerate(params)]
    sub = specs[1:]  # another tensor list: other chunk starts
    codec.perturb(params, 11, 5e-4)                                  # miss
    codec.perturb(params, 11, -1e-3)                                 # hit
    codec.perturb_step(specs, 11, [5e-4] * len(specs), 2.5)          # hit
    codec.perturb(params, 12, 5e-4)                                  # new seed: miss
    codec.perturb([s.tensor for s in sub], 12, 5e-4)                 # other layout, same seed: miss
    codec.directional_step(sub, [12], [0.75])                        # hit
    codec.directional_step(specs, [12], [0.75], shard=1, nshards=2)  # shard: other chunk starts
    codec.directional_step(specs, [12], [0.5])
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):                                    # another stream: hit
        codec.perturb(params, 12, 5e-4)
        codec.perturb(params, 13, 5e-4)
    torch.cuda.current_stream().wait_stream(side)
    codec.perturb(params, 13, -5e-4)                                 # back on the owning stream
    torch.cuda.synchronize()


CONFIGS = {"both": {}, "windows only": {"FKS_ZCACHE": "0"}, "z only": {"FKS_NO_WIN_CACHE": "1"},
           "none": {"FKS_ZCACHE": "0", "FKS_NO_WIN_CACHE": "1"}}


@pytest.mark.parametrize("dtype", ["bfloat16", "float32"])
def test_caches_match_uncached(dtype):
    from fate_llm.algo.fedkseed import _native as N
    dev = _dev()
    shapes = [4096 * 3, 7, 1000, 624 * 5 + 3, 64, 624 * 40]
    arrays = rand_params(shapes, dtype, seed=71)
    side = torch.cuda.Stream(dev)
    out = {}
    for name, env in CONFIGS.items():
        N.check(N.load().fks_plan_cache_clear())  # every configuration starts with empty caches
        os.environ.update(env)
        try:
            params = [from_np(a, dtype, dev) for a in arrays]
            _sequence(params, side)
            out[name] = [p.clone() for p in params]
        finally:
            for key in env:
                os.environ.pop(key, None)
    view = torch.int16 if dtype == "bfloat16" else torch.int32
    for name in ("both", "windows only", "z only"):
        for i, (a, b) in enumerate(zip(out[name], out["none"])):
            assert torch.equal(a.view(view), b.view(view)), f"{name}: tensor {i}"


def test_caches_match_uncached_mixed_dtypes():
    """bf16 tensors next to f32 and f16 ones (and numel < 16 and ragged ones) in one list:
    the bf16 fast segments replay their z indices while the f32 segments and the
    irregular runs still generate from the (cached) windows of the same call."""
    from fate_llm.algo.fedkseed import _native as N
    dev = _dev()
    layout = [("bfloat16", 4096 * 2), ("float32", 1024), ("bfloat16", 7), ("float16", 1000),
              ("bfloat16", 624 * 9 + 5), ("float32", 33), ("bfloat16", 4096)]
    arrays = [rand_params([n], dt, seed=91 + i)[0] for i, (dt, n) in enumerate(layout)]
    side = torch.cuda.Stream(dev)
    out = {}
    for name, env in CONFIGS.items():
        N.check(N.load().fks_plan_cache_clear())
        os.environ.update(env)
        try:
            params = [from_np(a, dt, dev) for a, (dt, _) in zip(arrays, layout)]
            _sequence(params, side)
            out[name] = [p.clone() for p in params]
        finally:
            for key in env:
                os.environ.pop(key, None)
    for name in ("both", "windows only", "z only"):
        for i, (a, b) in enumerate(zip(out[name], out["none"])):
            w = torch.int32 if a.dtype == torch.float32 else torch.int16
            assert torch.equal(a.view(w), b.view(w)), f"{name}: tensor {i} ({layout[i][0]})"


def test_zcache_other_bf16_layout_same_range():
    """Two tensor lists over the same stream range and seed whose bf16 segments cover
    different blocks (bf16 then f32, and f32 then bf16): the second list's update must
    not replay the first list's store, which holds no indices for its bf16 blocks."""
    from fate_llm.algo.fedkseed import _native as N
    from fate_llm.algo.fedkseed import codec
    dev = _dev()
    n = 624 * 64
    a_np = rand_params([n, n], "bfloat16", seed=5)
    b_np = rand_params([n, n], "float32", seed=6)
    out = {}
    for name, env in (("both", {}), ("none", {"FKS_ZCACHE": "0", "FKS_NO_WIN_CACHE": "1"})):
        N.check(N.load().fks_plan_cache_clear())
        os.environ.update(env)
        try:
            first = [from_np(a_np[0], "bfloat16", dev), from_np(b_np[1], "float32", dev)]
            second = [from_np(b_np[0], "float32", dev), from_np(a_np[1], "bfloat16", dev)]
            codec.perturb(first, 21, 5e-4)                      # stores the first list's bf16 blocks
            codec.directional_step([codec.ParamSpec(p, lr=1e-3) for p in second], [21], [0.75])
            torch.cuda.synchronize()
            out[name] = [p.clone() for p in first + second]
        finally:
            for key in env:
                os.environ.pop(key, None)
    for i, (a, b) in enumerate(zip(out["both"], out["none"])):
        w = torch.int32 if a.dtype == torch.float32 else torch.int16
        assert torch.equal(a.view(w), b.view(w)), f"tensor {i}"
