"""The jumped-window cache of one-seed calls (fks_capi.cpp WinCache): a sequence of
perturb / perturb_step / K=1 update calls that hits, misses (new seed, other tensor list
with other chunk starts, shard), and moves to another stream and back (the buffer passes
between streams through an event) gives the same parameters, bit for bit, as the same
sequence with the cache off (FKS_NO_WIN_CACHE, read per call)."""
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


@pytest.mark.parametrize("dtype", ["bfloat16", "float32"])
def test_window_cache_matches_uncached(dtype):
    dev = _dev()
    shapes = [4096 * 3, 7, 1000, 624 * 5 + 3, 64]
    arrays = rand_params(shapes, dtype, seed=71)
    side = torch.cuda.Stream(dev)
    out = {}
    for cached in (True, False):
        if cached:
            os.environ.pop("FKS_NO_WIN_CACHE", None)
        else:
            os.environ["FKS_NO_WIN_CACHE"] = "1"
        try:
            params = [from_np(a, dtype, dev) for a in arrays]
            _sequence(params, side)
            out[cached] = [p.clone() for p in params]
        finally:
            os.environ.pop("FKS_NO_WIN_CACHE", None)
    for i, (a, b) in enumerate(zip(out[True], out[False])):
        assert torch.equal(a.view(torch.int16 if a.dtype == torch.bfloat16 else torch.int32),
                           b.view(torch.int16 if b.dtype == torch.bfloat16 else torch.int32)), f"tensor {i}"
