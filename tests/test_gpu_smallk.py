"""GPU parity of the small-K passes (<= 4 seeds: the ZO step's perturb / update calls),
which run the double-buffered apply kernel (fks_apply_kernel<..., DB>: a sixth wave
twists window 0 of block b+1 out of place while the pair waves run block b; windows
1..3 are twisted by pair waves 4..2).

Bar: bit-exact against the CPU oracle (pinned to the reference's golden vectors).  The
layouts have several MT blocks per chunk (the 7B-style plan gives 5 x CUs chunks), so
both buffers alternate many times, and tensors change inside blocks.
"""
import numpy as np
import pytest
import torch

from oracle import fks_oracle as O
from test_gpu_parity import DTC, _dev, _gpu_reconstruct, from_np, rand_params, to_np
from conftest import assert_bitwise

pytestmark = pytest.mark.gpu

# 6.3M params: ~10,000 MT blocks, about 8 per chunk at 1280 chunks
SHAPES = [2**22, 48, 1234 * 16, 2**21, 4096 * 3, 16, 624 * 16 + 32]


def _seeds(k, seed):
    g = torch.Generator().manual_seed(seed)
    return (torch.randint(0, 2**32, (k,), generator=g).tolist(),
            (torch.randn(k, generator=g, dtype=torch.float64) * 20).tolist())


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
@pytest.mark.parametrize("k", [1, 2, 3, 4])
def test_smallk_reconstruct_vs_oracle(dtype, k):
    arrays = rand_params(SHAPES, dtype, seed=20 + k)
    seeds, vals = _seeds(k, 30 + k)
    lrs = [1e-3] * len(SHAPES)
    wds = [0.01, None, 0.0, 0.01, None, 0.01, 0.0]
    got = _gpu_reconstruct(arrays, dtype, lrs, wds, seeds, vals)
    O.reconstruct(arrays, [DTC[dtype]] * len(arrays), lrs, wds, seeds, vals)
    for i, (a, b) in enumerate(zip(got, arrays)):
        assert_bitwise(a, b, dtype, f"K={k} tensor {i}")


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
def test_smallk_zo_step_sequence_vs_oracle(dtype):
    """One zeroth-order step's three passes on the multi-block layout: perturb +1,
    perturb -2, then the fused restore (+1) and update (perturb_step)."""
    from fate_llm.algo.fedkseed import codec
    dev = _dev()
    arrays = rand_params(SHAPES, dtype, seed=7)
    ts = [from_np(a, dtype, dev) for a in arrays]
    eps, seed, g = 5e-4, 2718281828, -13.75
    for sf in (1.0, -2.0):
        codec.perturb(ts, seed, sf * eps)
        O.perturb_params(arrays, [DTC[dtype]] * len(arrays), seed, sf * eps)
    specs = [codec.ParamSpec(t, lr=1e-3, weight_decay=0.01) for t in ts]
    codec.perturb_step(specs, seed, [eps] * len(ts), g, value_is_tensor=False)
    torch.cuda.synchronize()
    O.perturb_params(arrays, [DTC[dtype]] * len(arrays), seed, eps)
    O.reconstruct(arrays, [DTC[dtype]] * len(arrays), [1e-3] * len(arrays), [0.01] * len(arrays), [seed], [g])
    for i, (t, a) in enumerate(zip(ts, arrays)):
        assert_bitwise(to_np(t), a, dtype, f"tensor {i}")


def test_smallk_shards_equal_oracle():
    """Element shards of a K=2 call (each shard its own small plan) tile the stream."""
    from fate_llm.algo.fedkseed import codec
    dev = _dev()
    arrays = rand_params(SHAPES[:4], "bfloat16", seed=8)
    seeds, vals = _seeds(2, 9)
    ts = [from_np(a, "bfloat16", dev) for a in arrays]
    specs = [codec.ParamSpec(t, lr=1e-3, weight_decay=0.01) for t in ts]
    for r in range(3):
        codec.directional_step(specs, seeds, vals, shard=r, nshards=3)
    torch.cuda.synchronize()
    O.reconstruct(arrays, [O.BF16] * 4, [1e-3] * 4, [0.01] * 4, seeds, vals)
    for i, (t, a) in enumerate(zip(ts, arrays)):
        assert_bitwise(to_np(t), a, "bfloat16", f"tensor {i}")
