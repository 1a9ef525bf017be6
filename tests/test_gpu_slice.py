"""GPU parity of the bf16 slice kernel (fks_apply_bs_kernel: bit-sliced MT19937, 64 seeds
per pass as two 32-seed slices, the second applied after the first), which takes the bf16
fast segments of every reconstruct of K >= 20 seeds.

Bar: bit-exact against the CPU oracle (itself pinned to the reference's golden vectors).
Cases: the smallest slice call (K = 20: slices of 10 + 10), one full slice (K = 32:
16 + 16), 33 (17 + 16), a full pass (K = 64), a full pass plus a one-seed pass (K = 65:
the second slice of the last pass is empty), 95 (64 + 16 + 15), 127 (64 + 32 + 31); the
three update modes (weight decay on every tensor, on none, mixed); many small segments
switching inside MT blocks; fp32 tensors interleaved (they stay on the 19-seed kernel); a
one-block stream (one task per chunk, five of a half's six waves idle); element shards;
chunks of many MT blocks.
"""
import numpy as np
import pytest
import torch

from oracle import fks_oracle as O
from test_gpu_parity import DTC, _dev, _gpu_reconstruct, from_np, rand_params, to_np
from conftest import assert_bitwise

pytestmark = pytest.mark.gpu


def _seeds(k, seed):
    g = torch.Generator().manual_seed(seed)
    seeds = torch.randint(0, 2**32, (k,), generator=g).tolist()
    vals = (torch.randn(k, generator=g, dtype=torch.float64) * 20).tolist()
    return seeds, vals


SHAPES = [2**17, 48, 1234 * 16, 2**16, 4096 * 3, 16, 624 * 16 + 32]


@pytest.mark.parametrize("k", [20, 32, 33, 64, 65, 95, 127])
@pytest.mark.parametrize("wdmode", ["all", "none", "mixed"])
def test_slice_reconstruct_vs_oracle(k, wdmode):
    arrays = rand_params(SHAPES, "bfloat16", seed=k)
    seeds, vals = _seeds(k, seed=100 + k)
    lrs = [1e-3] * len(SHAPES)
    wds = {"all": [0.01] * len(SHAPES), "none": [None] * len(SHAPES),
           "mixed": [0.01, None, 0.0, 0.01, None, 0.01, 0.0]}[wdmode]
    got = _gpu_reconstruct(arrays, "bfloat16", lrs, wds, seeds, vals)
    O.reconstruct(arrays, [O.BF16] * len(arrays), lrs, wds, seeds, vals)
    for i, (a, b) in enumerate(zip(got, arrays)):
        assert_bitwise(a, b, "bfloat16", f"K={k} {wdmode} tensor {i}")


def test_slice_many_small_segments_and_fp32_interleaved():
    """48 tensors of 16..1024 elements (segment changes inside MT blocks), every fourth
    one fp32 (the 19-seed kernel), K = 41."""
    from fate_llm.algo.fedkseed import codec
    dev = _dev()
    rng = np.random.default_rng(3)
    shapes = [int(16 * rng.integers(1, 65)) for _ in range(48)]
    dts = ["float32" if i % 4 == 3 else "bfloat16" for i in range(48)]
    arrays = [rand_params([n], d, seed=i)[0] for i, (n, d) in enumerate(zip(shapes, dts))]
    seeds, vals = _seeds(41, seed=9)
    ts = [from_np(a, d, dev) for a, d in zip(arrays, dts)]
    wds = [0.01 if i % 3 else None for i in range(48)]
    specs = [codec.ParamSpec(t, lr=2e-3, weight_decay=w) for t, w in zip(ts, wds)]
    codec.directional_step(specs, seeds, vals)
    torch.cuda.synchronize()
    O.reconstruct(arrays, [DTC[d] for d in dts], [2e-3] * 48, wds, seeds, vals)
    for i, (t, a, d) in enumerate(zip(ts, arrays, dts)):
        assert_bitwise(to_np(t), a, d, f"tensor {i} ({d}, {shapes[i]})")


def test_slice_one_block_stream():
    """A 16-element stream: one MT block, one chunk of one task."""
    arrays = rand_params([16], "bfloat16", seed=2)
    seeds, vals = _seeds(40, seed=3)
    got = _gpu_reconstruct(arrays, "bfloat16", [1e-3], [0.01], seeds, vals)
    O.reconstruct(arrays, [O.BF16], [1e-3], [0.01], seeds, vals)
    assert_bitwise(got[0], arrays[0], "bfloat16", "one block")


@pytest.mark.parametrize("nshards", [2, 5])
def test_slice_element_shards_equal_oracle(nshards):
    from fate_llm.algo.fedkseed import codec
    dev = _dev()
    shapes = [2**18, 624 * 40, 2**16 + 16]
    arrays = rand_params(shapes, "bfloat16", seed=4)
    seeds, vals = _seeds(50, seed=5)
    ts = [from_np(a, "bfloat16", dev) for a in arrays]
    specs = [codec.ParamSpec(t, lr=1e-3, weight_decay=0.01) for t in ts]
    for r in range(nshards):
        codec.directional_step(specs, seeds, vals, shard=r, nshards=nshards)
    torch.cuda.synchronize()
    O.reconstruct(arrays, [O.BF16] * 3, [1e-3] * 3, [0.01] * 3, seeds, vals)
    for i, (t, a) in enumerate(zip(ts, arrays)):
        assert_bitwise(to_np(t), a, "bfloat16", f"tensor {i}")


@pytest.mark.parametrize("k", [32, 95])
@pytest.mark.parametrize("wd", [0.0, None])
def test_slice_multiblock_chunks_vs_oracle(k, wd):
    """The regime of every 7B launch: each of the slice kernel's 256 chunks spans many MT
    blocks, so the tasks' twists carry block b into b + 1 inside a chunk and the second
    slice waits on the first one's stores (the bench's chain: weight decay 0.0 ->
    kModeUpdateWd0, None -> kModeUpdateNoWd).  4.2 M bf16 params = 6,771 MT blocks (26
    per chunk, 127 tasks); K = 32 is one pass of two 16-seed slices, K = 95 a full pass
    and a partial one.  Bit-exact against the oracle (fedkseed.py:136-141, zo_utils.py:47-52)."""
    from fate_llm.algo.fedkseed import codec
    dev = _dev()
    shapes = [1 << 22, 624 * 48 + 32]
    arrays = rand_params(shapes, "bfloat16", seed=1000 + k)
    seeds, vals = _seeds(k, seed=2000 + k)
    ts = [from_np(a, "bfloat16", dev) for a in arrays]
    assert codec.stream_length(ts) // 624 >= 16 * 256, "fewer than 16 MT blocks per chunk"
    specs = [codec.ParamSpec(t, lr=1e-5, weight_decay=wd) for t in ts]
    codec.directional_step(specs, seeds, vals)
    torch.cuda.synchronize()
    O.reconstruct(arrays, [O.BF16] * len(arrays), [1e-5] * len(arrays), [wd] * len(arrays), seeds, vals)
    for i, (t, a) in enumerate(zip(ts, arrays)):
        assert_bitwise(to_np(t), a, "bfloat16", f"K={k} wd={wd} tensor {i}")
