"""C2 at its full size (BASELINE configs[1]): the bench's workload itself -- the LLaMA-7B
bf16 layout (291 tensors, 6,738,415,616 parameters, N(0, 0.02^2)) reconstructed from the
bench's K=4096 (seed, scalar) list (4055 non-zero, lr 1e-5, weight decay 0.0 -- the bench's default and the HF value
ClientTrainer passes, fedkseed.py:140, i.e. the kModeUpdateWd0 chain with the packed (C,S)
table that bench.py times -- and 0.01, the full chain) -- checked through
properties that do not need the oracle to walk 6.7e9 MT words per seed:

  * chunking: the stream's 8 element shards (an 8-GPU run's jumps and chunk boundaries),
    run one after another, == the whole 1-GPU reconstruct, bit for bit;
  * seed order: the list applied as two calls (2048 + 2007 seeds) == one call -- the
    reference applies the seeds one by one in list order (fedkseed.py:136-141);
  * oracle prefix: the embedding's first 4096 elements (stream words 0..4095: the same
    words, hence the same z, as a lone 4096-element tensor) == the oracle's sequential
    reconstruct of those elements with all 4055 seeds.

Three 13.5 GB copies of the buffer stay resident (40 GB of the 288 GB)."""
import os
import sys

import numpy as np
import pytest
import torch

from oracle import fks_oracle as O
from conftest import assert_bitwise
from test_gpu_parity import _dev

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PREFIX = 4096


def _differ(a: torch.Tensor, b: torch.Tensor) -> int:
    return int((a.view(torch.int16) != b.view(torch.int16)).sum().item())


@pytest.mark.parametrize("wd", [0.0, 0.01])
def test_c2_full_size_chunking_seed_order_and_oracle_prefix(wd):
    sys.path.insert(0, ROOT)
    import bench
    from fate_llm.algo.fedkseed import codec
    dev = _dev()
    shapes = bench.llama7b_shapes()
    n = [bench.numel(s) for s in shapes]
    total = sum(n)
    assert total == bench.LLAMA7B_PARAMS
    seeds, scalars = bench.synthetic_seeds(4096)
    keep = [(s, g) for s, g in zip(seeds, scalars) if g != 0.0]
    ks, kv = [s for s, _ in keep], [g for _, g in keep]
    assert len(ks) == 4055

    whole = torch.empty(total, dtype=torch.bfloat16, device=dev)
    whole.normal_(0.0, 0.02, generator=torch.Generator(dev).manual_seed(0))
    prefix0 = whole[:PREFIX].view(torch.int16).cpu().numpy().view(np.uint16).copy()
    shards = whole.clone()
    split = whole.clone()

    def specs(buf):
        out, off = [], 0
        for s, m in zip(shapes, n):
            out.append(codec.ParamSpec(buf[off:off + m].view(s), lr=1e-5, weight_decay=wd))
            off += m
        return out

    codec.directional_step(specs(whole), ks, kv)
    for r in range(8):
        codec.directional_step(specs(shards), ks, kv, shard=r, nshards=8)
    sp = specs(split)
    codec.directional_step(sp, ks[:2048], kv[:2048])
    codec.directional_step(sp, ks[2048:], kv[2048:])
    torch.cuda.synchronize()

    assert _differ(whole, shards) == 0, "8 element shards differ from the whole reconstruct"
    del shards
    assert _differ(whole, split) == 0, "two calls (2048 + 2007 seeds) differ from one call"
    del split
    # the run changed the buffer (an update of ~lr*|g|*|z| moves most bf16 parameters)
    moved = int((whole[:PREFIX].view(torch.int16).cpu().numpy().view(np.uint16) != prefix0).sum())
    assert moved > PREFIX // 2, f"only {moved} of {PREFIX} prefix elements changed"

    ref = [prefix0.copy()]
    O.reconstruct(ref, [O.BF16], [1e-5], [wd], ks, kv)
    got = whole[:PREFIX].view(torch.int16).cpu().numpy().view(np.uint16)
    assert_bitwise(got, ref[0], "bfloat16", "embedding prefix vs oracle")


@pytest.mark.parametrize("wd", [0.0, 0.01, None])
def test_zo_steps_full_size_caches_and_oracle_prefix(wd):
    """Three local zeroth-order steps (perturb +eps, perturb -2 eps, fused restore +
    update; optimizer.py:108-150) over the full 7B bf16 layout: with the jumped-window
    and z-index caches (the second and third pass of a step replay the first pass's
    table indices) == with both caches off, bit for bit, and the embedding's first 4096
    elements == the oracle's perturb / update sequence."""
    sys.path.insert(0, ROOT)
    import bench
    from fate_llm.algo.fedkseed import _native as N
    from fate_llm.algo.fedkseed import codec
    dev = _dev()
    shapes = bench.llama7b_shapes()
    n = [bench.numel(s) for s in shapes]
    base = torch.empty(sum(n), dtype=torch.bfloat16, device=dev)
    base.normal_(0.0, 0.02, generator=torch.Generator(dev).manual_seed(3))
    prefix = [base[:PREFIX].view(torch.int16).cpu().numpy().view(np.uint16).copy()]
    eps, lr = 5e-4, 1e-5
    steps = [(2718281828, -13.75), (97, 4.5), (4294967295, 0.0625)]

    def run(buf):
        views, off = [], 0
        for s, m in zip(shapes, n):
            views.append(buf[off:off + m].view(s))
            off += m
        specs = [codec.ParamSpec(v, lr=lr, weight_decay=wd) for v in views]
        for seed, g in steps:
            codec.perturb(views, seed, eps)
            codec.perturb(views, seed, -2 * eps)
            codec.perturb_step(specs, seed, [eps] * len(specs), g, value_is_tensor=False)
        torch.cuda.synchronize()

    out = {}
    for name, env in (("cached", {}), ("uncached", {"FKS_ZCACHE": "0", "FKS_NO_WIN_CACHE": "1"})):
        N.check(N.load().fks_plan_cache_clear())
        os.environ.update(env)
        try:
            buf = base.clone()
            run(buf)
            out[name] = buf
        finally:
            for key in env:
                os.environ.pop(key, None)
    assert _differ(out["cached"], out["uncached"]) == 0, "z-index / window caches change the result"
    del out["uncached"]
    for seed, g in steps:
        O.perturb_params(prefix, [O.BF16], seed, eps)
        O.perturb_params(prefix, [O.BF16], seed, -2 * eps)
        O.perturb_params(prefix, [O.BF16], seed, eps)
        O.reconstruct(prefix, [O.BF16], [lr], [wd], [seed], [g])
    got = out["cached"][:PREFIX].view(torch.int16).cpu().numpy().view(np.uint16)
    assert_bitwise(got, prefix[0], "bfloat16", "embedding prefix vs oracle")
