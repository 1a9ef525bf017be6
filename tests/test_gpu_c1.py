"""C1 at its full size (BASELINE configs[0]): the FedKSeed tutorial's own model -- GPT-2
124M in fp32 (doc/tutorial/fedkseed/fedkseed-example.ipynb:160-178, pipeline :330-395:
`model_name_or_path = "gpt2"`, learning_rate 1e-5, fp16=False) -- reconstructed the way
ClientTrainer.train_once does it (fedkseed.py:130-141): the model grouped by
get_optimizer_parameters_grouped_with_decay (pytorch_utils.py:34-51: 98 no-decay tensors
-- LayerNorm weights and every bias -- then 50 decay tensors, which fixes the z-stream
order), every group updated with the explicit lr / weight_decay train_once passes, seeds
in the dict's insertion order, exact zeros skipped.

Random-init weights of that architecture (no network for the checkpoint); the bench's
K=4096 (seed, scalar) list (4055 non-zero).  Checked, for weight decay 0.0 (the HF default
the tutorial leaves in place) and 0.01, and at 0.0 on the libm flavour (a reference host under
ATen's DEFAULT CPU capability):

  * 8 element shards run one after another == the whole reconstruct, bit for bit;
  * the list applied as two calls (2048 + 2007 non-zero seeds) == one call;
  * the oracle: every element of the no-decay group (98 tensors, 121,344 elements) and the
    first 4096 elements of the first decay tensor (transformer.wte) == the oracle's
    sequential reconstruct with all 4055 seeds (the wte prefix takes the same stream words
    as a lone 4096-element tensor there: its size is a multiple of 16).
"""
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


class Args:
    learning_rate = 1e-5

    def __init__(self, dev, wd):
        self.device = dev
        self.weight_decay = wd


def _gpt2_124m():
    from transformers import GPT2Config, GPT2LMHeadModel
    torch.manual_seed(0)
    return GPT2LMHeadModel(GPT2Config()).float().eval()


def _flat(params):
    return torch.cat([p.detach().reshape(-1).view(torch.int32) for p in params])


@pytest.fixture(scope="module")
def model_0():
    return _gpt2_124m()


@pytest.mark.parametrize("wd,flavour", [(0.0, "avx"), (0.01, "avx"), (0.0, "libm")])
def test_c1_gpt2_124m_fp32_k4096(model_0, wd, flavour):
    """flavour "libm": the same run as a reference host under ATen's DEFAULT CPU capability
    draws it (glibc's logf / sinf / cosf for every fp32 tensor)."""
    from fate_llm.algo.fedkseed import codec
    codec.set_cpu_fp32_flavour(flavour)
    try:
        _c1(model_0, wd, O.CAP_DEFAULT if flavour == "libm" else O.CAP_AVX2)
    finally:
        codec.set_cpu_fp32_flavour(None)


def _c1(model_0, wd, cap):
    sys.path.insert(0, ROOT)
    import bench
    from fate_llm.algo.fedkseed import codec
    from fate_llm.algo.fedkseed.fedkseed import ClientTrainer
    from fate_llm.algo.fedkseed.pytorch_utils import get_optimizer_parameters_grouped_with_decay
    from fate_llm.algo.fedkseed.zo_utils import reconstruct_

    dev = _dev()
    groups0 = get_optimizer_parameters_grouped_with_decay(model_0, wd)
    assert [len(g["params"]) for g in groups0] == [98, 50]
    assert sum(p.numel() for g in groups0 for p in g["params"]) == 124_439_808

    seeds, scalars = bench.synthetic_seeds(4096)
    sums = dict(zip(seeds, scalars))
    assert len(sums) == 4096
    keep = [(s, g) for s, g in sums.items() if g != 0.0]
    assert len(keep) == 4055

    ct = ClientTrainer(None, model_0, None, Args(dev, wd), None, None, None, None, model_0_placement="host")
    whole = ct.reconstruct(sums)  # the train_once path: materialize + grouped reconstruct_
    assert whole.lm_head.weight is whole.transformer.wte.weight
    torch.cuda.synchronize()
    g_whole = get_optimizer_parameters_grouped_with_decay(whole, wd)
    params_whole = [p for g in g_whole for p in g["params"]]

    # 8 element shards, one after another, over a fresh copy of model_0
    sharded = ct.materialize()
    specs = codec.resolve_groups(get_optimizer_parameters_grouped_with_decay(sharded, wd), lr=1e-5, weight_decay=wd)
    ks, kv = [s for s, _ in keep], [g for _, g in keep]
    for r in range(8):
        codec.directional_step(specs, ks, kv, shard=r, nshards=8)
    # two calls, 2048 + 2007 non-zero seeds
    split = ct.materialize()
    gs = get_optimizer_parameters_grouped_with_decay(split, wd)
    reconstruct_(gs, ks[:2048], kv[:2048], lr=1e-5, weight_decay=wd)
    reconstruct_(gs, ks[2048:], kv[2048:], lr=1e-5, weight_decay=wd)
    torch.cuda.synchronize()

    a = _flat(params_whole)
    b = _flat([sp.tensor for sp in specs])
    assert int((a != b).sum()) == 0, "8 element shards differ from the whole reconstruct"
    c = _flat([p for g in gs for p in g["params"]])
    assert int((a != c).sum()) == 0, "two calls (2048 + 2007 seeds) differ from one call"

    # the oracle: the no-decay group in full, then the first 4096 elements of wte
    no_decay0 = [p.detach().reshape(-1).numpy().copy() for p in groups0[0]["params"]]
    wte0 = model_0.transformer.wte.weight.detach().reshape(-1)[:PREFIX].numpy().copy()
    assert groups0[1]["params"][0] is model_0.transformer.wte.weight
    ref = [a.copy() for a in no_decay0] + [wte0.copy()]
    O.reconstruct(ref, [O.F32] * len(ref), [1e-5] * len(ref), [wd] * len(ref), ks, kv, cap)
    got_nd = [p.detach().reshape(-1).cpu().numpy() for p in g_whole[0]["params"]]
    moved = 0
    for i, (g, r, p0) in enumerate(zip(got_nd, ref, no_decay0)):
        assert_bitwise(g, r, "float32", f"no-decay tensor {i} vs oracle")
        moved += int((g.view(np.uint32) != p0.view(np.uint32)).sum())
    assert moved > 121_344 // 2, f"only {moved} no-decay elements changed"
    got_wte = whole.transformer.wte.weight.detach().reshape(-1)[:PREFIX].cpu().numpy()
    assert_bitwise(got_wte, ref[-1], "float32", "wte prefix vs oracle")
