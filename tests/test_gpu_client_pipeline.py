"""The drop-in ClientTrainer's round pipeline (fedkseed.py ClientTrainer.materialize /
reconstruct; reference fedkseed.py:130-141): for every model_0 placement (host with
pinned staging, pinned, device-resident) the round's model equals the reference's
flow -- copy.deepcopy(model_0).to(device) then the reconstruct -- bit for bit, over
several rounds, with tied weights still tied and model_0 itself untouched."""
import copy

import numpy as np
import pytest
import torch
from torch import nn

from test_gpu_parity import _dev

pytestmark = pytest.mark.gpu


class Tiny(nn.Module):
    def __init__(self):
        super().__init__()
        g = torch.Generator().manual_seed(3)
        self.emb = nn.Embedding(300, 64)
        self.proj = nn.Linear(64, 300, bias=True)
        self.proj.weight = self.emb.weight  # tied (one z-stream slot, as named_parameters dedups)
        self.norm = nn.LayerNorm(64)
        self.big = nn.Parameter(torch.randn(3_000_017, generator=g) * 0.02)  # > one 64 MiB stage in f32? no: 12 MB
        self.huge = nn.Parameter(torch.randn(20_000_000, generator=g) * 0.02)  # 80 MB: crosses stage buffers
        self.register_buffer("steps", torch.arange(7))
        with torch.no_grad():
            self.emb.weight.copy_(torch.randn(300, 64, generator=g) * 0.02)


class Args:
    learning_rate = 1e-5
    weight_decay = 0.01

    def __init__(self, dev):
        self.device = dev


def _state(m):
    return {k: v.detach().cpu().clone() for k, v in m.state_dict(keep_vars=False).items()}


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("placement", ["host", "pinned", "device"])
def test_round_model_equals_reference_flow(placement, dtype):
    from fate_llm.algo.fedkseed.fedkseed import ClientTrainer
    from fate_llm.algo.fedkseed.pytorch_utils import get_optimizer_parameters_grouped_with_decay
    from fate_llm.algo.fedkseed.zo_utils import reconstruct_
    dev = _dev()
    model_0 = Tiny().to(dtype)
    before = _state(model_0)
    ct = ClientTrainer(None, model_0, None, Args(dev), None, None, None, None, model_0_placement=placement)
    g = torch.Generator().manual_seed(5)
    seeds = torch.randint(0, 2**32, (40,), generator=g).tolist()
    for rnd in range(3):
        sums = {s: float(v) for s, v in zip(seeds, torch.randn(40, generator=g, dtype=torch.float64) * 20)}
        sums[seeds[rnd]] = 0.0
        got = ct.reconstruct(sums)
        ref = copy.deepcopy(model_0).to(dev)  # the reference's flow (fedkseed.py:132-141)
        reconstruct_(get_optimizer_parameters_grouped_with_decay(ref, Args.weight_decay), list(sums), list(sums.values()),
                     lr=Args.learning_rate, weight_decay=Args.weight_decay)
        torch.cuda.synchronize()
        assert got.proj.weight is got.emb.weight
        for (k, a), (_, b) in zip(got.state_dict().items(), ref.state_dict().items()):
            assert a.device.type == "cuda" and a.dtype == b.dtype
            assert torch.equal(a.view(torch.uint8), b.view(torch.uint8)) if a.is_floating_point() else torch.equal(a, b), k
        del got, ref
    after = _state(model_0)
    for k in before:
        assert torch.equal(before[k], after[k]), f"model_0 changed: {k}"
    assert all(p.device.type == "cpu" for p in model_0.parameters())
    if placement == "pinned":
        assert all(p.is_pinned() for p in model_0.parameters())
