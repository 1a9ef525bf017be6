"""The torch_rocm stream (a reference client whose model sits on an MI355X: zo_utils.py:47
and optimizer.py:170-172 draw z on ``param.data.device``) at the configs' full sizes,
against the reference's own arithmetic run on the same GPU -- torch.manual_seed, then
per tensor torch.normal on the device and the update expression as torch ops
(zo_utils.py:42-52) -- bit for bit:

  * C2's LLaMA-7B bf16 layout (291 tensors, 6,738,415,616 parameters): three seeds (one
    past 2^32), weight decay 0.0; every tensor's Philox offset follows from the ones before
    it, so the last tensors check the whole chain of offsets; and the same layout as 8
    row-aligned element shards run one after another == the whole, the shards' element
    ranges tiling the buffer;
  * C1's GPT-2 124M fp32 model through ClientTrainer.reconstruct in torch_rocm mode (the
    tutorial pipeline's use_cpu=False), the reference's two groups, wd 0.01.
"""
import os
import sys

import pytest
import torch

from test_gpu_parity import _dev

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def reference_step(params, seed, g, lr, weight_decay):
    """zo_utils.directional_derivative_step's torch calls (zo_utils.py:42-52) on the
    parameters' device -- the reference's arithmetic, not the drop-in."""
    torch.manual_seed(seed)
    for p in params:
        z = torch.normal(mean=0, std=1, size=p.data.size(), device=p.data.device, dtype=p.data.dtype)
        if weight_decay is not None:
            p.data = p.data - lr * (g * z + weight_decay * p.data)
        else:
            p.data = p.data - lr * (g * z)


def _differ(a, b):
    w = torch.int16 if a.element_size() == 2 else torch.int32
    return int((a.view(w) != b.view(w)).sum().item())


def test_c2_7b_bf16_against_torch_on_device():
    sys.path.insert(0, ROOT)
    import bench
    from fate_llm.algo.fedkseed import codec
    dev = _dev()
    shapes = bench.llama7b_shapes()
    sizes = [bench.numel(s) for s in shapes]
    total = sum(sizes)
    seeds, vals = [12345, 2**32 + 7, 987654321], [3.5, -17.25, 0.625]  # one seed past 2^32
    base = torch.empty(total, dtype=torch.bfloat16, device=dev)
    base.normal_(0.0, 0.02, generator=torch.Generator(dev).manual_seed(0))

    got = base.clone()
    off, specs = 0, []
    for s, n in zip(shapes, sizes):
        specs.append(codec.ParamSpec(got[off:off + n].view(s), lr=1e-5, weight_decay=0.0))
        off += n
    codec.directional_step(specs, seeds, vals, stream_mode="torch_rocm")

    ref = []
    off = 0
    for s, n in zip(shapes, sizes):
        ref.append(torch.nn.Parameter(base[off:off + n].view(s).clone(), requires_grad=False))
        off += n
    del base
    for sd, g in zip(seeds, vals):
        reference_step(ref, sd, g, 1e-5, 0.0)
    torch.cuda.synchronize()
    off = 0
    for i, (p, n) in enumerate(zip(ref, sizes)):
        d = _differ(got[off:off + n], p.data.reshape(-1))
        assert d == 0, f"tensor {i} of 291: {d} elements differ"
        off += n


def test_c2_7b_bf16_shards_equal_whole():
    sys.path.insert(0, ROOT)
    import bench
    from fate_llm.algo.fedkseed import codec
    dev = _dev()
    shapes = bench.llama7b_shapes()
    sizes = [bench.numel(s) for s in shapes]
    total = sum(sizes)
    seeds, vals = [5, 2**40 + 3, 77], [1.5, -2.0, 9.0]
    base = torch.empty(total, dtype=torch.bfloat16, device=dev)
    base.normal_(0.0, 0.02, generator=torch.Generator(dev).manual_seed(1))

    def specs(buf):
        out, off = [], 0
        for s, n in zip(shapes, sizes):
            out.append(codec.ParamSpec(buf[off:off + n].view(s), lr=1e-5, weight_decay=0.0))
            off += n
        return out

    whole = base.clone()
    codec.directional_step(specs(whole), seeds, vals, stream_mode="torch_rocm")
    sp = specs(base)
    ends = [0]
    for r in range(8):
        lo, hi = codec.shard_range(sp, r, 8, stream_mode="torch_rocm")
        assert lo == ends[-1]
        ends.append(hi)
        codec.directional_step(sp, seeds, vals, shard=r, nshards=8, stream_mode="torch_rocm")
    assert ends[-1] == total
    torch.cuda.synchronize()
    assert _differ(base, whole) == 0


def test_c1_gpt2_fp32_reconstruct_torch_rocm():
    from transformers import GPT2Config, GPT2LMHeadModel
    from fate_llm.algo.fedkseed import codec
    from fate_llm.algo.fedkseed.fedkseed import ClientTrainer
    from fate_llm.algo.fedkseed.pytorch_utils import get_optimizer_parameters_grouped_with_decay

    class Args:
        learning_rate = 1e-5
        weight_decay = 0.01

        def __init__(self, dev):
            self.device = dev

    dev = _dev()
    torch.manual_seed(0)
    model_0 = GPT2LMHeadModel(GPT2Config()).float().eval()
    sums = {11: 2.5, 2**33 + 1: 0.0, 4242: -13.0, 3141592653: 0.75, 99: 6.0}
    old = codec.get_stream_mode()
    codec.set_stream_mode("torch_rocm")
    try:
        ct = ClientTrainer(None, model_0, None, Args(dev), None, None, None, None)
        got = ct.reconstruct(sums)
    finally:
        codec.set_stream_mode(old)
    # the reference's flow (fedkseed.py:132-141) with its own torch calls on the GPU
    ref = GPT2LMHeadModel(GPT2Config()).float().eval()
    ref.load_state_dict(model_0.state_dict())
    ref.to(dev)
    groups = get_optimizer_parameters_grouped_with_decay(ref, 0.01)
    params = [p for g in groups for p in g["params"]]
    for sd, g in sums.items():
        if g != 0.0:
            reference_step(params, sd, g, 1e-5, 0.01)
    torch.cuda.synchronize()
    gg = get_optimizer_parameters_grouped_with_decay(got, 0.01)
    for i, (a, b) in enumerate(zip([p for g in gg for p in g["params"]], params)):
        assert _differ(a.data.reshape(-1), b.data.reshape(-1)) == 0, f"tensor {i}"
