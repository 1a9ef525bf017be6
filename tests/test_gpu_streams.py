"""Stream ordering of the host side:

* ClientTrainer.materialize's staged H2D runs on a side stream; the destinations are
  allocated on the current stream, whose queued work may still write the memory's
  previous owner.  Materializing right after queueing such work -- no synchronisation
  between rounds -- must still give model_0's values (the side stream waits for the
  current stream first).
* The one-seed caches (the jumped-window cache and the caller-owned z-index buffer) are
  shared by every stream of a device.  Two streams interleaving zeroth-order-step calls
  with different seeds over two parameter lists, one stream held back by a device-side
  sleep (so a missing wait would let the other overtake it), plus a larger layout that
  makes both buffers grow while the first stream's calls are still queued, give the
  same bits as the same calls with both caches off.
* The device tail of zeroth_order_step takes exactly the losses the host path takes as
  a 0-dim tensor value; a shape-(1,) loss goes through the host path and is rejected
  there as it would be by the reference for a bf16 model (optimizer.py:147 rebinding
  param.data to f32).
"""
import copy
import os

import numpy as np
import pytest
import torch
from torch import nn

from test_gpu_parity import _dev, from_np, rand_params

pytestmark = pytest.mark.gpu


class _Net(nn.Module):
    def __init__(self):
        super().__init__()
        g = torch.Generator().manual_seed(11)
        self.a = nn.Parameter(torch.randn(9_000_000, generator=g) * 0.02)  # 36 MB: several DMA pieces
        self.b = nn.Parameter(torch.randn(1000, 64, generator=g) * 0.02)


class _Args:
    learning_rate = 1e-5
    weight_decay = 0.0

    def __init__(self, dev):
        self.device = dev


def test_materialize_after_queued_writes_no_sync():
    from fate_llm.algo.fedkseed.fedkseed import ClientTrainer
    dev = _dev()
    model_0 = _Net()
    want = {k: v.detach().clone() for k, v in model_0.state_dict().items()}
    ct = ClientTrainer(None, model_0, None, _Args(dev), None, None, None, None)
    for _ in range(3):
        # queue a long sleep and then a write into a buffer, free the buffer before the
        # write has run: its memory goes back to the current stream's pool at once
        junk = torch.empty(48_000_000, dtype=torch.uint8, device=dev)
        torch.cuda._sleep(200_000_000)
        junk.fill_(0x7F)
        del junk
        m = ct.materialize()  # no synchronisation since the queued write
        got = {k: v.detach().cpu() for k, v in m.state_dict().items()}
        for k in want:
            assert torch.equal(got[k], want[k]), k
        del m


def _zo_calls(views, specs, seed, g):
    from fate_llm.algo.fedkseed import codec
    codec.perturb(views, seed, 5e-4)
    codec.perturb(views, seed, -1e-3)
    codec.perturb_step(specs, seed, [5e-4] * len(specs), g)


def _two_stream_run(pa, pb, pc, dev):
    from fate_llm.algo.fedkseed import codec
    sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    spa = [codec.ParamSpec(p, lr=1e-3, weight_decay=0.0) for p in pa]
    spb = [codec.ParamSpec(p, lr=1e-3, weight_decay=None) for p in pb]
    spc = [codec.ParamSpec(p, lr=1e-3, weight_decay=0.01) for p in pc]
    cur = torch.cuda.current_stream(dev)
    sa.wait_stream(cur)
    sb.wait_stream(cur)
    for step in range(3):
        with torch.cuda.stream(sa):
            torch.cuda._sleep(50_000_000)  # stream a lags: its calls run after b's
            _zo_calls(pa, spa, 1000 + step, 2.5)
        with torch.cuda.stream(sb):
            _zo_calls(pb, spb, 2000 + step, -1.25)
            if step == 1:  # a larger layout: the window and z-index buffers grow
                _zo_calls(pc, spc, 3000, 0.5)
        with torch.cuda.stream(sa):
            codec.directional_step(spa, [2000 + step], [0.75])  # b's seed on a: a cache hit only if in order
    cur.wait_stream(sa)
    cur.wait_stream(sb)
    torch.cuda.synchronize()


def test_caches_two_streams_interleaved_match_uncached():
    from fate_llm.algo.fedkseed import _native as N
    from fate_llm.algo.fedkseed import codec
    dev = _dev()
    arr_a = rand_params([624 * 300, 4096, 48], "bfloat16", seed=1)
    arr_b = rand_params([624 * 200 + 16, 1000 * 16], "bfloat16", seed=2)
    arr_c = rand_params([624 * 2000, 2**16], "bfloat16", seed=3)
    out = {}
    for name, env in (("cached", {}), ("uncached", {"FKS_ZCACHE": "0", "FKS_NO_WIN_CACHE": "1"})):
        N.check(N.load().fks_plan_cache_clear())
        codec.zindex_release()
        os.environ.update(env)
        try:
            pa = [from_np(a, "bfloat16", dev) for a in arr_a]
            pb = [from_np(a, "bfloat16", dev) for a in arr_b]
            pc = [from_np(a, "bfloat16", dev) for a in arr_c]
            _two_stream_run(pa, pb, pc, dev)
            out[name] = [t.clone() for t in pa + pb + pc]
        finally:
            for key in env:
                os.environ.pop(key, None)
    for i, (x, y) in enumerate(zip(out["cached"], out["uncached"])):
        assert torch.equal(x.view(torch.int16), y.view(torch.int16)), f"tensor {i}"


def test_zindex_buffer_is_torch_memory_and_released():
    from fate_llm.algo.fedkseed import codec
    dev = _dev()
    codec.zindex_release()
    p = torch.zeros(624 * 1000, dtype=torch.bfloat16, device=dev)
    torch.cuda.synchronize()
    before = torch.cuda.memory_allocated(dev)
    codec.perturb([p], 5, 1e-3)
    torch.cuda.synchronize()
    grown = torch.cuda.memory_allocated(dev) - before
    assert grown >= p.numel(), "the z-index buffer (1 B per bf16 parameter) is not torch memory"
    codec.zindex_release()
    assert torch.cuda.memory_allocated(dev) - before < p.numel()
    # budget 0: no buffer, same values
    q = torch.zeros_like(p)
    old = codec.ZINDEX_BUDGET_FRAC
    codec.ZINDEX_BUDGET_FRAC = 0.0
    try:
        codec.perturb([q], 5, 1e-3)
    finally:
        codec.ZINDEX_BUDGET_FRAC = old
    assert torch.equal(p.view(torch.int16), q.view(torch.int16))


def test_zindex_skipped_when_memory_is_short_or_allocation_fails(monkeypatch):
    """The z-index buffer is a speed cache: a device short of free memory (headroom
    larger than what is free) or an allocation that raises OutOfMemoryError leaves it
    unattached and the perturb generates its z -- same values, no error."""
    from fate_llm.algo.fedkseed import codec
    dev = _dev()
    codec.zindex_release()
    p = torch.zeros(624 * 1000, dtype=torch.bfloat16, device=dev)
    codec.perturb([p], 9, 1e-3)
    codec.zindex_release()
    q, r = torch.zeros_like(p), torch.zeros_like(p)
    monkeypatch.setattr(codec, "ZINDEX_HEADROOM", 1 << 62)
    before = torch.cuda.memory_allocated(dev)
    codec.perturb([q], 9, 1e-3)
    assert torch.cuda.memory_allocated(dev) - before < p.numel()
    monkeypatch.setattr(codec, "ZINDEX_HEADROOM", 0)

    def oom(nbytes, device):
        raise torch.cuda.OutOfMemoryError("simulated")

    monkeypatch.setattr(codec, "_alloc_zindex", oom)
    assert codec.zindex_reserve(codec._Batch([codec.ParamSpec(r)])) is False
    codec.perturb([r], 9, 1e-3)
    torch.cuda.synchronize()
    assert torch.equal(p.view(torch.int16), q.view(torch.int16))
    assert torch.equal(p.view(torch.int16), r.view(torch.int16))


@pytest.mark.parametrize("shape,dtype", [((1,), torch.float32), ((), torch.float64)])
def test_device_tail_only_for_0dim_losses(shape, dtype):
    from fate_llm.algo.fedkseed.optimizer import ZerothOrderOptimizer
    dev = _dev()
    p = nn.Parameter(torch.zeros(4096, dtype=torch.bfloat16, device=dev))
    opt = ZerothOrderOptimizer([{"params": [p], "weight_decay": 0.0}], lr=1e-3, eps=5e-4, weight_decay=0.0,
                               grad_clip=-1.0)
    losses = iter([torch.full(shape, 2.5, dtype=dtype, device=dev), torch.full(shape, 2.25, dtype=dtype, device=dev)])
    if shape == (1,):
        with pytest.raises(NotImplementedError):
            opt.zeroth_order_step(7, lambda: next(losses))
    else:
        opt.zeroth_order_step(7, lambda: next(losses))
    assert not opt._last_step_on_device
