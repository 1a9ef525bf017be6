"""C4 (BASELINE configs[3]): the fp32 path run as HBM-sized chunks of the parameter
stream (codec element shards processed one after another, tools/c4_70b.py), checked
against the oracle -- the reference's fp32 expression p - lr*(g*z + wd*p)
(zo_utils.py:47-49) with the AVX2 Cephes z stream -- through the FULL 19-seed fp32
kernel (K >= 20: one full pass plus a partial pass per call)."""
import os
import sys

import numpy as np
import pytest
import torch

from oracle import fks_oracle as O
from conftest import assert_bitwise
from test_gpu_parity import _dev, from_np, rand_params, to_np

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _seeds(k, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randint(0, 2**32, (k,), generator=g).tolist(), \
        (torch.randn(k, generator=g, dtype=torch.float64) * 20).tolist()


@pytest.mark.parametrize("nshards", [2, 3, 8])
def test_fp32_element_shards_match_oracle(nshards):
    from fate_llm.algo.fedkseed import codec
    dev = _dev()
    # regular tensors over many MT blocks, a ragged one (tail recompute), tiny ones
    # (serial draws), a phase-shifted tensor after the ragged one
    shapes = [624 * 64, 2**17, 1000, 5, 8, 4096 * 3 + 16, 19, 624 * 33]
    arrays = rand_params(shapes, "float32", seed=41)
    seeds, vals = _seeds(40, seed=42)
    lrs, wds = [1e-5] * len(shapes), [0.01] * len(shapes)
    ref = [a.copy() for a in arrays]
    O.reconstruct(ref, [O.F32] * len(ref), lrs, wds, seeds, vals)
    ts = [from_np(a, "float32", dev) for a in arrays]
    specs = [codec.ParamSpec(t, lr=1e-5, weight_decay=0.01) for t in ts]
    for r in range(nshards):
        codec.directional_step(specs, seeds, vals, shard=r, nshards=nshards)
    torch.cuda.synchronize()
    for i, (t, w) in enumerate(zip(ts, ref)):
        assert_bitwise(to_np(t), w, "float32", f"tensor {i}")


def test_c4_scaled_70b_layout_chunked():
    """The LLaMA-70B tensor list (723 tensors, rows scaled by 1/1024: 68M fp32 params,
    the 8192-element norms become 8-element tensors on the serial path) reconstructed
    in 8 chunks == one unchunked call, bit for bit, and its first tensors == the oracle."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import c4_70b
    from fate_llm.algo.fedkseed import codec
    dev = _dev()
    shapes = [(max(1, s[0] // 1024),) + tuple(s[1:]) for s in c4_70b.llama70b_shapes()]
    n = [int(np.prod(s)) for s in shapes]
    total = sum(n)
    flat = torch.empty(total, dtype=torch.float32, device=dev).normal_(0.0, 0.02,
                                                                       generator=torch.Generator(dev).manual_seed(0))
    clone = flat.clone()

    def views(buf):
        out, off = [], 0
        for s, m in zip(shapes, n):
            out.append(buf[off:off + m].view(s))
            off += m
        return out

    seeds, vals = _seeds(40, seed=43)
    vals[3] = 0.0
    keep = [(s, v) for s, v in zip(seeds, vals) if v != 0.0]
    ks, kv = [s for s, _ in keep], [v for _, v in keep]
    prefix = 6  # embedding + the first layer's projections
    ref = [flat[:sum(n[:prefix])].cpu().numpy()[sum(n[:i]):sum(n[:i + 1])].copy() for i in range(prefix)]
    specs = [codec.ParamSpec(v, lr=1e-5, weight_decay=0.01) for v in views(flat)]
    for c in range(8):
        codec.directional_step(specs, ks, kv, shard=c, nshards=8)
    codec.directional_step([codec.ParamSpec(v, lr=1e-5, weight_decay=0.01) for v in views(clone)], ks, kv)
    torch.cuda.synchronize()
    differ = int((flat.view(torch.int32) != clone.view(torch.int32)).sum().item())
    assert differ == 0, f"{differ} of {total} elements differ between chunked and unchunked"
    # the prefix tensors sit at the same stream positions as in the whole layout
    O.reconstruct(ref, [O.F32] * prefix, [1e-5] * prefix, [0.01] * prefix, ks, kv)
    got = flat[:sum(n[:prefix])].cpu().numpy()
    for i in range(prefix):
        assert_bitwise(got[sum(n[:i]):sum(n[:i + 1])], ref[i], "float32", f"tensor {i}")
