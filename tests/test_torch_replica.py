"""The CPU baseline's replica of the reference arithmetic (oracle/torch_replica.py,
bench.py's cpu_baseline leg) computes what the reference computes: bit-exact against
the pinned oracle for bf16 and fp32 at weight decay 0.01, 0.0 and None -- the None
branch is zo_utils.py:50-52 (no decay term), the others :48-49."""
import numpy as np
import pytest
import torch

from conftest import assert_bitwise
from oracle import fks_oracle as O
from oracle import torch_replica as R


@pytest.mark.parametrize("dtype,code", [(torch.bfloat16, O.BF16), (torch.float32, O.F32)])
@pytest.mark.parametrize("wd", [0.01, 0.0, None])
def test_replica_matches_oracle(dtype, code, wd):
    g = torch.Generator().manual_seed(5)
    init = [(torch.randn(n, generator=g) * 0.02).to(dtype) for n in (4096, 48, 1000)]
    seeds = torch.randint(0, 2**32, (6,), generator=g).tolist()
    vals = (torch.randn(6, generator=g, dtype=torch.float64) * 20).tolist()
    vals[2] = 0.0  # skipped by the replica's loop, as fedkseed.py:137

    params = [t.clone() for t in init]
    assert R.reconstruct(params, seeds, vals, 1e-3, wd) == 5

    def bits(t):
        t = t.contiguous()
        return t.view(torch.int16).numpy().view(np.uint16).copy() if t.dtype == torch.bfloat16 else t.numpy().copy()

    ref = [bits(t) for t in init]
    keep = [(s, v) for s, v in zip(seeds, vals) if v != 0.0]
    O.reconstruct(ref, [code] * 3, [1e-3] * 3, [wd] * 3, [s for s, _ in keep], [v for _, v in keep])
    name = "bfloat16" if dtype == torch.bfloat16 else "float32"
    for i, (p, r) in enumerate(zip(params, ref)):
        assert_bitwise(bits(p), r, name, f"tensor {i}")
