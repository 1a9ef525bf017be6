"""One process, two GPUs: the bf16 / f16 tables (__constant__, per device), the kernels'
LDS attributes, the plan cache (keyed by device) and the one-seed window cache are set
up per device -- a reconstruct and a perturb on cuda:1 after the same calls on cuda:0
give the oracle's values on both.  Skipped on a one-GPU box."""
import numpy as np
import pytest
import torch

from conftest import assert_bitwise
from oracle import fks_oracle as O
from test_gpu_parity import DTC, from_np, rand_params, to_np

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", ["bfloat16", "float16"])
def test_same_calls_on_two_devices(dtype):
    if not torch.cuda.is_available() or torch.cuda.device_count() < 2:
        pytest.skip("needs two HIP devices")
    from fate_llm.algo.fedkseed import codec
    shapes = [4096 * 2, 1000, 33]
    arrays = rand_params(shapes, dtype, seed=81)
    seeds = [101, 202, 303, 404, 505] * 5  # 25 seeds: a 19-seed pass and a small one
    vals = [float(np.float32(0.5 + i / 7)) for i in range(len(seeds))]
    want = [a.copy() for a in arrays]
    O.reconstruct(want, [DTC[dtype]] * len(want), [1e-3] * len(want), [0.01] * len(want), seeds, vals)
    O.perturb_params(want, [DTC[dtype]] * len(want), 777, 5e-4)
    for d in (0, 1):
        dev = torch.device("cuda", d)
        params = [from_np(a, dtype, dev) for a in arrays]
        specs = [codec.ParamSpec(p, lr=1e-3, weight_decay=0.01) for p in params]
        codec.directional_step(specs, seeds, vals)
        codec.perturb(params, 777, 5e-4)
        torch.cuda.synchronize(dev)
        for i, (p, w) in enumerate(zip(params, want)):
            assert_bitwise(to_np(p), w, dtype, f"cuda:{d} tensor {i}")
