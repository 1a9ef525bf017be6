"""fp32 z of the CPU generator's stream under ATen's DEFAULT CPU capability -- the libm
flavour (FKS_LIBM; the kernels' kDtF32Libm): torch fills fp32 tensors of >= 16 elements with
normal_fill_16<float> and glibc's logf / sinf / cosf (DistributionTemplates.h:139-149)
instead of normal_fill_16_AVX2's Cephes functions when ATEN_CPU_CAPABILITY=default or the
host lacks AVX2 (csrc/fks_libm.h restates the three functions; tests/test_libm_float.py
checks them on every input of the path against the host's glibc).

* the reference's own stream drawn under that capability (tests/golden/normal_streams.npz
  "long_float32_default_capability", seed 2024, 2^18 elements);
* streams, reconstructs (the 19-seed kernel's full and partial passes, the small-K kernel,
  the irregular kernel's ragged tails), the perturbation and the seed-sharded delta against
  the oracle's CAP_DEFAULT restatement, with bf16 and short tensors in the same lists
  (whose z the flavour does not change);
* torch itself: a subprocess under ATEN_CPU_CAPABILITY=default, where the codec picks the
  flavour from torch's capability, runs the drop-in reconstruct_ and three zeroth-order
  steps on the GPU and the reference's loop and steps as torch ops on CPU tensors
  (oracle/torch_replica.py), bit for bit, generator state included.
"""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from conftest import assert_bitwise
from oracle import fks_oracle as O
from test_gpu_parity import DTC, TD, _dev, from_np, rand_params, to_np

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture
def libm():
    from fate_llm.algo.fedkseed import codec
    codec.set_cpu_fp32_flavour("libm")
    yield codec
    codec.set_cpu_fp32_flavour(None)


def test_golden_stream_drawn_under_default_capability(golden, libm):
    dev = _dev()
    ref = golden("normal_streams.npz")["long_float32_default_capability"]
    t = torch.empty(ref.size, dtype=torch.float32, device=dev)
    libm.normal_([t], 2024)
    assert_bitwise(to_np(t), ref, "float32", "long_float32_default_capability")
    # the flag is what changed it: the AVX flavour of the same seed is another stream
    libm.set_cpu_fp32_flavour("avx")
    libm.normal_([t], 2024)
    assert not np.array_equal(to_np(t), ref)


_MIXED = [(16, "float32"), (1000, "float32"), (64, "bfloat16"), (5, "float32"), (100003, "float32"),
          (624 * 3 + 16, "float32"), (17, "bfloat16"), (33, "float32"), (2**20, "float32"), (3, "bfloat16")]


@pytest.mark.parametrize("seed", [0, 7, 2**32 - 1, 2**40 + 3])
def test_streams_match_oracle(seed, libm):
    dev = _dev()
    ts = [torch.empty(n, dtype=TD[dt], device=dev) for n, dt in _MIXED]
    libm.normal_(ts, seed)
    gen = O.Generator(seed)
    for (n, dt), t in zip(_MIXED, ts):
        assert_bitwise(to_np(t), gen.normal(n, DTC[dt], O.CAP_DEFAULT), dt, f"seed {seed} n {n}")


_SHAPES = [4096, 1000, 7, 65536 + 16, 2**18, 40]


@pytest.mark.parametrize("k", [1, 3, 19, 45])
@pytest.mark.parametrize("wd", [None, 0.01, 0.0])
def test_reconstruct_matches_oracle(k, wd, libm):
    dev = _dev()
    arrays = rand_params(_SHAPES, "float32", seed=k)
    g = np.random.default_rng(k)
    seeds = [int(x) for x in g.integers(0, 2**32, k)]
    vals = [float(x) for x in g.standard_normal(k) * 20 + 0.5]
    lr = 1e-3
    ts = [from_np(a, "float32", dev) for a in arrays]
    specs = [libm.ParamSpec(t, lr=lr, weight_decay=wd) for t in ts]
    libm.directional_step(specs, seeds, vals)
    torch.cuda.synchronize()
    ref = [a.copy() for a in arrays]
    O.reconstruct(ref, [O.F32] * len(ref), [lr] * len(ref), [wd] * len(ref), seeds, vals, O.CAP_DEFAULT)
    for i, (t, r) in enumerate(zip(ts, ref)):
        assert_bitwise(to_np(t), r, "float32", f"k {k} wd {wd} tensor {i} (n {r.size})")


def test_reconstruct_mixed_dtypes_and_offset_views(libm):
    """fp32 beside bf16 in one call, an fp32 view at an odd element offset (the irregular
    kernel) and ragged sizes."""
    dev = _dev()
    base = torch.from_numpy(rand_params([70001], "float32", seed=5)[0]).to(dev)
    view = base[1:]  # 4-byte aligned, not 8: the irregular kernel's element pairs
    bf = from_np(rand_params([4096], "bfloat16", seed=6)[0], "bfloat16", dev)
    f2 = from_np(rand_params([3000], "float32", seed=7)[0], "float32", dev)
    seeds, vals = [11, 2**33 + 5, 99, 4], [1.5, -3.0, 0.25, 8.0]
    lr, wd = 1e-2, 0.01
    before = [to_np(view), to_np(bf), to_np(f2)]
    specs = [libm.ParamSpec(t, lr=lr, weight_decay=wd) for t in (view, bf, f2)]
    libm.directional_step(specs, seeds, vals)
    torch.cuda.synchronize()
    ref = [a.copy() for a in before]
    O.reconstruct(ref, [O.F32, O.BF16, O.F32], [lr] * 3, [wd] * 3, seeds, vals, O.CAP_DEFAULT)
    for name, t, r, dt in zip(("view", "bf16", "f32"), (view, bf, f2), ref, ("float32", "bfloat16", "float32")):
        assert_bitwise(to_np(t), r, dt, name)
    assert float(base[0]) == float(rand_params([70001], "float32", seed=5)[0][0])  # outside the view


def test_perturb_sequence_matches_oracle(libm):
    """optimizer.py:152-173 +1 / -2 / +1 with the same seed (the zeroth-order step)."""
    dev = _dev()
    arrays = rand_params(_SHAPES, "float32", seed=3)
    ts = [from_np(a, "float32", dev) for a in arrays]
    ref = [a.copy() for a in arrays]
    eps = 1e-3
    for sf in (1.0, -2.0, 1.0):
        libm.perturb(ts, 1234, [sf * eps] * len(ts))
        O.perturb_params(ref, [O.F32] * len(ref), 1234, sf * eps, O.CAP_DEFAULT)
        torch.cuda.synchronize()
        for i, (t, r) in enumerate(zip(ts, ref)):
            assert_bitwise(to_np(t), r, "float32", f"scale {sf} tensor {i}")


def test_delta_accumulate_matches_oracle(libm):
    """The seed-sharded variant's f32 delta on this flavour's z."""
    dev = _dev()
    arrays = rand_params(_SHAPES, "float32", seed=9)
    ts = [from_np(a, "float32", dev) for a in arrays]
    seeds = [5, 6, 2**32 + 9, 77, 123456]
    coefs = [1e-3, -2e-3, 5e-4, 3e-3, -1e-3]
    total = sum(a.size for a in arrays)
    delta = torch.zeros(total, dtype=torch.float32, device=dev)
    libm.delta_accumulate([libm.ParamSpec(t) for t in ts], seeds, coefs, delta)
    torch.cuda.synchronize()
    ref = np.zeros(total, np.float32)
    O.delta_accumulate([a.copy() for a in arrays], [O.F32] * len(arrays), seeds, coefs, ref,
                       capability=O.CAP_DEFAULT)
    assert_bitwise(delta.cpu().numpy(), ref, "float32", "delta")


_SCRIPT = r'''
import sys
sys.path.insert(0, "fate-llm_amd/python"); sys.path.insert(0, ".")
import torch
from fate_llm.algo.fedkseed import codec, zo_utils
from oracle import torch_replica as R
assert torch.backends.cpu.get_cpu_capability() == "DEFAULT"
assert codec.cpu_fp32_flavour() == "libm" and codec.get_stream_mode() == "torch_cpu"
g = torch.Generator().manual_seed(3)
init = [torch.randn(n, generator=g) * 0.02 for n in (4096, 1000, 7, 65552, 33)]
init.append((torch.randn(5000, generator=g) * 0.02).to(torch.bfloat16))  # bf16 draws the same z under either capability


def bits(t):
    return t.view(torch.int16 if t.element_size() == 2 else torch.int32)
seeds = [17, 2**32 + 1, 5, 90210]
vals = [2.0, -0.5, 0.0, 1.25]
lr, wd = 1e-3, 0.01
params = [torch.nn.Parameter(t.clone().cuda()) for t in init]
zo_utils.reconstruct_([{"params": params, "lr": 0.0, "weight_decay": 0.0}], seeds, vals, lr, wd)
got_state = torch.get_rng_state()
ref = [t.clone() for t in init]
R.reconstruct(ref, seeds, vals, lr, wd)  # the reference's loop: torch.normal on CPU tensors
for i, (p, r) in enumerate(zip(params, ref)):
    a, b = bits(p.detach().cpu()), bits(r)
    assert torch.equal(a, b), (i, int((a != b).sum()))
assert torch.equal(got_state, torch.get_rng_state()), "CPU generator"

# zeroth-order steps (perturb +1 / -2 / +1, then the update): the drop-in optimizer on the
# GPU copy against the reference's step on the CPU copy; the loss is a float64 sum taken on
# the CPU from the same bits on both sides
from fate_llm.algo.fedkseed.optimizer import ZerothOrderOptimizer
params_c = [torch.nn.Parameter(r.clone()) for r in ref]
def groups(ps):
    return [{"params": ps[:2], "weight_decay": 0.0, "lr": 1e-4, "eps": 1e-3},
            {"params": ps[2:], "weight_decay": 0.01, "lr": 1e-4, "eps": 1e-3}]
def closure_on(ps):
    return lambda: torch.stack([(p.detach().cpu().double() * (i + 1)).sum() for i, p in enumerate(ps)]).sum()
opt = ZerothOrderOptimizer(groups(params), lr=1e-4, eps=1e-3, weight_decay=0.01, grad_clip=0.0)
rg = groups(params_c)
for step, seed in enumerate([23, 2**35 + 1, 23]):
    g_ref, lr_ref, ll_ref = R.zeroth_order_step(rg, seed, closure_on(params_c), 1e-3)
    want = torch.get_rng_state()
    torch.manual_seed(999)  # the drop-in must move the generator itself
    g_got, lr_got, ll_got = opt.zeroth_order_step(seed, closure_on(params))
    assert float(lr_got) == float(lr_ref) and float(ll_got) == float(ll_ref) and float(g_got) == float(g_ref), step
    for i, (p, r) in enumerate(zip(params, params_c)):
        a, b = bits(p.detach().cpu()), bits(r.detach())
        assert torch.equal(a, b), (step, i, int((a != b).sum()))
    assert torch.equal(torch.get_rng_state(), want), f"step {step}: CPU generator"
# the same with the loss handed over as a device tensor (the optimizer's fused device path:
# perturb +1 / -2 on the GPU, g and the restore + update from device memory)
for step, seed in enumerate([41, 2**36 + 3]):
    g_ref, lr_ref, ll_ref = R.zeroth_order_step(rg, seed, closure_on(params_c), 1e-3)
    want = torch.get_rng_state()
    torch.manual_seed(998)
    g_got, lr_got, ll_got = opt.zeroth_order_step(seed, lambda: closure_on(params)().cuda())
    assert float(lr_got) == float(lr_ref) and float(ll_got) == float(ll_ref) and float(g_got) == float(g_ref), step
    for i, (p, r) in enumerate(zip(params, params_c)):
        a, b = bits(p.detach().cpu()), bits(r.detach())
        assert torch.equal(a, b), ("device loss", step, i, int((a != b).sum()))
    assert torch.equal(torch.get_rng_state(), want), f"device-loss step {step}: CPU generator"
print("ok")
'''


def test_torch_under_default_capability_subprocess():
    _dev()
    env = {k: v for k, v in os.environ.items() if k != "FKS_CPU_FP32_FLAVOUR"}
    env["ATEN_CPU_CAPABILITY"] = "default"
    env["FKS_STREAM_MODE"] = "torch_cpu"
    out = subprocess.run([sys.executable, "-c", _SCRIPT], cwd=ROOT, env=env, capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0 and out.stdout.strip().endswith("ok"), out.stdout[-2000:] + out.stderr[-4000:]
