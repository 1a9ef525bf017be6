"""GPU parity of the HIP product path (libfks.so through the drop-in API) against the
CPU oracle and the reference's golden vectors.

Bar: bit-exact (NaN matches NaN) for fp32 and bf16 -- the z stream is integer/table
work plus op-for-op restated float arithmetic, so there is nothing to tolerate.
"""
import numpy as np
import pytest
import torch

from conftest import as_float, assert_bitwise
from oracle import fks_oracle as O

pytestmark = pytest.mark.gpu

DTC = {"float32": O.F32, "bfloat16": O.BF16, "float16": O.F16}
TD = {"float32": torch.float32, "bfloat16": torch.bfloat16, "float16": torch.float16}


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda", 0)


def to_np(t: torch.Tensor) -> np.ndarray:
    """bits as stored in the golden files: uint16 for bf16/f16, float32 for f32"""
    t = t.detach().contiguous().cpu()
    if t.dtype in (torch.bfloat16, torch.float16):
        return t.view(torch.int16).numpy().view(np.uint16).copy()
    return t.numpy().copy()


def from_np(a: np.ndarray, dtype: str, dev) -> torch.Tensor:
    if dtype in ("bfloat16", "float16"):
        return torch.from_numpy(a.view(np.int16).copy()).view(TD[dtype]).to(dev)
    return torch.from_numpy(a.copy()).to(dev)


def rand_params(shapes, dtype, seed=0):
    g = torch.Generator().manual_seed(seed)
    return [to_np((torch.randn(n, generator=g) * 0.02).to(TD[dtype])) for n in shapes]


# ----------------------------------------------------------------------------- z streams
@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
@pytest.mark.parametrize("seed", [0, 7, 2**32 - 1, 3141592653, 2**40 + 3])
def test_normal_stream_matches_oracle(dtype, seed):
    from fate_llm.algo.fedkseed import codec
    dev = _dev()
    shapes = [16, 64, 624, 1248, 4096, 100000, 32, 2**18 + 48]
    ts = [torch.empty(n, dtype=TD[dtype], device=dev) for n in shapes]
    codec.normal_(ts, seed)
    gen = O.Generator(seed)
    for n, t in zip(shapes, ts):
        assert_bitwise(to_np(t), gen.normal(n, DTC[dtype]), dtype, f"seed {seed} n {n}")


@pytest.mark.parametrize("dtype,key", [("float32", "long_float32"), ("bfloat16", "long_bfloat16")])
def test_normal_stream_matches_golden(golden, dtype, key):
    from fate_llm.algo.fedkseed import codec
    dev = _dev()
    ref = golden("normal_streams.npz")[key]
    t = torch.empty(ref.size, dtype=TD[dtype], device=dev)
    codec.normal_([t], 2024)
    assert_bitwise(to_np(t), ref, dtype, key)


# ----------------------------------------------------------------------------- reconstruct
def _gpu_reconstruct(arrays, dtype, lrs, wds, seeds, scalars, tensor_value=False):
    from fate_llm.algo.fedkseed import codec
    dev = _dev()
    ts = [from_np(a, dtype, dev) for a in arrays]
    specs = [codec.ParamSpec(t, lr=lr, weight_decay=wd) for t, lr, wd in zip(ts, lrs, wds)]
    codec.directional_step(specs, list(seeds), list(scalars), value_is_tensor=tensor_value)
    torch.cuda.synchronize()
    return [to_np(t) for t in ts]


ALL_CASES = ["f32_wd", "f32_nowd", "bf16_wd", "bf16_nowd", "f16_wd", "f32_ragged", "bf16_ragged", "f32_sticky",
             "bf16_sticky", "f32_edge", "bf16_nan", "f32_k4096", "bf16_k4096", "f32_wdnone"]


@pytest.mark.parametrize("name", ALL_CASES)
def test_reconstruct_golden(golden, cases, name):
    """The train_once reconstruct loop through the drop-in zo_utils, vs the reference."""
    from fate_llm.algo.fedkseed import zo_utils
    dev = _dev()
    case = cases["reconstruct"][name]
    z = golden(f"reconstruct_{name}.npz")
    order = [n for grp in case["groups"] for n in grp]
    dt = case["dtype"]
    params = {n: torch.nn.Parameter(from_np(z[f"init/{n}"].reshape(-1), dt, dev)) for n in order}
    groups = [{"params": [params[n] for n in grp], "weight_decay": wd, "lr": lr}
              for grp, wd, lr in zip(case["groups"], case["group_wd"], case["group_lr"])]
    if case["sticky"]:
        for s, g in zip(z["seeds"].tolist(), z["scalars"].tolist()):
            if g != 0.0:
                zo_utils.directional_derivative_step(groups, int(s), g)
    else:
        zo_utils.reconstruct_(groups, z["seeds"].tolist(), z["scalars"].tolist(), lr=case["lr"],
                              weight_decay=case["wd"])
    torch.cuda.synchronize()
    for n in order:
        assert_bitwise(to_np(params[n].data), z[f"final/{n}"], dt, f"{name}/{n}")


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
def test_reconstruct_multichunk_vs_oracle(dtype):
    """4M params in 7 tensors, K=61 (three seed passes), ~512 chunks: every chunk start is a
    GF(2) jump; the full result must equal the oracle's sequential reconstruct bit for bit."""
    shapes = [2**20, 48, 1234 * 16, 2**21, 4096 * 3, 16, 2**19 + 4096]
    arrays = rand_params(shapes, dtype, seed=1)
    gg = torch.Generator().manual_seed(5)
    seeds = torch.randint(0, 2**32, (61,), generator=gg).tolist()
    vals = (torch.randn(61, generator=gg, dtype=torch.float64) * 20).tolist()
    lrs = [1e-3] * len(shapes)
    wds = [0.01, 0.0, 0.01, None, 0.01, 0.01, 0.0]
    got = _gpu_reconstruct(arrays, dtype, lrs, wds, seeds, vals)
    O.reconstruct(arrays, [DTC[dtype]] * len(arrays), lrs, wds, seeds, vals)
    for i, (a, b) in enumerate(zip(got, arrays)):
        assert_bitwise(a, b, dtype, f"tensor {i}")


def test_mixed_dtype_stream():
    """fp32 and bf16 tensors interleaved in one stream: each dtype pass must keep the
    other dtype's stream positions."""
    from fate_llm.algo.fedkseed import codec
    dev = _dev()
    shapes = [4096, 624 * 16, 2**16, 160, 2**15]
    dts = ["float32", "bfloat16", "float32", "bfloat16", "bfloat16"]
    arrays = [rand_params([n], d, seed=i)[0] for i, (n, d) in enumerate(zip(shapes, dts))]
    seeds, vals = [11, 22, 33], [3.5, -7.25, 100.0]
    ts = [from_np(a, d, dev) for a, d in zip(arrays, dts)]
    specs = [codec.ParamSpec(t, lr=1e-3, weight_decay=0.01) for t in ts]
    codec.directional_step(specs, seeds, vals)
    O.reconstruct(arrays, [DTC[d] for d in dts], [1e-3] * 5, [0.01] * 5, seeds, vals)
    for i, (t, a, d) in enumerate(zip(ts, arrays, dts)):
        assert_bitwise(to_np(t), a, d, f"tensor {i}")


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
def test_edge_values(dtype):
    """Denormals, zeros of both signs, infinities and NaNs in the parameters; huge,
    tiny, negative-zero and NaN directional values."""
    n = 4096
    base = rand_params([n], dtype, seed=3)[0]
    f = as_float(base, dtype).astype(np.float32)
    f[:8] = [0.0, -0.0, np.inf, -np.inf, np.nan, 1e-40, -1e-39, 3e38]
    f[8:16] = np.float32(1.2e-38) * np.arange(8, dtype=np.float32)
    arr = f if dtype == "float32" else to_np(torch.from_numpy(f).to(torch.bfloat16))
    seeds = [1, 2, 3, 4, 5, 6]
    vals = [1e30, -0.0, 1e-45, float("nan"), 5.0, -3e38]
    got = _gpu_reconstruct([arr], dtype, [1e-2], [0.5], seeds, vals)
    O.reconstruct([arr], [DTC[dtype]], [1e-2], [0.5], seeds, vals)
    assert_bitwise(got[0], arr, dtype, "edge")


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
@pytest.mark.parametrize("wd", [0.0, -0.0])
@pytest.mark.parametrize("k", [1, 3, 24, 40])
def test_zero_weight_decay_edge_values(dtype, wd, k):
    """weight_decay = +-0.0 (the HF default the reference's ClientTrainer passes) runs the
    kModeUpdateWd0 chain, t = fma(wd, p, g*z) in place of rnd(g*z + rnd(wd*p)): it must keep
    the reference's bits for zeros of both signs, infinities (inf*0 = NaN), NaNs and
    denormals, with negative, tiny (g*z underflows to -0) and huge directional values.
    K = 1, 3 take the small-K kernel, 24 / 40 the 19-seed fp32 or the 32-seed bf16 slice
    kernel (one full pass and a partial one)."""
    n = 64 * 1024
    base = rand_params([n], dtype, seed=4)[0]
    f = as_float(base, dtype).astype(np.float32)
    f[:8] = [0.0, -0.0, np.inf, -np.inf, np.nan, 1e-40, -1e-39, 3e38]
    f[8:16] = np.float32(-1.2e-38) * np.arange(8, dtype=np.float32)
    f[5000:5016] = -0.0
    f[7000:7016] = 0.0
    arr = f if dtype == "float32" else to_np(torch.from_numpy(f).to(torch.bfloat16))
    gg = torch.Generator().manual_seed(17 + k)
    seeds = torch.randint(0, 2**32, (k,), generator=gg).tolist()
    vals = (torch.randn(k, generator=gg, dtype=torch.float64) * 20).tolist()
    edge = [-1e-45, 1e-45, -3e38, -5.0, 1e30, -0.5]
    for i in range(1, min(k, len(edge) + 1)):  # seed 0 keeps an ordinary value
        vals[i] = edge[i - 1]
    got = _gpu_reconstruct([arr], dtype, [1e-2], [wd], seeds, vals)
    O.reconstruct([arr], [DTC[dtype]], [1e-2], [wd], seeds, vals)
    assert_bitwise(got[0], arr, dtype, f"wd {wd} k {k}")
    # the specialised chain must have changed something besides the edge values
    assert not np.array_equal(got[0][16:4096], base[16:4096])


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
def test_tensor_valued_step_rounds_value_to_param_dtype(dtype):
    """zeroth_order_step passes g as a 0-dim fp32 tensor, the FIRST operand of g*z: torch
    casts it to the parameter dtype first (bf16 rounding)."""
    arr = rand_params([2048], dtype, seed=4)[0]
    g = float(np.float32(0.125) / np.float32(2 * 5e-4))
    got = _gpu_reconstruct([arr], dtype, [1e-3], [0.0], [12345678], [g], tensor_value=True)
    gg = g
    if dtype == "bfloat16":
        gg = float(torch.tensor(g, dtype=torch.float32).to(torch.bfloat16).float())
    O.reconstruct([arr], [DTC[dtype]], [1e-3], [0.0], [12345678], [gg])
    assert_bitwise(got[0], arr, dtype, "tensor-valued g")


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
def test_perturb_sequence_vs_oracle(dtype):
    """+1, -2, +1 perturbations (optimizer.py:128-136) on a regular layout, and the
    per-group eps (mixed scales) path."""
    from fate_llm.algo.fedkseed import codec
    dev = _dev()
    shapes = [4800, 48, 48, 6912, 144, 6912, 48, 48]
    arrays = rand_params(shapes, dtype, seed=6)
    ts = [from_np(a, dtype, dev) for a in arrays]
    eps = 5e-4
    for sf in (1.0, -2.0, 1.0):
        codec.perturb(ts, 987654321, sf * eps)
        O.perturb_params(arrays, [DTC[dtype]] * len(arrays), 987654321, sf * eps)
        for i, (t, a) in enumerate(zip(ts, arrays)):
            assert_bitwise(to_np(t), a, dtype, f"sf {sf} tensor {i}")
    scales = [1e-3 if i % 2 else 5e-4 for i in range(len(ts))]
    codec.perturb(ts, 42, scales)
    gen = O.Generator(42)
    for i, (t, a) in enumerate(zip(ts, arrays)):
        zz = gen.normal(a.size, DTC[dtype])
        O.perturb(a, zz, DTC[dtype], scales[i])
        assert_bitwise(to_np(t), a, dtype, f"mixed-eps tensor {i}")


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
def test_zeroth_order_optimizer_golden(golden, cases, dtype):
    """ZerothOrderOptimizer on the ragged TinyLM (tiny, ragged and 7-element tensors, a
    frozen tensor kept in its group): three perturbations, then zeroth_order_step with
    pre-set losses -- every snapshot bit-exact against the reference run."""
    from fate_llm.algo.fedkseed.optimizer import ZerothOrderOptimizer
    dev = _dev()
    case = cases["optimizer"][dtype]
    z = golden(f"optimizer_{dtype}.npz")
    order = [n for grp in case["groups"] for n in grp]
    params = {n: torch.nn.Parameter(from_np(z[f"s0/{n}"].reshape(-1), dtype, dev),
                                    requires_grad=case["requires_grad"][n]) for n in order}
    groups = [{"params": [params[n] for n in grp], "weight_decay": wd}
              for grp, wd in zip(case["groups"], (0.0, case["wd"]))]
    opt = ZerothOrderOptimizer(groups, lr=case["lr"], eps=case["eps"], weight_decay=case["wd"], grad_clip=-100.0)
    for step, sf in enumerate((1.0, -2.0, 1.0), start=1):
        opt.random_perturb_parameters(case["perturb_seed"], scaling_factor=sf)
        torch.cuda.synchronize()
        for n in order:
            assert_bitwise(to_np(params[n].data), z[f"s{step}/{n}"], dtype, f"perturb {step}/{n}")
    losses = iter([torch.tensor(x) for x in case["losses"]])
    g, _, _ = opt.zeroth_order_step(case["step_seed"], lambda: next(losses))
    torch.cuda.synchronize()
    assert float(g) == float(z["g"][0])
    for n in order:
        assert_bitwise(to_np(params[n].data), z[f"s4/{n}"], dtype, f"zo step/{n}")


# ----------------------------------------------------------------------------- irregular layouts
IRREGULAR_SHAPES = [3, 48, 7, 185, 37, 5, 1, 336, 1, 15, 17, 624 * 2 + 5, 2, 4096, 13, 31, 16, 9]


@pytest.mark.parametrize("dtype", ["float32", "bfloat16", "float16"])
def test_irregular_layout_vs_oracle(dtype):
    """Tiny tensors (serial double path with the cached sample carried across tensors),
    ragged tensors (tail recompute), tensors at odd stream phases and 16-aligned ones
    interleaved; K=23 covers a full and a partial seed pass."""
    shapes = IRREGULAR_SHAPES
    arrays = rand_params(shapes, dtype, seed=7)
    gg = torch.Generator().manual_seed(8)
    seeds = torch.randint(0, 2**32, (23,), generator=gg).tolist()
    vals = (torch.randn(23, generator=gg, dtype=torch.float64) * 20).tolist()
    lrs = [1e-3] * len(shapes)
    wds = [0.01 if i % 3 else 0.0 for i in range(len(shapes))]
    wds[4] = None
    got = _gpu_reconstruct(arrays, dtype, lrs, wds, seeds, vals)
    O.reconstruct(arrays, [DTC[dtype]] * len(arrays), lrs, wds, seeds, vals)
    for i, (a, b) in enumerate(zip(got, arrays)):
        assert_bitwise(a, b, dtype, f"tensor {i} (numel {shapes[i]})")


@pytest.mark.parametrize("dtype", ["float32", "bfloat16", "float16"])
def test_irregular_normal_stream_vs_oracle(dtype):
    """z itself (torch.normal per tensor, one seed) over the irregular layout."""
    from fate_llm.algo.fedkseed import codec
    dev = _dev()
    ts = [torch.empty(n, dtype=TD[dtype], device=dev) for n in IRREGULAR_SHAPES]
    codec.normal_(ts, 2718281828)
    gen = O.Generator(2718281828)
    for n, t in zip(IRREGULAR_SHAPES, ts):
        assert_bitwise(to_np(t), gen.normal(n, DTC[dtype]), dtype, f"n {n}")


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
def test_phase_shifted_large_tensor_multichunk(dtype):
    """A 5-element tensor first shifts every later tensor to stream phase 12: 1.5M params
    on the irregular kernel across many chunks, every chunk start a GF(2) jump."""
    shapes = [5, 2**20 + 2**19, 40, 2**16]
    arrays = rand_params(shapes, dtype, seed=9)
    seeds, vals = [5, 6, 7], [1.5, -2.5, 30.0]
    got = _gpu_reconstruct(arrays, dtype, [1e-3] * 4, [0.01] * 4, seeds, vals)
    O.reconstruct(arrays, [DTC[dtype]] * 4, [1e-3] * 4, [0.01] * 4, seeds, vals)
    for i, (a, b) in enumerate(zip(got, arrays)):
        assert_bitwise(a, b, dtype, f"tensor {i}")


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
def test_odd_element_offsets(dtype):
    """Views of one flat buffer at odd element offsets (the fast kernel moves aligned
    element pairs; these go through the irregular kernel)."""
    from fate_llm.algo.fedkseed import codec
    dev = _dev()
    shapes = [4096, 160, 2**15]
    arrays = rand_params(shapes, dtype, seed=10)
    flat = torch.zeros(1 + sum(shapes) + 3, dtype=TD[dtype], device=dev)
    views, off = [], 1
    for a in arrays:
        v = flat[off:off + a.size]
        v.copy_(from_np(a, dtype, dev))
        views.append(v)
        off += a.size + 1
    specs = [codec.ParamSpec(v, lr=1e-3, weight_decay=0.01) for v in views]
    codec.directional_step(specs, [77, 78], [2.0, -3.0])
    O.reconstruct(arrays, [DTC[dtype]] * 3, [1e-3] * 3, [0.01] * 3, [77, 78], [2.0, -3.0])
    for i, (v, a) in enumerate(zip(views, arrays)):
        assert_bitwise(to_np(v), a, dtype, f"view {i}")


@pytest.mark.parametrize("nshards", [2, 3, 8])
def test_element_shards_equal_whole(nshards):
    """Element sharding (what each rank of bench.py / the N-GPU reconstruct runs): the
    union of all shards equals the unsharded reconstruct bit for bit, irregular work
    included."""
    from fate_llm.algo.fedkseed import codec
    dev = _dev()
    shapes = [2**18, 37, 3, 2**16 + 16, 185, 624 * 40]
    arrays = rand_params(shapes, "bfloat16", seed=11)
    seeds, vals = list(range(100, 125)), [float(i) - 12.5 for i in range(25)]
    whole = _gpu_reconstruct(arrays, "bfloat16", [1e-3] * 6, [0.01] * 6, seeds, vals)
    ts = [from_np(a, "bfloat16", dev) for a in arrays]
    specs = [codec.ParamSpec(t, lr=1e-3, weight_decay=0.01) for t in ts]
    for r in range(nshards):
        codec.directional_step(specs, seeds, vals, shard=r, nshards=nshards)
    torch.cuda.synchronize()
    for i, (t, w) in enumerate(zip(ts, whole)):
        assert_bitwise(to_np(t), w, "bfloat16", f"tensor {i}")


@pytest.mark.parametrize("dtype", ["float32", "bfloat16", "float16"])
def test_fused_restore_and_step_vs_oracle(dtype):
    """codec.perturb_step (restore perturbation + directional step in one pass) equals
    the reference's two separate steps, on regular and irregular tensors, with a
    0-dim-tensor g (rounded to the parameter dtype first)."""
    from fate_llm.algo.fedkseed import codec
    dev = _dev()
    shapes = [4800, 48, 7, 185, 6912, 3, 37, 144]
    arrays = rand_params(shapes, dtype, seed=12)
    ts = [from_np(a, dtype, dev) for a in arrays]
    lrs = [1e-3] * len(shapes)
    wds = [0.0 if i % 2 else 0.01 for i in range(len(shapes))]
    specs = [codec.ParamSpec(t, lr=lr, weight_decay=wd) for t, lr, wd in zip(ts, lrs, wds)]
    eps, seed = 5e-4, 24681357
    g = float(np.float32(0.125) / np.float32(2 * eps))
    codec.perturb_step(specs, seed, [eps] * len(ts), g, value_is_tensor=True, update=True)
    torch.cuda.synchronize()
    O.perturb_params(arrays, [DTC[dtype]] * len(arrays), seed, eps)
    gg = float(torch.tensor(g, dtype=torch.float32).to(TD[dtype]).float())
    O.reconstruct(arrays, [DTC[dtype]] * len(arrays), lrs, wds, [seed], [gg])
    for i, (t, a) in enumerate(zip(ts, arrays)):
        assert_bitwise(to_np(t), a, dtype, f"tensor {i}")


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
def test_zeroth_order_step_fused_equals_unfused(dtype):
    """ZerothOrderOptimizer.zeroth_order_step takes the fused path when every grouped
    parameter requires grad; the result equals the reference sequence (perturb +1, -2,
    +1 with the oracle, then the update)."""
    from fate_llm.algo.fedkseed.optimizer import ZerothOrderOptimizer
    dev = _dev()
    shapes = [4800, 48, 48, 6912, 144, 7, 37]
    arrays = rand_params(shapes, dtype, seed=13)
    params = [torch.nn.Parameter(from_np(a, dtype, dev)) for a in arrays]
    groups = [{"params": params[:3], "weight_decay": 0.0}, {"params": params[3:], "weight_decay": 0.01}]
    opt = ZerothOrderOptimizer(groups, lr=1e-3, eps=5e-4, weight_decay=0.01, grad_clip=-100.0)
    assert opt._fusable()
    losses = iter([torch.tensor(2.5), torch.tensor(2.375)])
    g, _, _ = opt.zeroth_order_step(777, lambda: next(losses))
    torch.cuda.synchronize()
    for sf in (1.0, -2.0, 1.0):
        O.perturb_params(arrays, [DTC[dtype]] * len(arrays), 777, sf * 5e-4)
    gv = float(g)
    if dtype == "bfloat16":
        gv = float(torch.tensor(gv, dtype=torch.float32).to(torch.bfloat16).float())
    # sticky: group 0's wd (0.0) and the optimizer lr stick for every tensor
    O.reconstruct(arrays, [DTC[dtype]] * len(arrays), [1e-3] * len(arrays), [0.0] * len(arrays), [777], [gv])
    for i, (p, a) in enumerate(zip(params, arrays)):
        assert_bitwise(to_np(p.data), a, dtype, f"tensor {i}")


def test_cpu_tensors_rejected():
    from fate_llm.algo.fedkseed import codec
    _dev()
    with pytest.raises(ValueError):
        codec.normal_([torch.empty(32)], 1)
