"""Pin the CPU oracle (oracle/) against the golden vectors captured from the reference.

The oracle is the checker for every GPU parity test, so it must itself reproduce the
reference bit for bit: MT19937 states, torch.normal z streams (fp32 AVX2 + libm
flavours, bf16, f16, f64, tail recompute, numel<16 serial path with its cached
sample), and the reconstruct / perturb / zeroth-order-step results of
fate_llm.algo.fedkseed (tests/golden/make_golden.py).
"""
import numpy as np
import pytest

from conftest import assert_bitwise

from oracle import fks_oracle as O

DTC = {"float32": O.F32, "bfloat16": O.BF16, "float16": O.F16, "float64": O.F64}


def test_mt_states(golden):
    g = golden("mt.npz")
    i = 0
    for s in g["seeds"]:
        for n in g["draws"]:
            gen = O.Generator(int(s))
            gen.u32(int(n))
            assert np.array_equal(gen.state_words(), g["states"][i]), (s, n)
            left, nxt = gen.left_next()
            assert left == g["left"][i] and nxt == g["next"][i]
            i += 1


def test_random64_high_word_first(golden):
    g = golden("mt.npz")
    for s, ref in zip(g["seeds"], g["random64_mod63"]):
        gen = O.Generator(int(s))
        got = [gen.random64() % (1 << 63) for _ in range(len(ref))]
        assert got == [int(x) for x in ref]


@pytest.mark.parametrize("dtype", list(DTC))
def test_sequential_streams(golden, dtype):
    g = golden("normal_streams.npz")
    for s in g["seeds"]:
        gen = O.Generator(int(s))
        got = np.concatenate([gen.normal(int(n), DTC[dtype]) for n in g["shapes"]])
        ref = g[f"seq_{dtype}_{int(s)}"]
        assert got.dtype == ref.dtype
        assert np.array_equal(got.view(np.uint8), ref.view(np.uint8)), (dtype, s)


@pytest.mark.parametrize("dtype,key,cap", [
    ("float32", "long_float32", O.CAP_AVX2),
    ("bfloat16", "long_bfloat16", O.CAP_AVX2),
    ("float16", "long_float16", O.CAP_AVX2),
    ("float32", "long_float32_default_capability", O.CAP_DEFAULT),
])
def test_long_streams_bitwise(golden, dtype, key, cap):
    ref = golden("normal_streams.npz")[key]
    got = O.Generator(2024).normal(ref.size, DTC[dtype], cap)
    assert np.array_equal(got.view(np.uint8), ref.view(np.uint8))


def test_bf16_stream_covers_box_muller_table(golden):
    """Every (u1, u2) byte pair the bf16 tables can see occurs in the pinned long stream."""
    ref = golden("normal_streams.npz")["long_bfloat16"]
    gen = O.Generator(2024)
    u = gen.u32(ref.size) & 0xFF
    blocks = u.reshape(-1, 16)
    pairs = (blocks[:, :8].astype(np.int64) << 8) | blocks[:, 8:]
    assert np.unique(pairs).size > 65536 - 64


def resolve_lr_wd(groups_wd, groups_lr, lr, wd, ngroups_tensors):
    """zo_utils.py:43-45 sticky resolution, restated for the checker."""
    out = []
    for gi, n in enumerate(ngroups_tensors):
        wd = groups_wd[gi] if wd is None else wd
        lr = groups_lr[gi] if lr is None else lr
        out.extend([(lr, wd)] * n)
    return out


@pytest.mark.parametrize("name", [
    "f32_wd", "f32_nowd", "bf16_wd", "bf16_nowd", "f16_wd", "f32_ragged", "bf16_ragged",
    "f32_sticky", "bf16_sticky", "f32_edge", "bf16_nan", "f32_k4096", "bf16_k4096", "f32_wdnone"])
def test_reconstruct_cases(golden, cases, name):
    case = cases["reconstruct"][name]
    z = golden(f"reconstruct_{name}.npz")
    order = [n for grp in case["groups"] for n in grp]
    lrwd = resolve_lr_wd(case["group_wd"], case["group_lr"],
                         None if case["sticky"] else case["lr"],
                         None if case["sticky"] else case["wd"],
                         [len(grp) for grp in case["groups"]])
    arrays = [z[f"init/{n}"].copy().reshape(-1) for n in order]
    dt = DTC[case["dtype"]]
    O.reconstruct(arrays, [dt] * len(arrays), [a for a, _ in lrwd], [b for _, b in lrwd],
                  z["seeds"], z["scalars"])
    for n, a in zip(order, arrays):
        assert_bitwise(a, z[f"final/{n}"], case["dtype"], f"{name}/{n}")


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
def test_perturb_and_zo_step(golden, cases, dtype):
    case = cases["optimizer"][dtype]
    z = golden(f"optimizer_{dtype}.npz")
    order = [n for grp in case["groups"] for n in grp]
    live = [n for n in order if case["requires_grad"][n]]
    arrays = {n: z[f"s0/{n}"].copy().reshape(-1) for n in order}
    dt = DTC[dtype]
    for step, sf in enumerate((1.0, -2.0, 1.0), start=1):
        O.perturb_params([arrays[n] for n in live], [dt] * len(live), case["perturb_seed"], sf * case["eps"])
        for n in order:
            assert_bitwise(arrays[n], z[f"s{step}/{n}"], dtype, f"step{step}/{n}")
    # zeroth_order_step: +1, -2, +1 perturbs then the K=1 update with sticky lr/wd
    for sf in (1.0, -2.0, 1.0):
        O.perturb_params([arrays[n] for n in live], [dt] * len(live), case["step_seed"], sf * case["eps"])
    lo, hi = case["losses"]
    g = float(np.float32(np.float32(lo) - np.float32(hi)) / np.float32(2 * case["eps"]))
    assert g == pytest.approx(float(z["g"][0]), rel=0, abs=0)
    if dtype == "bfloat16":
        # g is a 0-dim fp32 tensor here and the FIRST operand of `g * z` (zo_utils.py:49):
        # TensorIterator casts it to the common dtype (bf16) before the multiply.
        # (A python-float g, as in train_once, is the second operand of mul and stays fp32.)
        g = float((np.array([g], np.float32).view(np.uint32) + 0x7FFF + ((np.array([g], np.float32).view(np.uint32) >> 16) & 1)
                   >> 16 << 16).view(np.float32)[0])
    # sticky: group 0 (no-decay) wd 0.0 sticks for every group; lr from the optimizer defaults
    ts = [arrays[n] for n in order]
    O.reconstruct(ts, [dt] * len(ts), [case["lr"]] * len(ts), [0.0] * len(ts), [case["step_seed"]], [g])
    for n in order:
        assert_bitwise(arrays[n], z[f"s4/{n}"], dtype, f"zo_step/{n}")
