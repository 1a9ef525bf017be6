"""The torch_rocm z stream (FKS_STREAM_ROCM): a reference client whose model sits on a GPU
draws z on the device (zo_utils.py:47 and optimizer.py:170-172 pass
``device=param.data.device``), i.e. torch's HIP generator -- Philox4x32-10 with rocrand's
Box-Muller in torch's grid-stride mapping (ATen/native/cuda/DistributionTemplates.h).
The oracle for this stream is torch itself on the same GPU (the installed PyTorch-ROCm,
not the reference): after torch.manual_seed(seed), torch.normal(..., device="cuda") for
each tensor in order, and the reference's update expression as torch ops on the device
(oracle/torch_replica.py).  Bar: bit-exact.

f16 on the device: torch's elementwise kernels round a Half "f32 scalar * f16 tensor"
product twice (f32, then f16) on their 8-wide vectorized path and once (v_fma_mixlo_f16)
on the unrolled path -- the partial last block of 2048 elements, or a tensor not 16-byte
aligned (profiles/r05_f16_rounding.log); the kernel follows both (fks_device.hip
mul_f16_ref).  test_zero_weight_decay_edge_values caught it: g z = 37.390625 in f32, an
f16 midpoint, in the tail of a 5647-element tensor; test_f16_products_follow_torchs_paths
crafts such midpoints everywhere.

Cases: fp32 / bf16 / f16; tensors below one 256-thread block, between blocks, past the
grid cap (several Philox calls per thread), empty tensors in the list (no draw, no
offset); several seeds including 0, 2^32-1 and one past 2^32; reconstructs at weight
decay 0.01 / 0.0 / None with zero scalars skipped; the perturb +1/-2/+1 sequence with a
frozen tensor; element shards."""
import pytest
import torch

from oracle import torch_replica as R
from test_gpu_parity import _dev

pytestmark = pytest.mark.gpu

DT = {"float32": torch.float32, "bfloat16": torch.bfloat16, "float16": torch.float16}
SHAPES = [(1,), (7,), (256,), (1000,), (4097,), (0,), (33, 65), (600_000,), (3_000_001,), (16,)]


def _bits(t):
    return t.view(torch.int16) if t.element_size() == 2 else t.view(torch.int32)


def _assert_same(got, want, what):
    if not torch.equal(_bits(got), _bits(want)):
        bad = (_bits(got) != _bits(want)).nonzero()
        i = bad[0].tolist()
        raise AssertionError(f"{what}: {bad.shape[0]} of {got.numel()} elements differ, first at {i}: "
                             f"{got[tuple(i)].item()} vs {want[tuple(i)].item()}")


@pytest.mark.parametrize("dtype", ["float32", "bfloat16", "float16"])
@pytest.mark.parametrize("seed", [0, 42, 2**32 - 1, 2**40 + 3])
def test_normal_stream_matches_torch_on_device(dtype, seed):
    from fate_llm.algo.fedkseed import codec
    dev = _dev()
    torch.manual_seed(seed)
    want = [torch.normal(mean=0, std=1, size=s, device=dev, dtype=DT[dtype]) for s in SHAPES]
    got = [torch.empty(s, device=dev, dtype=DT[dtype]) for s in SHAPES]
    codec.normal_(got, seed, stream_mode="torch_rocm")
    torch.cuda.synchronize()
    for s, g, w in zip(SHAPES, got, want):
        _assert_same(g, w, f"seed {seed} shape {s}")


def _params(dtype, dev, seed=0):
    g = torch.Generator().manual_seed(seed)
    shapes = [(4096,), (48,), (1000, 17), (700_001,), (0,), (9,)]
    return [(torch.randn(s, generator=g) * 0.02).to(DT[dtype]).to(dev) for s in shapes]


@pytest.mark.parametrize("dtype", ["float32", "bfloat16", "float16"])
@pytest.mark.parametrize("wd", [0.01, 0.0, None])
@pytest.mark.parametrize("k", [40, 37])
def test_reconstruct_matches_torch_on_device(dtype, wd, k):
    """ClientTrainer.train_once's loop (fedkseed.py:136-141) run by the reference's own
    arithmetic on the GPU vs the codec's reconstruct in the torch_rocm stream.  k 40:
    launches of 32 + 7 non-zero seeds; k 37: 32 + 4."""
    from fate_llm.algo.fedkseed import codec
    dev = _dev()
    g = torch.Generator().manual_seed(7)
    seeds = torch.randint(0, 2**32, (k,), generator=g).tolist()
    vals = (torch.randn(k, generator=g, dtype=torch.float64) * 20).tolist()
    vals[5] = 0.0
    ref = _params(dtype, dev)
    got = [p.clone() for p in ref]
    R.reconstruct(ref, seeds, vals, 1e-3, wd)
    keep = [(s, v) for s, v in zip(seeds, vals) if v != 0.0]
    specs = [codec.ParamSpec(p, lr=1e-3, weight_decay=wd) for p in got]
    codec.directional_step(specs, [s for s, _ in keep], [v for _, v in keep], stream_mode="torch_rocm")
    torch.cuda.synchronize()
    for i, (a, b) in enumerate(zip(got, ref)):
        _assert_same(a, b, f"tensor {i}")


@pytest.mark.parametrize("wd", [0.0, -0.0])
@pytest.mark.parametrize("gscale", [20.0, 1e36])
@pytest.mark.parametrize("keep_fma", [False, True])
def test_zero_weight_decay_edge_values(wd, gscale, keep_fma, monkeypatch):
    """wd = +-0 (the HF default the reference's ClientTrainer passes, fedkseed.py:140) with
    zeros of both signs, +-inf, NaN, subnormals and huge values among the parameters, bf16
    / f32 / f16 tensors in one call: wd = +0 on bf16 / f32 with a bounded |lr g z| takes
    kModeUpdateWdPos0 (t = g z, an infinite parameter set to NaN at load), everything else
    the fma chain; FKS_PHX_KEEP_WD_FMA=1 forces the fma chain.  Against the reference's
    expression as torch ops on the device, bit for bit (NaN payloads aside)."""
    from fate_llm.algo.fedkseed import codec
    if keep_fma:
        monkeypatch.setenv("FKS_PHX_KEEP_WD_FMA", "1")
    dev = _dev()
    edge = torch.tensor([0.0, -0.0, float("inf"), float("-inf"), float("nan"), 1e-40, -1e-42, 3e38, -3e38,
                         1e-3, -2.5e-2, 65000.0, 1.0, -1.0, 1e-8, 7e-39], dtype=torch.float32)
    base = []
    for i, dt in enumerate(["bfloat16", "float32", "bfloat16", "float16"]):
        g = torch.Generator().manual_seed(11 + i)
        x = torch.randn(4096 + 517 * i, generator=g) * 0.02
        x[: edge.numel()] = edge
        x[1000:1000 + edge.numel()] = edge
        base.append(x.to(DT[dt]).to(dev))
    if wd == 0.0 and str(wd) == "0.0":  # +0: drop the f16 tensor so the launch can take WdPos0
        base = base[:3] if not keep_fma else base
    g = torch.Generator().manual_seed(3)
    seeds = torch.randint(0, 2**32, (35,), generator=g).tolist()
    vals = (torch.randn(35, generator=g, dtype=torch.float64) * gscale).tolist()
    vals[4] = -vals[4]
    vals[9], vals[10] = 1e-45, -1e-45  # g z rounds to zeros of both signs
    ref = [b.clone() for b in base]
    R.reconstruct(ref, seeds, vals, 1e-5, wd)
    got = [b.clone() for b in base]
    codec.directional_step([codec.ParamSpec(t, lr=1e-5, weight_decay=wd) for t in got], seeds, vals,
                           stream_mode="torch_rocm")
    torch.cuda.synchronize()
    for i, (a, b) in enumerate(zip(got, ref)):
        an, bn = torch.isnan(a.float()), torch.isnan(b.float())
        assert torch.equal(an, bn), f"tensor {i}: NaN positions differ"
        _assert_same(torch.where(an, torch.zeros_like(a), a), torch.where(bn, torch.zeros_like(b), b), f"tensor {i}")


@pytest.mark.parametrize("n", [5647, 177489, 1000003])
@pytest.mark.parametrize("off", [0, 1])
@pytest.mark.parametrize("wd", [None, 0.01])
@pytest.mark.parametrize("k", [8, 3])
def test_f16_products_follow_torchs_paths(n, off, wd, k):
    """f16 parameters, many products: about one in 10^4 f32 products g z / lr t / wd p lands
    on an f16 rounding midpoint, where torch's vectorized path (full 2048-element blocks
    of 16-byte-aligned tensors) and its unrolled path (the partial last block, unaligned
    tensors) round differently.  The parameter is a view at element offset `off` of a
    larger buffer (off 1: 2-byte aligned: the first seed's wd p takes the unrolled path in
    the reference).  Against the reference's expression as torch ops on the device."""
    from fate_llm.algo.fedkseed import codec
    dev = _dev()
    gen = torch.Generator(dev).manual_seed(n + off)
    buf = (torch.randn(n + off + 64, device=dev, generator=gen) * 0.05).to(torch.float16)
    ref_buf, got_buf = buf.clone(), buf.clone()
    ref, got = [ref_buf[off:off + n]], got_buf[off:off + n]
    g = torch.Generator().manual_seed(9)
    seeds = torch.randint(0, 2**32, (k,), generator=g).tolist()
    vals = (torch.randn(k, generator=g, dtype=torch.float64) * 20).tolist()
    R.reconstruct(ref, seeds, vals, 1e-3, wd)
    codec.directional_step([codec.ParamSpec(got, lr=1e-3, weight_decay=wd)], seeds, vals, stream_mode="torch_rocm")
    torch.cuda.synchronize()
    _assert_same(got, ref[0], f"n {n} off {off} wd {wd}")


@pytest.mark.parametrize("dtype", ["float32", "bfloat16", "float16"])
def test_perturb_sequence_with_frozen_tensor(dtype):
    """random_perturb_parameters (optimizer.py:152-173) +1, -2, +1: frozen tensors draw
    nothing; the restore is not bit-exact (three roundings), the same in both."""
    from fate_llm.algo.fedkseed import codec
    dev = _dev()
    ref = _params(dtype, dev, seed=3)
    frozen = [False, True, False, False, False, False]
    got = [p.clone() for p in ref]
    eps, seed = 5e-4, 123456789
    for sf in (1.0, -2.0, 1.0):
        torch.manual_seed(seed)
        for p, fz in zip(ref, frozen):
            if not fz:
                z = torch.normal(mean=0, std=1, size=p.size(), device=p.device, dtype=p.dtype)
                p.data = p.data + sf * eps * z
        codec.perturb([p for p, fz in zip(got, frozen) if not fz], seed, sf * eps, stream_mode="torch_rocm")
    torch.cuda.synchronize()
    for i, (a, b) in enumerate(zip(got, ref)):
        _assert_same(a, b, f"tensor {i}")


def test_element_shards_equal_whole():
    from fate_llm.algo.fedkseed import codec
    dev = _dev()
    g = torch.Generator().manual_seed(9)
    seeds = torch.randint(0, 2**32, (35,), generator=g).tolist()
    vals = (torch.randn(35, generator=g, dtype=torch.float64) * 20).tolist()
    whole = _params("bfloat16", dev, seed=5)
    shards = [p.clone() for p in whole]
    codec.directional_step([codec.ParamSpec(p, lr=1e-3, weight_decay=0.01) for p in whole], seeds, vals,
                           stream_mode="torch_rocm")
    sp = [codec.ParamSpec(p, lr=1e-3, weight_decay=0.01) for p in shards]
    for r in range(3):
        codec.directional_step(sp, seeds, vals, shard=r, nshards=3, stream_mode="torch_rocm")
    torch.cuda.synchronize()
    for i, (a, b) in enumerate(zip(shards, whole)):
        _assert_same(a, b, f"tensor {i}")


@pytest.mark.parametrize("nshards", [2, 3, 8])
def test_element_shards_are_contiguous_runs_census(nshards):
    """Element shards of the torch_rocm stream are runs of whole Philox rows: each shard
    writes exactly the contiguous element range fks_shard_census reports for it (in the
    tensors' concatenation, frozen and empty tensors included), the ranges tile the
    buffer, and the per-tensor counts add up -- what bench.py --gather broadcasts."""
    from fate_llm.algo.fedkseed import codec
    dev = _dev()
    g = torch.Generator().manual_seed(13)
    sizes = [4096, 48, 0, 9_000_017, 17_000, 700_001, 9]
    frozen = [False, False, False, False, True, False, False]
    total = sum(sizes)
    flat0 = (torch.randn(total, generator=g) * 0.02).to(torch.bfloat16).to(dev)
    seeds = torch.randint(0, 2**32, (3,), generator=g).tolist()
    vals = (torch.randn(3, generator=g, dtype=torch.float64) * 20).tolist()

    def specs(flat):
        out, off = [], 0
        for n, fz in zip(sizes, frozen):
            out.append(codec.ParamSpec(flat[off:off + n], lr=1e-3, weight_decay=None, frozen=fz))
            off += n
        return out

    whole = flat0.clone()
    codec.directional_step(specs(whole), seeds, vals, stream_mode="torch_rocm")
    ends, counts = [0], [0] * len(sizes)
    for r in range(nshards):
        one = flat0.clone()
        sp = specs(one)
        b = codec._Batch(sp, "torch_rocm")
        import ctypes
        from fate_llm.algo.fedkseed import _native as N
        rng = (ctypes.c_int64 * 2)()
        wr = (ctypes.c_int64 * len(sizes))()
        N.check(N.load().fks_shard_census(ctypes.addressof(b.arr), b.n, r, nshards, rng, wr))
        lo, hi = int(rng[0]), int(rng[1])
        assert lo == ends[-1] and hi >= lo
        ends.append(hi)
        assert codec.shard_range(sp, r, nshards, stream_mode="torch_rocm") == (lo, hi)
        codec.directional_step(sp, seeds, vals, shard=r, nshards=nshards, stream_mode="torch_rocm")
        torch.cuda.synchronize()
        changed = (one.view(torch.int16) != flat0.view(torch.int16)).nonzero().flatten()
        if changed.numel():
            assert int(changed.min()) >= lo and int(changed.max()) < hi, (r, lo, hi)
        # inside its range the shard equals the whole reconstruct, outside it is untouched
        assert torch.equal(one[lo:hi].view(torch.int16), whole[lo:hi].view(torch.int16))
        for i in range(len(sizes)):
            counts[i] += int(wr[i])
    assert ends[-1] == total
    assert counts == [0 if fz else n for n, fz in zip(sizes, frozen)]


def _reference_zo_steps(groups, seeds, losses, eps):
    """The reference's ZerothOrderOptimizer.zeroth_order_step (optimizer.py:113-148, its
    random_perturb_parameters :152-173) and zo_utils.directional_derivative_step
    (zo_utils.py:42-52) as torch ops on the parameters' device: frozen tensors draw no
    perturbation but are updated; the first group's lr and wd hold for every group."""
    rets, it = [], iter(losses)

    def perturb(seed, sf):
        torch.manual_seed(seed)
        for grp in groups:
            for p in grp["params"]:
                if p.requires_grad:
                    z = torch.normal(mean=0, std=1, size=p.data.size(), device=p.data.device, dtype=p.data.dtype)
                    p.data = p.data + sf * eps * z

    for seed in seeds:
        perturb(seed, 1.0)
        right = next(it)
        perturb(seed, -2.0)
        left = next(it)
        perturb(seed, 1.0)
        if torch.isnan(right) or torch.isnan(left):
            rets.append(float("nan"))
            continue
        g = (right - left) / (2 * eps)
        torch.manual_seed(seed)
        lr = wd = None
        for grp in groups:
            wd = grp["weight_decay"] if wd is None else wd
            lr = grp["lr"] if lr is None else lr
            for p in grp["params"]:
                z = torch.normal(mean=0, std=1, size=p.data.size(), device=p.data.device, dtype=p.data.dtype)
                p.data = p.data - lr * (g * z + wd * p.data)
        rets.append(float(g))
    return rets


@pytest.mark.parametrize("dtype", ["float32", "bfloat16", "float16"])
@pytest.mark.parametrize("wd0", [0.0, 0.01])
@pytest.mark.parametrize("path", ["device", "host", "frozen"])
def test_zo_steps_match_the_reference_on_device(dtype, wd0, path):
    """The drop-in optimizer's local steps on a GPU client, under the default stream
    setting ("auto" -> torch_rocm for cuda tensors), against the reference's steps as torch
    ops on the same GPU: four steps with device losses, the third with a NaN loss (restore,
    no update); the fused device tail (losses stay on the device), the host tail, and a
    group holding a frozen tensor (perturb skips it, the update does not; unfused)."""
    from fate_llm.algo.fedkseed import codec
    from fate_llm.algo.fedkseed.optimizer import ZerothOrderOptimizer
    dev = _dev()
    eps = 5e-4
    data = _params(dtype, dev, seed=21)
    frozen = [False] * len(data)
    if path == "frozen":
        frozen[2] = True
    seeds = [7, 2**32 - 1, 123456789, 2**40 + 5]
    loss_vals = [2.5, 2.25, 2.375, 2.5, float("nan"), 2.0, 3.0, 2.875]

    def build():
        ps = [torch.nn.Parameter(t.clone(), requires_grad=not fz) for t, fz in zip(data, frozen)]
        return ps, [{"params": ps[:3], "weight_decay": wd0, "lr": 1e-3, "eps": eps},
                    {"params": ps[3:], "weight_decay": 0.01 - wd0, "lr": 2e-3, "eps": eps}]

    ref, ref_groups = build()
    want = _reference_zo_steps(ref_groups, seeds, [torch.tensor(x, device=dev) for x in loss_vals], eps)
    got, groups = build()
    old = codec.get_stream_mode()
    codec.set_stream_mode("auto")
    try:
        opt = ZerothOrderOptimizer(groups, lr=1e-3, eps=eps, weight_decay=wd0, grad_clip=-100.0)
        opt.device_step = path == "device"
        it = iter([torch.tensor(x, device=dev) for x in loss_vals])
        rets = []
        for s in seeds:
            g, _, _ = opt.zeroth_order_step(s, lambda: next(it))
            assert opt._last_step_on_device == (path == "device")
            rets.append(float(g))
    finally:
        codec.set_stream_mode(old)
    torch.cuda.synchronize()
    assert [str(x) for x in rets] == [str(x) for x in want]
    for i, (a, b) in enumerate(zip(got, ref)):
        _assert_same(a.data, b.data, f"tensor {i}")


@pytest.mark.parametrize("nt", [300, 600])
def test_tensor_tables_in_and_out_of_lds(nt):
    """fks_philox_vec_kernel looks tensors up in an LDS copy of the table for launches of at
    most 512 tensors and in device memory beyond: both against the reference as torch ops,
    with sizes that put tensor boundaries inside a wave's 64 groups (per-lane lookups)."""
    from fate_llm.algo.fedkseed import codec
    dev = _dev()
    g = torch.Generator().manual_seed(nt)
    sizes = torch.randint(1, 6000, (nt,), generator=g).tolist()
    sizes[nt // 2] = 300_000
    ref = [(torch.randn(n, generator=g) * 0.02).to(torch.bfloat16).to(dev) for n in sizes]
    got = [p.clone() for p in ref]
    seeds = torch.randint(0, 2**32, (35,), generator=g).tolist()
    vals = (torch.randn(35, generator=g, dtype=torch.float64) * 20).tolist()
    R.reconstruct(ref, seeds, vals, 1e-3, 0.01)
    codec.directional_step([codec.ParamSpec(p, lr=1e-3, weight_decay=0.01) for p in got], seeds, vals,
                           stream_mode="torch_rocm")
    codec.perturb(got, seeds[0], 5e-4, stream_mode="torch_rocm")
    torch.manual_seed(seeds[0])
    for i, p in enumerate(ref):
        ref[i] = p + 5e-4 * torch.normal(mean=0, std=1, size=p.size(), device=p.device, dtype=p.dtype)
    torch.cuda.synchronize()
    for i, (a, b) in enumerate(zip(got, ref)):
        _assert_same(a, b, f"tensor {i}")


def test_f16_unaligned_view_later_calls_read_a_fresh_tensor(monkeypatch):
    """The reference rebinds param.data to a tensor torch allocates at every update and
    perturbation (zo_utils.py:49, optimizer.py:173), so from a parameter's second call on,
    the first seed's wd * p reads a 16-byte-aligned tensor and takes torch's vectorized path
    (two roundings of an f16 product), even when the parameter started as an unaligned view;
    the drop-in updates the view in place and carries that as ParamSpec.fresh / FKS_FRESH
    (codec.mark_rebound).  Three directional_derivative_step calls and an unfused
    zeroth-order step (a frozen tensor in the groups) on an f16 view at element offset 1,
    wd 0.01, against the reference's calls on the device.  With the record switched off the
    drop-in takes the single rounding there and differs -- the case is exercised.  The
    zeroth-order step's losses are CPU tensors, so its g is a CPU scalar: torch multiplies
    its f32 value into z on the GPU without casting it to f16 first (zo_utils._value_kind)."""
    from fate_llm.algo.fedkseed import codec, zo_utils
    from fate_llm.algo.fedkseed.optimizer import ZerothOrderOptimizer
    dev = _dev()
    n, off = 3_000_001, 1
    gen = torch.Generator(dev).manual_seed(21)
    buf = (torch.randn(n + off + 64, device=dev, generator=gen) * 0.05).to(torch.float16)
    frozen0 = (torch.randn(777, device=dev, generator=gen) * 0.05).to(torch.float16)

    def run(record):
        if not record:
            monkeypatch.setattr(codec, "is_rebound", lambda p: False)
        ref_buf, got_buf = buf.clone(), buf.clone()
        ref = [torch.nn.Parameter(ref_buf[off:off + n]), torch.nn.Parameter(frozen0.clone(), requires_grad=False)]
        got = [torch.nn.Parameter(got_buf[off:off + n]), torch.nn.Parameter(frozen0.clone(), requires_grad=False)]
        assert got[0].data_ptr() % 16 != 0
        # g z of the size of wd p (|g| ~ 1e-3), so that wd p's rounding shows in t = g z + wd p,
        # and lr 0.1, so that lr t shows in p
        rg = [{"params": ref, "lr": 0.1, "weight_decay": 0.01, "eps": 1e-3}]
        gg = [{"params": got, "lr": 0.1, "weight_decay": 0.01, "eps": 1e-3}]
        codec.set_stream_mode("torch_rocm")
        try:
            for seed, v in [(5, 2e-3), (6, -1.5e-3), (7, 1e-3)]:
                R.directional_derivative_step(rg, seed, v)
                zo_utils.directional_derivative_step(gg, seed, v)
            opt = ZerothOrderOptimizer(gg, lr=0.1, eps=1e-3, weight_decay=0.01, grad_clip=0.0)

            def closure_on(ps):  # a CPU loss: the host path, g a CPU scalar (zo_utils._value_kind)
                return lambda: ps[0].detach()[:4096].float().sum().cpu() * 1e-6

            R.zeroth_order_step(rg, 99, closure_on(ref), 1e-3)
            opt.zeroth_order_step(99, closure_on(got))
        finally:
            codec.set_stream_mode("torch_cpu")
            monkeypatch.undo()
        torch.cuda.synchronize()
        return got[0].detach(), ref[0].detach()

    got, ref = run(record=True)
    _assert_same(got, ref, "f16 view at offset 1, later calls")
    got_off, ref_off = run(record=False)
    assert not torch.equal(_bits(got_off), _bits(ref_off)), "no midpoint hit: the case is not exercised"
