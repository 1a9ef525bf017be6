"""C3 (BASELINE configs[2]): the north star's seed-sharded reconstruct with one
all-reduce of the f32 delta, held to the north star's bar at its own K.

* ``test_c3_k4096_deviation``: at K = 4096 (the C3 seed count), fp32 and bf16, the
  variant against the pinned sequential oracle (= the reference's own FedKSeed path,
  tests/test_oracle_golden.py) and both against exact (float64) arithmetic on the same z
  streams.  The bar is the north star's 1e-6 relative (normwise) in fp32; the measured
  numbers are written to gpurun_out/c3_deviation.json for DESIGN.md §7.
* ``test_c3_two_processes_gloo_on_cuda``: ``zo_utils.reconstruct_seed_sharded_`` in two
  processes on cuda:0 over a gloo group with device tensors: the GPU kernels and the
  collective together, end to end, bit for bit against the oracle's f32 restatement of
  the same two-way split (fedkseed.py:136-141 sharded by seed); on both streams -- for
  torch_rocm each rank's part is restated from torch.normal(device="cuda") draws.
"""
import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from oracle import fks_oracle as O
from test_gpu_parity import DTC, _dev, from_np, rand_params, to_np

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _seeds(k, seed):
    g = torch.Generator().manual_seed(seed)
    seeds = torch.randint(0, 2**32, (k,), generator=g).tolist()
    vals = (torch.randn(k, generator=g, dtype=torch.float64) * 20).tolist()
    return seeds, vals


def _values(bits: np.ndarray, dtype: str) -> np.ndarray:
    if dtype == "bfloat16":
        return (bits.astype(np.uint32) << 16).view(np.float32).astype(np.float64)
    return bits.astype(np.float64)


def _exact(a0, dtype, seeds, vals, lr, wd):
    """The K sequential steps in float64 on the reference's own z streams and f32
    scalars (lr, wd, g as the reference's opmath sees them), no per-op rounding."""
    p = _values(a0, dtype)
    lr32, wd32 = float(np.float32(lr)), (None if wd is None else float(np.float32(wd)))
    for s, g in zip(seeds, vals):
        if g == 0.0:
            continue
        z = _values(O.Generator(s).normal(p.size, DTC[dtype]), dtype)
        g32 = float(np.float32(g))
        p = p - lr32 * (g32 * z + (wd32 * p if wd32 is not None else 0.0))
    return p


def _rel(a, b):
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))


RESULTS = {}


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
@pytest.mark.parametrize("wd", [None, 0.01])
def test_c3_k4096_deviation(dtype, wd):
    from fate_llm.algo.fedkseed import zo_utils
    dev = _dev()
    n, k, lr = 65536, 4096, 1e-5
    a0 = rand_params([n], dtype, seed=21)[0]
    seeds, vals = _seeds(k, seed=22)
    for i in range(0, k, 100):
        vals[i] = 0.0  # skipped, as train_once does
    ref = a0.copy()
    O.reconstruct([ref], [DTC[dtype]], [lr], [wd], seeds, vals)  # the reference's path
    p = torch.nn.Parameter(from_np(a0, dtype, dev))
    groups = [{"params": [p], "lr": 0.0, "weight_decay": 0.0}]
    zo_utils.reconstruct_seed_sharded_(groups, seeds, vals, lr=lr, weight_decay=wd)
    torch.cuda.synchronize()
    got = _values(to_np(p), dtype)
    refv = _values(ref, dtype)
    exact = _exact(a0, dtype, seeds, vals, lr, wd)
    r = {"n": n, "k": k, "lr": lr, "wd": wd,
         "variant_vs_reference": _rel(got, refv),
         "reference_vs_exact": _rel(refv, exact),
         "variant_vs_exact": _rel(got, exact),
         "variant_vs_reference_max_abs": float(np.abs(got - refv).max()),
         "elements_differing_frac": float(np.mean(got != refv))}
    r["meets_1e-6"] = r["variant_vs_reference"] <= 1e-6
    RESULTS[f"{dtype}_wd{wd}"] = r
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "c3_deviation.json"), "w") as f:
        json.dump(RESULTS, f, indent=1)
    print(dtype, wd, r)
    if dtype == "float32":
        # the stated outcome against the north star's bar: the variant is
        # closer to exact arithmetic than the reference itself is, and misses the 1e-6
        # bar against the reference by the reference's own rounding noise
        assert r["variant_vs_exact"] < r["reference_vs_exact"]
        assert not r["meets_1e-6"], r
        assert r["variant_vs_reference"] < 5e-6, r
    else:
        # bf16: the reference rounds every op of every seed to bf16 (most single-seed
        # updates fall below half an ulp); the variant rounds once -- a different function
        assert not r["meets_1e-6"], r


# ------------------------------------------------------------------ two processes
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, dtype, a0, seeds, vals, lr, wd, q, stream="torch_cpu"):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "fate-llm_amd", "python"))
    import torch.distributed as dist
    from fate_llm.algo.fedkseed import codec, zo_utils
    codec.set_stream_mode(stream)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    p = torch.nn.Parameter(from_np(a0, dtype, dev))
    groups = [{"params": [p], "lr": 0.0, "weight_decay": 0.0}]
    n = zo_utils.reconstruct_seed_sharded_(groups, seeds, vals, lr=lr, weight_decay=wd)
    torch.cuda.synchronize()
    q.put((rank, n, to_np(p)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("stream", ["torch_cpu", "torch_rocm"])
@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
def test_c3_two_processes_gloo_on_cuda(dtype, stream):
    from fate_llm.algo.fedkseed import zo_utils
    from test_gpu_torch_rocm_big import _fma32
    dev = _dev()
    world, n, k, lr, wd = 2, 1 << 16, 512, 1e-5, 0.01
    a0 = rand_params([n], dtype, seed=31)[0]
    seeds, vals = _seeds(k, seed=32)
    vals[5] = 0.0
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, dtype, a0, seeds, vals, lr, wd, q, stream))
             for r in range(world)]
    for pr in procs:
        pr.start()
    outs = sorted(q.get(timeout=120) for _ in range(world))
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    # the oracle's restatement of the same split: each rank's seed range with its global
    # coefficients accumulated in f32, the two parts summed (what gloo's all-reduce does
    # for two ranks), one fma + rounding per element
    keep = [(s, v) for s, v in zip(seeds, vals) if v != 0.0]
    parts = []
    for r in range(world):
        lo, hi, coefs, decay = zo_utils.seed_shard_coefficients([v for _, v in keep], lr, wd, r, world)
        d = np.zeros(n, np.float32)
        if stream == "torch_cpu":
            O.delta_accumulate([a0.copy()], [DTC[dtype]], [s for s, _ in keep[lo:hi]], coefs, d)
        else:
            for (s, _), c in zip(keep[lo:hi], coefs):
                torch.manual_seed(s)
                z = torch.normal(0, 1, size=(n,), device=dev, dtype=getattr(torch, dtype)).float().cpu().numpy()
                d = _fma32(np.float32(c), z, d)
        parts.append(d)
    ref = a0.copy()
    O.delta_apply([ref], [DTC[dtype]], parts[0] + parts[1], [decay])
    for rank, applied, got in outs:
        assert applied == len(keep)
        w = np.uint16 if got.itemsize == 2 else np.uint32
        assert np.array_equal(got.view(w), ref.view(w)), f"rank {rank}: {int((got.view(w) != ref.view(w)).sum())} differ"


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
@pytest.mark.parametrize("wd", [None, 0.01])
def test_c3_k4096_deviation_torch_rocm(dtype, wd):
    """The same measurement on the default stream (torch_rocm): the reference's path is its
    own loop as torch ops on the device (oracle/torch_replica.py), exact arithmetic the K
    steps in float64 on the same device z; the variant draws the same z
    (fks_philox_vec_kernel<kModeDelta>).  Reported, not asserted beyond sanity."""
    from fate_llm.algo.fedkseed import codec, zo_utils
    from oracle import torch_replica as R
    dev = _dev()
    dt = getattr(torch, dtype)
    n, k, lr = 65536, 4096, 1e-5
    p0 = (torch.randn(n, generator=torch.Generator().manual_seed(21)) * 0.02).to(dt).to(dev)
    seeds, vals = _seeds(k, seed=22)
    for i in range(0, k, 100):
        vals[i] = 0.0
    ref = [p0.clone()]
    R.reconstruct(ref, seeds, vals, lr, wd)
    exact = p0.double()
    lr32, wd32 = float(np.float32(lr)), (None if wd is None else float(np.float32(wd)))
    for s, g in zip(seeds, vals):
        if g == 0.0:
            continue
        torch.manual_seed(s)
        z = torch.normal(mean=0, std=1, size=(n,), device=dev, dtype=dt).double()
        exact = exact - lr32 * (float(np.float32(g)) * z + (wd32 * exact if wd32 is not None else 0.0))
    p = torch.nn.Parameter(p0.clone())
    codec.set_stream_mode("torch_rocm")
    try:
        zo_utils.reconstruct_seed_sharded_([{"params": [p], "lr": 0.0, "weight_decay": 0.0}], seeds, vals, lr=lr,
                                           weight_decay=wd)
    finally:
        codec.set_stream_mode("torch_cpu")
    torch.cuda.synchronize()
    got, rf, ex = p.detach().double().cpu().numpy(), ref[0].double().cpu().numpy(), exact.cpu().numpy()
    r = {"variant_vs_reference": _rel(got, rf), "reference_vs_exact": _rel(rf, ex), "variant_vs_exact": _rel(got, ex)}
    RESULTS[f"torch_rocm {dtype} wd={wd}"] = r
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "c3_deviation_rocm.json"), "w") as f:
        json.dump({k_: v for k_, v in RESULTS.items() if k_.startswith("torch_rocm")}, f, indent=1)
    assert r["variant_vs_exact"] < 1e-2 and r["reference_vs_exact"] < 0.2
