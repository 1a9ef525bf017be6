"""Seed-sharded variant (BASELINE config C3), host logic on CPU:

* ``seed_shard_coefficients``: the ranks' seed ranges tile [0, K) in order and the
  coefficients are lr g_k a^(K-1-k) of the GLOBAL seed index k;
* ``reconstruct_seed_sharded_`` over gloo, world 2 and 3: each rank accumulates its
  seeds, one all-reduce sums the parts, every rank applies p = a^K p_0 - delta.  The
  device kernels are swapped for the oracle's f32 restatement of the same operations
  (tests only; the GPU kernels are pinned to it bit for bit in
  tests/test_gpu_seed_shard.py), so this checks the sharding and the collective, and
  that every rank ends with the same parameters as a single rank (within f32 summation
  order) and within the north star's tolerance of the sequential reference.
"""
import math
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from fate_llm.algo.fedkseed import zo_utils


@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("wd", [None, 0.01])
def test_coefficients_tile_and_match(world, wd):
    vals = [float(v) for v in np.random.default_rng(0).normal(0, 20, 37)]
    lr = 1e-5
    lr32 = float(np.float32(lr))
    a = 1.0 if wd is None else 1.0 - lr32 * float(np.float32(wd))
    seen = []
    for r in range(world):
        lo, hi, coefs, decay = zo_utils.seed_shard_coefficients(vals, lr, wd, r, world)
        assert len(coefs) == hi - lo
        seen.extend(range(lo, hi))
        for i, c in zip(range(lo, hi), coefs):
            assert math.isclose(c, lr32 * vals[i] * a ** (36 - i), rel_tol=1e-12)
        assert math.isclose(decay, a ** 37, rel_tol=1e-12)
    assert seen == list(range(37))


def _oracle_codec(monkeypatch):
    """Route the two device calls through the oracle (CPU tensors, f32 restatement)."""
    from fate_llm.algo.fedkseed import codec
    from oracle import fks_oracle as O

    def acc(specs, seeds, coefs, delta):
        arrays = [sp.tensor.detach().numpy() for sp in specs]
        d = delta.numpy()
        O.delta_accumulate(arrays, [O.F32] * len(arrays), seeds, coefs, d,
                           frozen=[int(sp.frozen) for sp in specs])

    def app(specs, delta, decays):
        arrays = [sp.tensor.detach().numpy() for sp in specs]
        O.delta_apply(arrays, [O.F32] * len(arrays), delta.numpy(), decays)

    monkeypatch.setattr(codec, "delta_accumulate", acc)
    monkeypatch.setattr(codec, "delta_apply", app)
    # the generator placement needs the device (tests/test_gpu_generator_state.py pins it)
    monkeypatch.setattr(codec, "leave_generators", lambda specs, seed, stream_mode=None: torch.manual_seed(seed))


SHAPES = [4096, 37, 3, 2000]


def _problem():
    g = torch.Generator().manual_seed(0)
    init = [torch.randn(n, generator=g) * 0.02 for n in SHAPES]
    seeds = torch.randint(0, 2**32, (24,), generator=g).tolist()
    vals = (torch.randn(24, generator=g, dtype=torch.float64) * 20).tolist()
    vals[5] = 0.0  # skipped, as fedkseed.py:137 does
    return init, seeds, vals


def _run_variant(init, seeds, vals):
    params = [torch.nn.Parameter(t.clone()) for t in init]
    groups = [{"params": params[:2], "lr": 0.0, "weight_decay": 0.0},
              {"params": params[2:], "lr": 0.0, "weight_decay": 0.01}]
    n = zo_utils.reconstruct_seed_sharded_(groups, seeds, vals, lr=1e-5, weight_decay=0.01)
    return n, [p.detach().clone() for p in params]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mp_ = pytest.MonkeyPatch()
        _oracle_codec(mp_)
        init, seeds, vals = _problem()
        n, out = _run_variant(init, seeds, vals)
        gathered = [None] * world
        dist.all_gather_object(gathered, [t.numpy() for t in out])
        if rank == 0:
            q.put((n, gathered))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_seed_sharded_reconstruct_gloo(world, monkeypatch):
    from oracle import fks_oracle as O

    _oracle_codec(monkeypatch)
    init, seeds, vals = _problem()
    n1, single = _run_variant(init, seeds, vals)
    assert n1 == 23
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    n, gathered = q.get(timeout=120)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert n == 23
    for r in range(1, world):  # every rank holds the same result
        for a, b in zip(gathered[0], gathered[r]):
            assert np.array_equal(a, b)
    # same as one rank up to the f32 summation order of the all-reduce (a few ulp of p)
    for a, b in zip(gathered[0], single):
        assert np.allclose(a, b.numpy(), rtol=2.0**-21, atol=1e-8), np.abs(a - b.numpy()).max()
    # and within the north star's tolerance of the sequential reference restatement
    ref = [t.numpy().copy() for t in init]
    O.reconstruct(ref, [O.F32] * 4, [1e-5] * 4, [0.01] * 4, seeds, vals)
    got = np.concatenate([a.ravel() for a in gathered[0]]).astype(np.float64)
    r = np.concatenate([a.ravel() for a in ref]).astype(np.float64)
    assert np.linalg.norm(got - r) / np.linalg.norm(r) < 1e-6
