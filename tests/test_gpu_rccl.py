"""The RCCL ("nccl" backend) branches of the multi-GPU path, executed on a one-GPU box.

RCCL refuses two ranks on one device, so the N > 1 rehearsals (test_gpu_bench_ranks.py,
test_gpu_c3.py) talk over gloo.  Here a WORLD-SIZE-1 RCCL group on cuda:0 runs the same
code the 8-GPU node runs, through the collective library on device tensors:

* ``zo_utils.reconstruct_seed_sharded_`` -- its all-reduce of the f32 delta (the north
  star's C3 form of fedkseed.py:136-141) -- bit-exact against the oracle's f32
  restatement of the unsplit sum;
* ``bench.py`` under torch.distributed.run with one rank: the RCCL process group, the
  max-over-ranks timing all-reduce (a float64 device tensor), element-shard ``--gather``
  (RCCL broadcasts) and ``--mode seed-shard``.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from oracle import fks_oracle as O
from test_gpu_parity import DTC, _dev, from_np, rand_params, to_np

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _seeds(k, seed):
    g = torch.Generator().manual_seed(seed)
    return (torch.randint(0, 2**32, (k,), generator=g).tolist(),
            (torch.randn(k, generator=g, dtype=torch.float64) * 20).tolist())


def _rank0(port, dtype, a0, seeds, vals, lr, wd, q):
    sys.path.insert(0, os.path.join(ROOT, "fate-llm_amd", "python"))
    import torch.distributed as dist
    from fate_llm.algo.fedkseed import zo_utils
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    try:
        p = torch.nn.Parameter(from_np(a0, dtype, dev))
        groups = [{"params": [p], "lr": 0.0, "weight_decay": 0.0}]
        n = zo_utils.reconstruct_seed_sharded_(groups, seeds, vals, lr=lr, weight_decay=wd)
        t = torch.tensor([1.5], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        torch.cuda.synchronize()
        q.put((dist.get_backend(), n, to_np(p), float(t.item())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
def test_seed_sharded_reconstruct_over_rccl_world1(dtype):
    from fate_llm.algo.fedkseed import zo_utils
    _dev()
    n, k, lr, wd = 1 << 16, 256, 1e-5, 0.01
    a0 = rand_params([n], dtype, seed=41)[0]
    seeds, vals = _seeds(k, seed=42)
    vals[7] = 0.0
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pr = ctx.Process(target=_rank0, args=(_free_port(), dtype, a0, seeds, vals, lr, wd, q))
    pr.start()
    backend, applied, got, tmax = q.get(timeout=150)
    pr.join(timeout=60)
    assert pr.exitcode == 0
    assert backend == "nccl" and tmax == 1.5
    keep = [(s, v) for s, v in zip(seeds, vals) if v != 0.0]
    assert applied == len(keep)
    lo, hi, coefs, decay = zo_utils.seed_shard_coefficients([v for _, v in keep], lr, wd, 0, 1)
    d = np.zeros(n, np.float32)
    O.delta_accumulate([a0.copy()], [DTC[dtype]], [s for s, _ in keep[lo:hi]], coefs, d)
    ref = a0.copy()
    O.delta_apply([ref], [DTC[dtype]], d, [decay])
    w = np.uint16 if got.itemsize == 2 else np.uint32
    assert np.array_equal(got.view(w), ref.view(w)), f"{int((got.view(w) != ref.view(w)).sum())} differ"


@pytest.mark.parametrize("extra", [["--gather"], ["--mode", "seed-shard"]])
def test_bench_under_torchrun_world1_rccl(extra):
    _dev()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "FKS_BENCH_SHARE_GPU"):
        env.pop(v, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1", "--master-addr=127.0.0.1",
           f"--master-port={_free_port()}", os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "2", "--warmup",
           "1", "--params", str(1 << 24), "--k", "64", "--no-cpu-baseline"] + extra
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = lines[0]
    assert out["n_gpus"] == 1 and out["backend"] == "nccl" and "shared_gpu" not in out
    assert out["value"] > 0 and out["steps"] == 2
    if "--gather" in extra:
        assert out["gather_ms"] > 0 and out["config"]["parallelism"] == "element-shard1"
    else:
        assert out["config"]["parallelism"] == "seed-shard1"
