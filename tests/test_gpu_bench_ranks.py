"""bench.py's multi-rank GPU path, rehearsed on a one-GPU box: `--gpus 2` re-launches the
script under torch.distributed.run, both ranks run the codec on the visible GPU
(FKS_BENCH_SHARE_GPU=1: they share it and talk over gloo instead of RCCL), each rank
reconstructs its element shard of one buffer (--scaling strong, the default), its own
buffer (--scaling weak, opt-in, under its own metric name) or (--mode seed-shard)
accumulates its seeds' delta and all-reduces it; rank 0 prints one JSON line with the
world size the process group saw.
The measured 8-GPU run is the driver's (one GPU per rank, RCCL)."""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("extra", [[], ["--scaling", "weak"], ["--gather"], ["--mode", "seed-shard"]])
def test_bench_two_ranks_on_one_gpu(extra):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", FKS_BENCH_SHARE_GPU="1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup",
                        "1", "--params", str(1 << 24), "--k", "64", "--no-cpu-baseline"] + extra,
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = lines[0]
    assert out["n_gpus"] == 2 and out["backend"] == "gloo" and out["shared_gpu"]
    assert out["value"] > 0 and out["steps"] == 2
    want = "seed-shard2" if "seed-shard" in extra else "client-per-gpu2" if "weak" in extra else "element-shard2"
    assert out["config"]["parallelism"] == want
    assert out["scaling"] == ("weak" if want == "client-per-gpu2" else "strong")
    assert out["metric"].endswith("[weak scaling: one buffer per GPU]") == (want == "client-per-gpu2")
    if "--gather" in extra:
        assert out["gather_ms"] > 0
