"""bench.py's multi-rank path on CPU (no GPU): `--gpus N` re-launches itself under
torch.distributed.run with N ranks, the ranks time a dummy step with the barrier +
max-over-ranks protocol over gloo (`--selftest`), and rank 0 alone prints one JSON line
reporting the world size the process group saw.  Also the CPU-baseline leg on a tiny
budget (the reference's CPU path through oracle/torch_replica.py)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None, timeout=180):
    e = dict(os.environ, MASTER_ADDR="127.0.0.1")
    e.pop("WORLD_SIZE", None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          timeout=timeout, env=e, cwd=ROOT)


def _json_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_flag_launches_n_ranks(n):
    r = _run(["--gpus", str(n), "--selftest", "--steps", "3", "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout  # rank 0 only
    assert lines[0]["n_gpus"] == n and lines[0]["steps"] == 3 and lines[0]["selftest"]


def test_world_size_mismatch_fails_loudly():
    r = _run(["--gpus", "2", "--selftest"], env={"WORLD_SIZE": "1"})
    assert r.returncode != 0
    assert "WORLD_SIZE" in r.stderr


@pytest.mark.parametrize("wd", [0.0, None])
def test_cpu_baseline_leg_runs(wd):
    sys.path.insert(0, ROOT)
    import bench

    cb = bench.cpu_baseline(3.0, wd)
    assert cb["kind"] == "port" and cb["unit"] == "GB/s" and cb["value"] > 0
    # one single-thread process per CPU this job may use; the host's count beside it
    assert cb["cores"] == bench.usable_cpus()[0] and cb["nproc"] == os.cpu_count()
    assert ("all_host_cores_extrapolated" in cb) == (cb["cores"] < cb["nproc"])
    sp = cb["single_process"]
    # linear in N: the per-(seed*param) cost at 2^22 and 2^24 params agrees within 2x
    assert 0.5 < sp["ns_per_seed_param_2^22"] / sp["ns_per_seed_param_2^24"] < 2.0
