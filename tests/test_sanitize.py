"""SURVEY.md §5's sanitizer row: the host code -- the oracle and libfks.so's plan cache,
layout, GF(2) jump-polynomial and table code behind the C ABI -- built with
-fsanitize=address,undefined (make -C oracle asan, make -C fate-llm_amd asan) and the
CPU suite's host tests run against those builds (tools/sanitize.sh: g++'s ASan runtime
preloaded, FKS_ORACLE_LIB / FKS_LIB_OVERRIDE pointing at the sanitized libraries).  Any
ASan or UBSan report aborts the run.  Host code only: no GPU sanitizer on this pool."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None or not os.path.exists("/opt/rocm/include/hip/hip_runtime_api.h"),
                    reason="needs g++ and the HIP runtime headers")
def test_host_code_under_asan_ubsan():
    env = {k: v for k, v in os.environ.items() if k not in ("LD_PRELOAD", "FKS_LIB_OVERRIDE", "FKS_ORACLE_LIB")}
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "sanitize.sh")], capture_output=True, text=True,
                       timeout=900, env=env, cwd=ROOT)
    tail = (r.stdout + r.stderr)[-4000:]
    assert r.returncode == 0, tail
    assert "passed" in r.stdout and "AddressSanitizer" not in tail and "runtime error" not in tail, tail
