import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
PKG_PY = os.path.join(ROOT, "fate-llm_amd", "python")
for p in (ROOT, PKG_PY):
    if p not in sys.path:
        sys.path.insert(0, p)
# The parity tests compare with the oracle, which restates torch's CPU-generator stream;
# the drop-in's default ("auto": torch_rocm on a HIP device) is pinned by its own tests
# (test_stream_tag.py, test_gpu_torch_rocm.py).  Subprocesses inherit this.
os.environ.setdefault("FKS_STREAM_MODE", "torch_cpu")

# A tree that arrives without libfks.so / liboracle.so is built here, in a subprocess, before
# any test touches the GPU (__graft_entry__.ensure_built: make -C fate-llm_amd, make -C oracle).
import __graft_entry__  # noqa: E402

_COMPILED = __graft_entry__.ensure_built()


def pytest_report_header(config):
    import torch  # noqa: F401  (before libfks.so: _native.load)
    from fate_llm.algo.fedkseed import _native
    try:
        bid = _native.build_id()
    except OSError as e:  # reported, and every codec test then fails loudly
        bid = f"not loadable ({e})"
    try:
        sid = _native.source_id()
    except OSError:
        sid = None
    return (f"libfks.so build id {bid}, source id {sid} (this tree: {__graft_entry__.source_id()}); "
            f"compile commands run by this session's conftest: {_COMPILED}")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device; parity tests of the product path")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def cases():
    with open(os.path.join(GOLDEN, "cases.json")) as f:
        return json.load(f)


def load_npz(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def golden():
    return load_npz


def as_float(a: np.ndarray, dtype: str) -> np.ndarray:
    """Decode stored bits (uint16 for bf16/f16) to float64 for NaN tests / error metrics."""
    if dtype == "bfloat16":
        return (a.astype(np.uint32) << 16).view(np.float32).astype(np.float64)
    if dtype == "float16":
        return a.view(np.float16).astype(np.float64)
    return a.astype(np.float64)


def assert_bitwise(got: np.ndarray, ref: np.ndarray, dtype: str, what=""):
    """Bit-exact equality, except that any NaN matches any NaN.

    torch's CPU kernels encode a NaN differently by position (the vectorised
    bf16 conversion emits 0xFFFF, the scalar c10::BFloat16 one 0x7FC0, and which
    elements take which path depends on vector-body/tail split and the thread
    partition), so NaN payload bits are not part of the contract."""
    got = np.ascontiguousarray(got).reshape(-1)
    ref = np.ascontiguousarray(ref).reshape(-1)
    assert got.shape == ref.shape, what
    gn = np.isnan(as_float(got, dtype))
    rn = np.isnan(as_float(ref, dtype))
    assert np.array_equal(gn, rn), f"{what}: NaN positions differ ({gn.sum()} vs {rn.sum()})"
    w = np.uint16 if got.itemsize == 2 else (np.uint32 if got.itemsize == 4 else np.uint64)
    bad = (got.view(w) != ref.view(w)) & ~rn
    assert not bad.any(), f"{what}: {int(bad.sum())} of {bad.size} elements differ (first at {int(np.argmax(bad))})"
