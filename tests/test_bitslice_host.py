"""Host build of the slice kernel's bit-sliced MT19937 primitives (fks_bitslice.h) checked
against the scalar generator (tools/bs/bs_selftest.cpp): the 32-seed transpose into bit
planes, three blocks of the in-place round-by-round twist (the twist wave's schedule:
all reads of a 64-row round before its writes, plane 31 of row i-1 from the neighbour
lane), the low-byte tempering map (MT19937RNGEngine.h:141-145 restricted to the bf16
uniform's 8 bits), the 8x8 bit-block transpose and the byte extraction."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_bitslice_primitives_match_scalar_mt19937(tmp_path):
    exe = tmp_path / "bs_selftest"
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "fate-llm_amd", "csrc"),
                    os.path.join(ROOT, "tools", "bs", "bs_selftest.cpp"), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "bs_selftest ok" in r.stdout
