"""Adds each serial_straddle.json case's two 53-bit uniforms (hex integers a, b with
u1 = a 2^-53, u2 = b 2^-53) -- what tools/straddle_search.c now prints -- to the fixture,
by stepping the oracle's MT19937 to the case's stream position.  Test infrastructure."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from oracle import fks_oracle as O  # noqa: E402

p = Path(__file__).resolve().parents[1] / "tests" / "golden" / "serial_straddle.json"
d = json.loads(p.read_text())
M = (1 << 53) - 1
for c in d["cases"]:
    g = O.Generator(c["seed"])
    left = c["pos"]
    while left:
        n = min(left, 1 << 24)
        g.u32(n)
        left -= n
    c["u1_bits"] = hex(g.random64() & M)
    c["u2_bits"] = hex(g.random64() & M)
p.write_text(json.dumps(d, indent=1) + "\n")
