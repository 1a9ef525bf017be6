"""Diagnostic (GPU): how torch's device kernel rounds a Half "python float * tensor"
product -- once (the exact product to f16) or twice (to f32, then f16) -- by element
position, tensor size and alignment.  Only the products whose f32 value lies exactly on an
f16 rounding midpoint tell the two apart; counts them by (index mod 8, once/twice)."""
import collections
import json
import sys

import numpy as np
import torch

dev = torch.device("cuda", 0)


def classify(z, g, a):
    z32 = z.float().cpu().numpy().astype(np.float64)
    prod64 = z32 * np.float64(np.float32(g))         # exact (24 x 11 bits)
    prod32 = (z.float() * np.float32(g)).cpu().numpy()  # f32-rounded product
    twice = prod32.astype(np.float16)
    # once: round the exact product to f16 -- via float64 (exact) -> f16 (one rounding)
    once = prod64.astype(np.float16)
    got = a.cpu().numpy()
    diff = np.nonzero(once.view(np.uint16) != twice.view(np.uint16))[0]
    out = collections.Counter()
    for i in diff:
        kind = "once" if got[i].view(np.uint16) == once[i].view(np.uint16) else (
            "twice" if got[i].view(np.uint16) == twice[i].view(np.uint16) else "neither")
        out[(int(i) % 8, kind)] += 1
    return out, len(diff)


res = {}
for n, off in ((177489, 0), (5647, 0), (1 << 20, 0), (1 << 20, 1), (1 << 20, 3), (1001, 0), (64, 0)):
    tot = collections.Counter()
    cases = 0
    for rep in range(40):
        g = float(np.random.default_rng(rep).normal(0, 20))
        buf = torch.randn(n + off, device=dev).to(torch.float16)
        z = buf[off:]
        a = g * z
        torch.cuda.synchronize()
        c, m = classify(z, g, a)
        tot.update(c)
        cases += m
    res[f"n={n},off={off}"] = {"midpoint_cases": cases, "by_pos_kind": {f"{k[0]}:{k[1]}": v for k, v in sorted(tot.items())}}
    print(json.dumps({f"n={n},off={off}": res[f"n={n},off={off}"]}), flush=True)
# lr * tensor too, small scalar
tot = collections.Counter()
for rep in range(40):
    buf = (torch.randn(1 << 20, device=dev) * 30).to(torch.float16)
    a = 1e-5 * buf
    torch.cuda.synchronize()
    c, m = classify(buf, 1e-5, a)
    tot.update(c)
print(json.dumps({"lr=1e-5": {f"{k[0]}:{k[1]}": v for k, v in sorted(tot.items())}}), flush=True)
