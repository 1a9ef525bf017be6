"""Diagnostic (GPU): torch_rocm f16 update vs torch's device ops, seed by seed, on the
layout of tests/test_gpu_fuzz.py::test_random_call_matches_torch_on_device[2]; for each
differing element: the inputs and which rounding (once / twice) of g z and of lr t the
device result follows."""
import json
import os
import sys
from fractions import Fraction as Fr

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fate-llm_amd", "python"))
import torch  # noqa: E402

from fate_llm.algo.fedkseed import codec  # noqa: E402

TD = {"float32": torch.float32, "bfloat16": torch.bfloat16, "float16": torch.float16}
dev = torch.device("cuda", 0)


def rn16(fr):  # exact rational -> nearest f16, ties to even
    v = np.float16(float(fr))
    c = [v, np.nextafter(v, np.float16(np.inf)), np.nextafter(v, np.float16(-np.inf))]
    return min(c, key=lambda h: (abs(Fr(float(h)) - fr), int(np.array(h).view(np.uint16)) & 1))


def combos(p, z, g, lr):
    out = {}
    g32 = np.float32(g)
    for gn in ("once", "twice"):
        gz = rn16(Fr(float(g32)) * Fr(float(z))) if gn == "once" else np.float16(np.float32(g32) * np.float32(z))
        for wn in ("once", "twice"):
            w = rn16(Fr(float(np.float32(lr))) * Fr(float(gz))) if wn == "once" else np.float16(np.float32(lr) * np.float32(gz))
            out[f"gz_{gn}/w_{wn}"] = float(rn16(Fr(float(p)) - Fr(float(w))))
    return out


rng = np.random.default_rng(5000 + 2)
nt = int(rng.integers(1, 8))
sizes = [int(rng.choice([int(rng.integers(1, 64)), int(rng.integers(64, 5000)), int(rng.integers(5000, 1 << 20))]))
         for _ in range(nt)]
dtypes = [str(rng.choice(["bfloat16", "bfloat16", "bfloat16", "float32", "float16"])) for _ in range(nt)]
lrs = [float(rng.choice([1e-5, 1e-3])) for _ in range(nt)]
wds = [[None, 0.0, 0.01][int(rng.integers(0, 3))] for _ in range(nt)]
k = int(rng.integers(1, 9))
seeds = [int(s) for s in rng.integers(0, 2**40, k)]
vals = [float(v) for v in rng.normal(0.0, 20.0, k)]
gen = torch.Generator(dev).manual_seed(2)
base = [torch.empty(n, dtype=TD[d], device=dev).normal_(0.0, 0.02, generator=gen) for n, d in zip(sizes, dtypes)]
print(json.dumps({"sizes": sizes, "dtypes": dtypes, "lrs": lrs, "wds": wds}), flush=True)
ref = [b.clone() for b in base]
got = [b.clone() for b in base]
tally = {}
for sd, g in zip(seeds, vals):
    torch.manual_seed(sd)
    zs = [torch.normal(mean=0, std=1, size=p.size(), device=dev, dtype=p.dtype) for p in ref]
    before = [p.clone() for p in ref]
    for p, z, lr, wd in zip(ref, zs, lrs, wds):
        p.data = (p.data - lr * (g * z + wd * p.data)) if wd is not None else (p.data - lr * (g * z))
    codec.directional_step([codec.ParamSpec(t, lr=lr, weight_decay=wd) for t, lr, wd in zip(got, lrs, wds)], [sd], [g],
                           stream_mode="torch_rocm")
    torch.cuda.synchronize()
    for i, d in enumerate(dtypes):
        if d != "float16":
            continue
        diff = (got[i].view(torch.int16) != ref[i].view(torch.int16)).nonzero().flatten().tolist()
        for e in diff[:6]:
            pb, z = np.float16(before[i][e].item()), np.float16(zs[i][e].item())
            c = combos(pb, z, g, lrs[i])
            match = [kk for kk, v in c.items() if v == ref[i][e].item()]
            for m in match:
                tally[m] = tally.get(m, 0) + 1
            print(json.dumps({"seed": sd, "g": g, "lr": lrs[i], "wd": wds[i], "elem": e, "p": float(pb), "z": float(z),
                              "torch": ref[i][e].item(), "codec": got[i][e].item(), "matches": match}), flush=True)
        got[i].copy_(ref[i])
print(json.dumps({"tally": tally}), flush=True)
