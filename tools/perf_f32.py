"""fp32 reconstruct cost (C4's kernel, the full 19-seed fp32 pass): ps per seed*param of
the apply kernels, HIP events.  python tools/perf_f32.py [log2 N] [K] [reps]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "fate-llm_amd", "python"))
import torch  # noqa: E402

from fate_llm.algo.fedkseed import codec  # noqa: E402

n = 1 << (int(sys.argv[1]) if len(sys.argv) > 1 else 28)
k = int(sys.argv[2]) if len(sys.argv) > 2 else 38
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
dev = torch.device("cuda", 0)
buf = torch.empty(n, dtype=torch.float32, device=dev).normal_(0, 0.02)
specs = [codec.ParamSpec(buf, lr=1e-5, weight_decay=0.01)]
g = torch.Generator().manual_seed(1)
seeds = torch.randint(0, 2**32, (k,), generator=g).tolist()
vals = (torch.randn(k, generator=g, dtype=torch.float64) * 20).tolist()
codec.directional_step(specs, seeds, vals)
torch.cuda.synchronize()
t0 = time.perf_counter()
with codec.profile() as prof:
    for _ in range(reps):
        codec.directional_step(specs, seeds, vals)
    torch.cuda.synchronize()
wall = (time.perf_counter() - t0) / reps
print(json.dumps({"params": n, "k": k, "wall_s": round(wall, 4), "apply_ms": round(prof.apply_ms / reps, 3),
                  "jump_ms": round(prof.jump_ms / reps, 3),
                  "ps_per_seed_param": round(prof.apply_ms / reps * 1e9 / (n * k), 4)}))
