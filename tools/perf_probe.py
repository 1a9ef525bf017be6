"""Quick timing probe of the codec on the GPU (development tool, not the bench)."""
import sys, time, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "fate-llm_amd", "python"))
import torch
from fate_llm.algo.fedkseed import codec

def run(n, k, dtype, reps=2):
    dev = torch.device("cuda", 0)
    buf = torch.empty(n, dtype=dtype, device=dev).normal_(0, 0.02)
    specs = [codec.ParamSpec(buf, lr=1e-5, weight_decay=0.01)]
    g = torch.Generator().manual_seed(1)
    seeds = torch.randint(0, 2**32, (k,), generator=g).tolist()
    vals = (torch.randn(k, generator=g, dtype=torch.float64) * 20).tolist()
    codec.directional_step(specs, seeds[:28], vals[:28])  # warm (jump polys, tables)
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        t = time.time(); codec.directional_step(specs, seeds, vals); torch.cuda.synchronize(); best = min(best, time.time() - t)
    el = n * k
    print(f"{dtype} n={n} k={k}: {best*1e3:.1f} ms  {el/best/1e9:.2f} G seed-elem/s  "
          f"{best/el*1e12:.2f} ps/seed-elem  7B K=4096 est {6738415616*4096*best/el:.1f} s", flush=True)

for dt in (torch.bfloat16, torch.float32):
    run(1 << 24, 28, dt)
    run(1 << 26, 56, dt)
    run(1 << 28, 280, dt, reps=1)
