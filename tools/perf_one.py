"""One bf16 reconstruct pass (28 seeds, 64M params) for counter collection."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "fate-llm_amd", "python"))
import torch
from fate_llm.algo.fedkseed import codec
dev = torch.device("cuda", 0)
n, k = 1 << 26, 28
dt = torch.bfloat16 if (len(sys.argv) < 2 or sys.argv[1] == "bf16") else torch.float32
buf = torch.empty(n, dtype=dt, device=dev).normal_(0, 0.02)
specs = [codec.ParamSpec(buf, lr=1e-5, weight_decay=0.01)]
g = torch.Generator().manual_seed(1)
seeds = torch.randint(0, 2**32, (k,), generator=g).tolist()
vals = (torch.randn(k, generator=g, dtype=torch.float64) * 20).tolist()
for _ in range(2):
    codec.directional_step(specs, seeds, vals)
torch.cuda.synchronize()
print("done")
