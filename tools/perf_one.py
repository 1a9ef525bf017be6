"""One reconstruct of K seeds over an N-param buffer, twice, for kernel timing /
counter collection (rocprofv3 around it).  python tools/perf_one.py [bf16|f32] [log2 N] [K]
Defaults: bf16, N = 2^30, weight decay PERF_WD (default 0.01) (chunks as long as the 7B bench's order of magnitude), K = 19;
PERF_STREAM=torch_rocm draws the torch_rocm stream (fks_philox_vec_kernel)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "fate-llm_amd", "python"))
import torch  # noqa: E402

from fate_llm.algo.fedkseed import codec  # noqa: E402

dev = torch.device("cuda", 0)
dt = torch.float32 if (len(sys.argv) > 1 and sys.argv[1] == "f32") else torch.bfloat16
n = 1 << (int(sys.argv[2]) if len(sys.argv) > 2 else 30)
k = int(sys.argv[3]) if len(sys.argv) > 3 else 19
buf = torch.empty(n, dtype=dt, device=dev).normal_(0, 0.02)
wd = os.environ.get("PERF_WD", "0.01")  # 'none' = no weight-decay term
specs = [codec.ParamSpec(buf, lr=1e-5, weight_decay=None if wd == "none" else float(wd))]
g = torch.Generator().manual_seed(1)
seeds = torch.randint(0, 2**32, (k,), generator=g).tolist()
vals = (torch.randn(k, generator=g, dtype=torch.float64) * 20).tolist()
for _ in range(2):
    codec.directional_step(specs, seeds, vals, stream_mode=os.environ.get("PERF_STREAM", "torch_cpu"))
torch.cuda.synchronize()
print("done")
