"""The torch_rocm stream at the bench's size: one reconstruct of the LLaMA-7B bf16 layout
(bench.llama7b_shapes) from K seeds through the codec (fks_philox_kernel) and, for a few
seeds, the reference's own arithmetic as torch ops on the same GPU (oracle/torch_replica.py:
torch.manual_seed, torch.normal(device="cuda"), the update expression) -- the two are
bit-identical (tests/test_gpu_torch_rocm.py); printed: ms per seed of each, scaled to
the 4055 non-zero seeds of K=4096.
  python tools/perf_rocm.py [K] [replica_seeds]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fate-llm_amd", "python"))
import torch  # noqa: E402

import bench  # noqa: E402
from fate_llm.algo.fedkseed import codec  # noqa: E402
from oracle import torch_replica as R  # noqa: E402


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    kr = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    dev = torch.device("cuda", 0)
    shapes = bench.llama7b_shapes()
    n = [bench.numel(s) for s in shapes]
    flat = torch.empty(sum(n), dtype=torch.bfloat16, device=dev).normal_(0, 0.02)
    views, off = [], 0
    for s, m in zip(shapes, n):
        views.append(flat[off:off + m].view(s))
        off += m
    seeds, vals = bench.synthetic_seeds(k)
    keep = [(s, g) for s, g in zip(seeds, vals) if g != 0.0]
    ks, kv = [s for s, _ in keep], [g for _, g in keep]
    specs = [codec.ParamSpec(v, lr=1e-5, weight_decay=0.0) for v in views]
    codec.directional_step(specs, ks[:2], kv[:2], stream_mode="torch_rocm")  # plan
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with codec.profile() as prof:
        codec.directional_step(specs, ks, kv, stream_mode="torch_rocm")
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ms_seed = dt * 1e3 / len(ks)
    params = [v.clone() for v in views[:]]
    del flat
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    R.reconstruct(params, ks[:kr], kv[:kr], 1e-5, 0.0)
    torch.cuda.synchronize()
    ref_ms_seed = (time.perf_counter() - t0) * 1e3 / kr
    print(json.dumps({"params": sum(n), "k": len(ks), "codec_torch_rocm_ms_per_seed": round(ms_seed, 3),
                      "codec_kernel_ms": round(prof.apply_ms, 1), "launches": prof.n_apply,
                      "codec_7b_k4096_s": round(ms_seed * 4055 / 1e3, 2),
                      "reference_torch_ops_on_gpu_ms_per_seed": round(ref_ms_seed, 2),
                      "reference_7b_k4096_s": round(ref_ms_seed * 4055 / 1e3, 1),
                      "speedup": round(ref_ms_seed / ms_seed, 2)}), flush=True)


if __name__ == "__main__":
    main()
