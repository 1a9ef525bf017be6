"""The reference's GPU path beside the drop-in's, on the 7B bf16 layout (one MI355X).

A reference client whose model sits on the GPU draws z with torch's HIP generator
(zo_utils.py:47 passes device=param.data.device) and applies the update with torch ops
(zo_utils.py:48-52); reference_step below repeats exactly those torch calls.  Timed here:
  * reference loop on the GPU (torch.normal + elementwise ops per tensor and seed), a few
    seeds, per seed;
  * the drop-in's torch_rocm stream (bit-identical to that loop, tests/test_gpu_torch_rocm.py)
    and torch_cpu stream, K seeds each, per seed.
Prints one JSON line.  python tools/rocm_rate.py [--k 64] [--ref-seeds 3] [--wd 0.0]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fate-llm_amd", "python"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def reference_step(params, seed, g, lr, weight_decay):
    """zo_utils.directional_derivative_step's torch calls (zo_utils.py:42-52), here on the
    parameters' device: the reference's own GPU path, the baseline -- not the drop-in."""
    torch.manual_seed(seed)
    for p in params:
        z = torch.normal(mean=0, std=1, size=p.data.size(), device=p.data.device, dtype=p.data.dtype)
        if weight_decay is not None:
            p.data = p.data - lr * (g * z + weight_decay * p.data)
        else:
            p.data = p.data - lr * (g * z)


def timed(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    return time.perf_counter() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=64)
    ap.add_argument("--ref-seeds", type=int, default=3)
    ap.add_argument("--wd", type=float, default=0.0)
    ap.add_argument("--modes", default="torch_rocm,torch_cpu", help="drop-in streams to time")
    args = ap.parse_args()
    from fate_llm.algo.fedkseed import codec
    dev = torch.device("cuda", 0)
    shapes = bench.llama7b_shapes()
    params = [torch.empty(s, dtype=torch.bfloat16, device=dev).normal_(0.0, 0.02) for s in shapes]
    total = sum(p.numel() for p in params)
    g = torch.Generator().manual_seed(7)
    seeds = torch.randint(0, 2**32, (args.k,), generator=g).tolist()
    vals = (torch.randn(args.k, generator=g, dtype=torch.float64) * 20).tolist()
    out = {"params": total, "dtype": "bf16", "weight_decay": args.wd, "lr": 1e-5}

    # the reference's loop on the GPU (its own torch calls), first seed as warm-up
    ref_s = None
    if args.ref_seeds > 0:
        reference_step(params, seeds[0], vals[0], 1e-5, args.wd)
        t = timed(lambda: [reference_step(params, s, v, 1e-5, args.wd)
                           for s, v in zip(seeds[1:1 + args.ref_seeds], vals[1:1 + args.ref_seeds])])
        ref_s = t / args.ref_seeds
        out["reference_gpu_torch"] = {"s_per_seed": round(ref_s, 5), "seeds_timed": args.ref_seeds,
                                      "reconstruct_4055_seeds_s": round(ref_s * 4055, 1)}
    out["lib"] = os.environ.get("FKS_LIB_OVERRIDE", "libfks.so")
    specs = [codec.ParamSpec(p, lr=1e-5, weight_decay=args.wd) for p in params]
    for mode in args.modes.split(","):
        codec.directional_step(specs, seeds[:20], vals[:20], stream_mode=mode)  # plans, warm-up
        t = timed(lambda: codec.directional_step(specs, seeds, vals, stream_mode=mode))
        out[mode] = {"s_per_seed": round(t / args.k, 5), "k": args.k,
                     "reconstruct_4055_seeds_s": round(t / args.k * 4055, 2),
                     "vs_reference_gpu": round(ref_s / (t / args.k), 2) if ref_s else None}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
