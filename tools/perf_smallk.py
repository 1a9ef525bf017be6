"""Small-K cost on the 7B bf16 layout (the ZO local step's perturb / update calls):
wall time per call (synchronised), device time of the apply and jump kernels, and the
host-side share.  Every repetition uses a new seed (the jumped-window cache misses);
"zo_step" is the three calls of one zeroth-order step with one seed (perturb +eps,
perturb -2 eps, restore + update), where the second and third reuse the windows.
python tools/perf_smallk.py [--params N] [--reps R]"""
import argparse
import json
import os
os.environ.setdefault("FKS_STREAM_MODE", "torch_cpu")  # the CPU-generator stream these measurements use
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fate-llm_amd", "python"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--params", type=int, default=0)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--ks", default="1,2,4,8,19")
    ap.add_argument("--calls", default="", help="comma list: perturb,perturb_step,zo_step,replay (default all)")
    args = ap.parse_args()
    from fate_llm.algo.fedkseed import codec

    dev = torch.device("cuda", 0)
    shapes = [(args.params,)] if args.params else bench.llama7b_shapes()
    total = sum(bench.numel(s) for s in shapes)
    flat = torch.empty(total, dtype=torch.bfloat16, device=dev).normal_(0.0, 0.02)
    views, off = [], 0
    for s in shapes:
        views.append(flat[off:off + bench.numel(s)].view(s))
        off += bench.numel(s)
    specs = [codec.ParamSpec(v, lr=1e-5, weight_decay=0.01) for v in views]
    seeds, scalars = bench.synthetic_seeds(64)
    scalars = [g if g != 0.0 else 1.0 for g in scalars]

    def measure(name, fn):
        fn(0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with codec.profile() as prof:
            for i in range(args.reps):
                fn(1 + i)
            torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / args.reps * 1e3
        t1 = time.perf_counter()
        for i in range(args.reps):
            fn(1 + args.reps + i)
        host = (time.perf_counter() - t1) / args.reps * 1e3  # enqueue only (async)
        torch.cuda.synchronize()
        rec = {"call": name, "wall_ms": round(wall, 3), "apply_ms": round(prof.apply_ms / args.reps, 3),
               "jump_ms": round(prof.jump_ms / args.reps, 3), "enqueue_ms": round(host, 3),
               "GBps": round(total * 2 / wall * 1e-6, 1)}
        print(json.dumps(rec), flush=True)

    sd = lambda i: seeds[i % len(seeds)]  # noqa: E731

    def zo_step(i):
        codec.perturb(views, sd(i), 5e-4)
        codec.perturb(views, sd(i), -1e-3)
        codec.perturb_step(specs, sd(i), [5e-4] * len(specs), 1.5)

    want = set(args.calls.split(",")) if args.calls else {"perturb", "perturb_step", "zo_step", "replay"}
    if "perturb" in want:
        measure("perturb", lambda i: codec.perturb(views, sd(i), 5e-4))
    if "perturb_step" in want:
        measure("perturb_step", lambda i: codec.perturb_step(specs, sd(i), [5e-4] * len(specs), 1.5))
    if "zo_step" in want:
        measure("zo_step (3 calls)", zo_step)
    if "replay" in want:
        # the same seed every time: after the first call, perturbs replay the stored z indices
        measure("perturb, same seed (z-index replay)", lambda i: codec.perturb(views, sd(0), -1e-3))
    for k in [int(x) for x in args.ks.split(",") if x]:
        measure(f"directional_step K={k}",
                lambda i: codec.directional_step(specs, [sd(i + j) for j in range(k)], scalars[:k]))


if __name__ == "__main__":
    main()
