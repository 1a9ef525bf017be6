"""Per-rank work of the element-sharded reconstruct, measured on ONE GPU: rank 0's shard of
the 7B bf16 K=4096 reconstruct for N = 1, 2, 4, 8 (the work each rank of an N-GPU run
does; ranks share nothing on the data path).  Predicts the driver's strong-scaling
efficiency t_1 / (N t_N) up to the max-over-ranks skew.  --warm: every rank keeps its
shard's jumped windows in the reconstruct window cache (codec cache_windows, a client's
second and later rounds): the cold call fills it, the timed call finds every seed there.
python tools/shard_rank_time.py [--ns 1,2,4,8] [--wd 0.0] [--warm]"""
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
    ap.add_argument("--ns", default="1,2,4,8")
    ap.add_argument("--wd", type=float, default=0.0, help="weight decay (bench.py's default 0.0)")
    ap.add_argument("--warm", action="store_true", help="time the second reconstruct with the window cache filled")
    args = ap.parse_args()
    from fate_llm.algo.fedkseed import codec
    dev = torch.device("cuda", 0)
    shapes = bench.llama7b_shapes()
    total = sum(bench.numel(s) for s in shapes)
    flat = torch.empty(total, dtype=torch.bfloat16, device=dev).normal_(0.0, 0.02)
    views, off = [], 0
    for s in shapes:
        views.append(flat[off:off + bench.numel(s)].view(s))
        off += bench.numel(s)
    specs = [codec.ParamSpec(v, lr=1e-5, weight_decay=args.wd) for v in views]
    seeds, vals = bench.synthetic_seeds(4096)
    keep = [(s, v) for s, v in zip(seeds, vals) if v != 0.0]
    ks, kv = [s for s, _ in keep], [v for _, v in keep]
    t1 = None
    for n in [int(x) for x in args.ns.split(",")]:
        if args.warm:  # fill the cache with this shard's windows of every seed
            codec.directional_step(specs, ks, kv, shard=0, nshards=n, cache_windows=True)
        else:
            codec.directional_step(specs, ks[:40], kv[:40], shard=0, nshards=n)  # plan + warm-up
        torch.cuda.synchronize()
        h0, m0 = codec.jwin_stats()
        t0 = time.perf_counter()
        with codec.profile() as prof:
            codec.directional_step(specs, ks, kv, shard=0, nshards=n, cache_windows=args.warm)
            torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        h1, m1 = codec.jwin_stats()
        t1 = t1 or dt * n
        print(json.dumps({"wd": args.wd, "nshards": n, "warm": args.warm, "rank0_s": round(dt, 3),
                          "apply_s": round(prof.apply_ms / 1e3, 3), "jump_s": round(prof.jump_ms / 1e3, 3),
                          "jwin_hits": h1 - h0, "jwin_misses": m1 - m0,
                          "predicted_efficiency": round(t1 / (n * dt), 4)}), flush=True)


if __name__ == "__main__":
    main()
