"""C4 (BASELINE.json configs[3]): LLaMA-70B-shaped fp32 buffer, K=4096, fp32 path.

The 723 tensors (68,976,648,192 params, 275.9 GB fp32) stay resident in
one MI355X's HBM (288 GB).  The stream is processed in HBM-sized chunks: chunk c of C is
the c-th run of MT19937 blocks of the parameter stream (codec element shard c/C, the
multi-GPU sharding run one chunk after another), each chunk taking every seed in order,
so the result is bit-identical to one unchunked call.

Full K=4096 is 214 passes of 19 seeds over 69e9 params (about ten minutes): the run
times a sample of K_s seeds (whole passes) per chunk and scales linearly in the pass
count (linearity checked on two sample sizes).  Prints one JSON line.

  python tools/c4_70b.py [--chunks 8] [--ks 19,38] [--scale 1.0] [--check K]

--check K (needs room for a second copy of the buffer, e.g. --scale 0.4): before timing,
reconstruct K seeds chunked and, on a clone, in one unchunked call, and report whether
the two agree bit for bit (tests/test_gpu_c4.py holds the oracle comparison).
"""
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


def llama70b_shapes():
    """LlamaConfig(hidden 8192, 80 layers, intermediate 28672, vocab 32000, 64 heads,
    8 KV heads) in named_parameters order: 723 tensors, 68,976,648,192 elements."""
    h, inter, v, L, kv = 8192, 28672, 32000, 80, 1024
    shapes = [(v, h)]
    for _ in range(L):
        shapes += [(h, h), (kv, h), (kv, h), (h, h), (inter, h), (inter, h), (h, inter), (h,), (h,)]
    shapes += [(h,), (v, h)]
    return shapes


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", type=int, default=8)
    ap.add_argument("--ks", default="19,38")
    ap.add_argument("--scale", type=float, default=1.0, help="fraction of every tensor's rows (smoke runs)")
    ap.add_argument("--progress", action="store_true", help="one stderr line per chunk (long runs)")
    ap.add_argument("--check", type=int, default=0, help="K seeds: chunked vs unchunked, bit for bit")
    args = ap.parse_args()
    from fate_llm.algo.fedkseed import codec

    dev = torch.device("cuda", 0)
    shapes = llama70b_shapes()
    if args.scale != 1.0:
        shapes = [(max(1, int(s[0] * args.scale)),) + tuple(s[1:]) for s in shapes]
    total = sum(bench.numel(s) for s in shapes)
    need = total * 4
    free, cap = torch.cuda.mem_get_info(dev)
    if need + (2 << 30) > free:
        print(json.dumps({"error": f"needs {need / 1e9:.1f} GB, {free / 1e9:.1f} GB free of {cap / 1e9:.1f}"}))
        return 1
    flat = torch.empty(total, dtype=torch.float32, device=dev)
    flat.normal_(0.0, 0.02, generator=torch.Generator(device=dev).manual_seed(0))
    views, off = [], 0
    for s in shapes:
        views.append(flat[off:off + bench.numel(s)].view(s))
        off += bench.numel(s)
    specs = [codec.ParamSpec(v, lr=1e-5, weight_decay=0.01) for v in views]
    seeds, scalars = bench.synthetic_seeds(4096)
    keep = [(s, g) for s, g in zip(seeds, scalars) if g != 0.0]
    k_full = len(keep)
    passes_full = -(-k_full // 19)

    if args.check:
        ks, kv = [s for s, _ in keep[:args.check]], [g for _, g in keep[:args.check]]
        clone = flat.clone()
        cviews, off = [], 0
        for s in shapes:
            cviews.append(clone[off:off + bench.numel(s)].view(s))
            off += bench.numel(s)
        for c in range(args.chunks):
            codec.directional_step(specs, ks, kv, shard=c, nshards=args.chunks)
        codec.directional_step([codec.ParamSpec(v, lr=1e-5, weight_decay=0.01) for v in cviews], ks, kv)
        torch.cuda.synchronize()
        differ = int((flat.view(torch.int32) != clone.view(torch.int32)).sum().item())
        print(json.dumps({"check": "chunked vs unchunked", "k": len(ks), "chunks": args.chunks, "params": total,
                          "elements_differing": differ, "bit_identical": differ == 0}), flush=True)
        del clone, cviews
        if differ:
            return 2

    # warm the plan caches (one per chunk) with one seed
    for c in range(args.chunks):
        codec.directional_step(specs, [keep[0][0]], [keep[0][1]], shard=c, nshards=args.chunks)
    torch.cuda.synchronize()

    samples = []
    for k in [int(x) for x in args.ks.split(",")]:
        ks, kv = [s for s, _ in keep[:k]], [g for _, g in keep[:k]]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with codec.profile() as prof:
            for c in range(args.chunks):
                codec.directional_step(specs, ks, kv, shard=c, nshards=args.chunks)
                if args.progress:  # chunks run back to back anyway; the sync only reports
                    torch.cuda.synchronize()
                    print(json.dumps({"k": k, "chunk": c, "t_s": round(time.perf_counter() - t0, 2)}),
                          file=sys.stderr, flush=True)
            torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        passes = -(-len(ks) // 19)
        samples.append({"k": len(ks), "passes": passes, "s": round(dt, 3), "s_per_pass": round(dt / passes, 4),
                        "apply_ms_per_launch": round(prof.apply_ms / max(prof.n_apply, 1), 3),
                        "launches": prof.n_apply, "jump_ms": round(prof.jump_ms, 1)})
        print(json.dumps(samples[-1]), flush=True)
    per_pass = samples[-1]["s_per_pass"]
    t_full = per_pass * passes_full
    out = {
        "config": "C4: 1xMI355X, LLaMA-70B-shaped fp32 buffer, K=4096, HBM-resident, chunked",
        "params": total, "bytes": need, "tensors": len(shapes), "chunks": args.chunks,
        "k_nonzero": k_full, "passes_full": passes_full, "samples": samples,
        "linearity_s_per_pass": [s["s_per_pass"] for s in samples],
        "t_full_s_extrapolated": round(t_full, 1),
        "GBps_extrapolated": round(need / t_full / 1e9, 4),
        "seed_param_per_s": round(total * 19 / per_pass, 1),
        "data": "synthetic: random-init N(0, 0.02^2) fp32, seeds/scalars of bench.synthetic_seeds(4096)",
    }
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
