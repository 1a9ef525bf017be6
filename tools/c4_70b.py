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

--verify OUT.npz (full size, with --ks 4096): checks of the 276 GB result itself, around
the timed run (zo_utils.py:47-49 over 723 tensors, fedkseed.py:136-141):
  * the first 4096 elements of embed_tokens before and after the whole reconstruct, with
    the seeds and scalars, are written to OUT.npz; tests/test_c4_fullsize_record.py
    replays them through the oracle (tools/ does not run the oracle);
  * a chunk boundary recomputed by ONE call: the elements within --window of the boundary
    between chunks C/2 - 1 and C/2 (computed by two calls in the timed run) are saved,
    reset to their initial values and reconstructed again by a single element-shard call
    whose shard holds the boundary in its interior (the rest of that shard is updated a
    second time, which the check ignores); the window must come back bit for bit.
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
    ap.add_argument("--verify", default="", help="OUT.npz: full-size checks of the reconstructed buffer")
    ap.add_argument("--window", type=int, default=1 << 24, help="--verify: elements on each side of the boundary")
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
    if args.verify:
        if len(args.ks.split(",")) != 1:
            raise SystemExit("--verify times one sample: give --ks a single K (4096 for the full run)")
        # the values the timed run starts from (the warm-up seed above is one more step of
        # the same stream: the oracle replay starts after it as well)
        emb0 = flat[:4096].cpu().numpy().copy()
        bnd = codec.shard_range(specs, args.chunks // 2, args.chunks)[0]  # first element of chunk C/2
        lo, hi = max(0, bnd - args.window), min(total, bnd + args.window)
        win0 = flat[lo:hi].cpu()

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
    verify = None
    if args.verify:
        ks, kv = [s for s, _ in keep[:samples[-1]["k"]]], [g for _, g in keep[:samples[-1]["k"]]]
        emb1 = flat[:4096].cpu().numpy().copy()
        win1 = flat[lo:hi].cpu()
        # the single call: the element shard of an N-way split that holds [lo, hi) inside
        one = None
        for n in range(3, 64):
            for r in range(n):
                a, b = codec.shard_range(specs, r, n)
                if a < lo and hi < b:
                    one = (r, n, a, b)
                    break
            if one:
                break
        flat[lo:hi].copy_(win0.to(dev))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        codec.directional_step(specs, ks, kv, shard=one[0], nshards=one[1])
        torch.cuda.synchronize()
        t_one = time.perf_counter() - t0
        win2 = flat[lo:hi].cpu()
        differ = int((win1.view(torch.int32) != win2.view(torch.int32)).sum().item())
        import numpy as np
        np.savez_compressed(args.verify, embed_before=emb0, embed_after=emb1,
                            seeds=np.asarray(ks, dtype=np.uint64), scalars=np.asarray(kv, dtype=np.float64),
                            lr=np.float64(1e-5), weight_decay=np.float64(0.01), params=np.int64(total))
        verify = {"embed_prefix_file": os.path.basename(args.verify), "boundary_element": bnd,
                  "window": [lo, hi], "single_call_shard": [one[0], one[1]], "single_call_elements": [one[2], one[3]],
                  "single_call_s": round(t_one, 2), "window_elements_differing": differ,
                  "boundary_bit_identical": differ == 0,
                  "changed_by_reconstruct": int((win1.view(torch.int32) != win0.view(torch.int32)).sum().item())}
        print(json.dumps({"verify": verify}), flush=True)
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
        "stream": codec.resolve_stream_mode("cuda"),
        "fp32_flavour": codec.cpu_fp32_flavour(),
    }
    if verify is not None:
        out["verify"] = verify
    print(json.dumps(out), flush=True)
    return 0 if verify is None or verify["boundary_bit_identical"] else 3


if __name__ == "__main__":
    sys.exit(main())
