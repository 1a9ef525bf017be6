"""bench.py -- FedKSeed reconstruct throughput on MI355X (BASELINE.json metric).

One "step" = one reconstruct of the LLaMA-7B-shaped bf16 parameter buffer
(291 tensors, 6,738,415,616 params, random init N(0, 0.02^2)) from K = 4096
(seed, scalar) pairs -- the loop of ClientTrainer.train_once (fedkseed.py:136-141)
-- device-resident, through the drop-in fate_llm.algo.fedkseed codec (libfks.so).

  python bench.py [--gpus N] [--steps K] [--warmup W]

N > 1 (torch.distributed.run, one rank per GPU): the parameter stream is cut into N
equal runs of MT19937 blocks and rank r reconstructs run r (element sharding: every
element still sees every seed in order, so the result is bit-identical to N = 1 and
no collective touches the data path).  Total work is fixed: "scaling": "strong".

--mode seed-shard runs the north star's C3 variant instead: rank r takes a contiguous
1/N of the seeds, accumulates its f32 delta over the whole buffer (fks_delta_accumulate),
one RCCL all-reduce sums the deltas over xGMI, every rank applies p = a^K p_0 - delta.
Not the reference's rounding (DESIGN.md §7 gives its measured deviation); the default
(--mode sequential) is the bit-exact path.

Rank 0 prints ONE JSON line: the metric, the dominant kernel's roofline (HBM, as the
north star asks, plus the VALU roofline that actually binds), and the reference CPU
path timed on this host in the same run (cpu_baseline).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "fate-llm_amd", "python"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

LLAMA7B_PARAMS = 6_738_415_616
HBM_PEAK_GBS = 8000.0                 # MI355X spec (MI355X_MICROARCH.md)
# non-packed VALU issue peak: 256 CUs x 4 SIMDs x 16 lanes x 2.4 GHz (a wave64 instruction
# occupies its SIMD for 4 cycles) = 39.3 T lane-op/s; packed f32 ops count once here
VALU_PEAK_TLANEOPS = 256 * 4 * 16 * 2.4e9 / 1e12


def llama7b_shapes():
    """Parameter shapes of LlamaConfig() (hidden 4096, 32 layers, intermediate 11008,
    vocab 32000) in named_parameters order; all land in the decay group (RMSNorm is not
    in ALL_LAYERNORM_LAYERS, no biases), SURVEY.md §8."""
    h, inter, v, L = 4096, 11008, 32000, 32
    shapes = [(v, h)]
    for _ in range(L):
        shapes += [(h, h), (h, h), (h, h), (h, h), (inter, h), (inter, h), (h, inter), (h,), (h,)]
    shapes += [(h,), (v, h)]
    return shapes


def numel(s):
    n = 1
    for d in s:
        n *= d
    return n


def synthetic_seeds(k):
    g1 = torch.Generator().manual_seed(1)
    seeds = torch.randint(0, 2**32, (k,), generator=g1, dtype=torch.int64).tolist()
    g2 = torch.Generator().manual_seed(2)
    scalars = (torch.randn(k, generator=g2, dtype=torch.float64) * 20.0).tolist()
    for i in range(0, k, 100):  # 1 % exact zeros: skipped, as fedkseed.py:137 does
        scalars[i] = 0.0
    return seeds, scalars


PMC_SUMMARY = "pmc_apply_r01e.json"   # the bf16 slice kernel (fks_apply_bs_kernel)


def load_pmc_summary():
    """Per-launch HBM traffic and VALU lane-ops per seed-element of the dominant kernel,
    from the committed rocprofv3 --pmc pass (profiles/PMC_SUMMARY)."""
    p = os.path.join(ROOT, "profiles", PMC_SUMMARY)
    try:
        with open(p) as f:
            return json.load(f)
    except OSError:
        return {}


def cpu_baseline(dtype, budget_s):
    """The reference's CPU path (torch.manual_seed + torch.normal + the update
    expression of zo_utils.py:49, re-typed in oracle/torch_replica.py) on a bounded
    sample, scaled to the metric: GB/s of the 7B buffer reconstructed from K=4096."""
    from oracle import torch_replica as R
    threads = torch.get_num_threads()
    n = 1 << 24
    p = [torch.randn(n, generator=torch.Generator().manual_seed(0)).mul_(0.02).to(dtype)]
    seeds, scalars = synthetic_seeds(4096)
    seeds, scalars = [s for s, g in zip(seeds, scalars) if g != 0.0], [g for g in scalars if g != 0.0]
    done, t0 = 0, time.perf_counter()
    while done < len(seeds) and time.perf_counter() - t0 < budget_s:
        R.reconstruct(p, seeds[done:done + 2], scalars[done:done + 2], 1e-5, 0.01)
        done += 2
    dt = time.perf_counter() - t0
    ns_per = dt / (n * done) * 1e9
    t7b = LLAMA7B_PARAMS * 4096 * 0.99 * ns_per * 1e-9
    return {
        "value": LLAMA7B_PARAMS * 2 / t7b / 1e9, "unit": "GB/s",
        "cores": threads, "kind": "port",
        "sample": f"torch CPU replica of zo_utils.directional_derivative_step (oracle/torch_replica.py), "
                  f"{n} bf16 params x {done} seeds in {dt:.1f} s = {ns_per:.2f} ns per seed*param, "
                  f"scaled linearly to 6.74e9 params x 4055 non-zero seeds ({t7b / 3600:.1f} h); "
                  f"torch.normal holds the generator mutex (single-threaded RNG), elementwise ops on "
                  f"{threads} threads",
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--k", type=int, default=4096)
    ap.add_argument("--params", type=int, default=0, help="override: flat buffer of this many params (dev only)")
    ap.add_argument("--cpu-budget", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--mode", choices=("sequential", "seed-shard"), default="sequential")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=dev)

    from fate_llm.algo.fedkseed import codec

    dtype = torch.bfloat16
    shapes = [(args.params,)] if args.params else llama7b_shapes()
    total = sum(numel(s) for s in shapes)
    flat = torch.empty(total, dtype=dtype, device=dev)
    gen = torch.Generator(device=dev).manual_seed(0)
    flat.normal_(0.0, 0.02, generator=gen)
    views, off = [], 0
    for s in shapes:
        views.append(flat[off:off + numel(s)].view(s))
        off += numel(s)
    specs = [codec.ParamSpec(v, lr=1e-5, weight_decay=0.01) for v in views]
    seeds, scalars = synthetic_seeds(args.k)
    keep = [(s, g) for s, g in zip(seeds, scalars) if g != 0.0]
    ks, kv = [s for s, _ in keep], [g for _, g in keep]
    seed_shard = args.mode == "seed-shard"
    if seed_shard:
        from fate_llm.algo.fedkseed import zo_utils
        groups = [{"params": views, "lr": 1e-5, "weight_decay": 0.01}]
        delta = torch.empty(total, dtype=torch.float32, device=dev)

    def step():
        if seed_shard:
            zo_utils.reconstruct_seed_sharded_(groups, ks, kv, lr=1e-5, weight_decay=0.01, delta=delta)
        else:
            codec.directional_step(specs, ks, kv, shard=rank, nshards=world)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with codec.profile() as prof:
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    ms_per_step = dt / args.steps * 1e3
    buf_bytes = total * 2
    value = buf_bytes / (dt / args.steps) / 1e9

    # roofline of the dominant kernel, per launch, this rank: the bf16 slice kernel
    # (fks_apply_bs_kernel, 32 seeds per launch) for every reconstruct of >= 20 seeds
    rank_params = total if seed_shard else total / world
    n_apply = max(prof.n_apply, 1)
    avg_apply_s = prof.apply_ms / n_apply / 1e3
    rank_seeds = len(ks) * (rank + 1) // world - len(ks) * rank // world if seed_shard else len(ks)
    seeds_per_launch = rank_seeds * args.steps / n_apply
    # read + write the (shard of the) buffer once: bf16 parameters, or the f32 delta
    alg_bytes = 2 * rank_params * (4 if seed_shard else 2)
    hbm_achieved = alg_bytes / avg_apply_s / 1e9
    pmc = load_pmc_summary()
    lane_ops = pmc.get("valu_lane_ops_per_seed_param")
    units = rank_params * seeds_per_launch               # seed*param updates per launch
    valu = None
    if lane_ops:
        ach = units * lane_ops / avg_apply_s / 1e12
        valu = {"bound": "valu", "achieved": round(ach, 3), "peak": VALU_PEAK_TLANEOPS, "unit": "Tlane-op/s",
                "frac": round(ach / VALU_PEAK_TLANEOPS, 4), "lane_ops_per_unit": lane_ops,
                "unit_def": "one seed*param update (z draw + update); lane-ops = rocprofv3 SQ_INSTS_VALU x 64 per "
                            f"seed*param (profiles/{PMC_SUMMARY}); peak = non-packed VALU issue rate"}
    traffic = None if seed_shard else pmc.get("hbm_bytes_per_param_per_launch")
    if seed_shard:
        valu = None  # the committed PMC summary is the sequential kernel's
    out = {
        "metric": "GB/s param buffer reconstructed from (seed,scalar) list, device-resident",
        "value": round(value, 4), "unit": "GB/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 2), "higher_is_better": True, "scaling": "strong",
        "mode": args.mode,
        "vs_baseline": None, "dtype": "bf16", "data": "synthetic (random-init LLaMA-7B shapes, seeded seeds/scalars)",
        "config": {"workload": (f"{world}xMI355X: same 7B / K={args.k}, seeds sharded {len(ks) // world}/GPU, "
                                f"RCCL all-reduce of delta over xGMI") if seed_shard else
                   "1xMI355X: 7B-param bf16 buffer, K=4096 seeds" if world == 1 else
                   f"{world}xMI355X: 7B-param bf16 buffer, K=4096 seeds, element-sharded",
                   "params": total, "k": args.k, "k_nonzero": len(ks), "tensors": len(shapes),
                   "parallelism": f"seed-shard{world}" if seed_shard else f"element-shard{world}"},
        "roofline": {"bound": "hbm", "achieved": round(hbm_achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(hbm_achieved / HBM_PEAK_GBS, 6),
                     "traffic": (round(traffic * rank_params) if traffic else None),
                     "kernel": "fks_apply_bs_kernel" if len(ks) >= 20 else "fks_apply_kernel",
                     "launches": prof.n_apply,
                     "avg_launch_ms": round(prof.apply_ms / n_apply, 3),
                     "alg_bytes_per_launch": alg_bytes},
        "roofline_valu": valu,
        "jump_kernel_ms_per_step": round(prof.jump_ms / args.steps, 2),
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(dtype, args.cpu_budget)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
