"""bench.py -- FedKSeed reconstruct throughput on MI355X (BASELINE.json metric).

One "step" = one reconstruct of the LLaMA-7B-shaped bf16 parameter buffer
(291 tensors, 6,738,415,616 params, random init N(0, 0.02^2)) from K = 4096
(seed, scalar) pairs -- the loop of ClientTrainer.train_once (fedkseed.py:136-141)
-- device-resident, through the drop-in fate_llm.algo.fedkseed codec (libfks.so).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--mode sequential|seed-shard]
                  [--scaling weak|strong] [--gather]

--gpus N > 1 without WORLD_SIZE in the environment re-launches this script under
torch.distributed.run with N ranks (one per GPU, 127.0.0.1) as a CHILD process, before
anything touches the GPU, and exits with its status; run under torch.distributed.run
directly, WORLD_SIZE must equal --gpus.

--mode sequential (default, bit-exact):
  --scaling strong (default): BASELINE's 8xMI355X config -- one 7B buffer, K=4096,
    split over the GPUs: the buffer is cut into N equal runs of MT19937 blocks and rank r
    reconstructs run r (element sharding: every element still sees every seed in order,
    so the union is bit-identical to N = 1 and no collective touches the data path);
    value = ONE buffer / the slowest rank's time; --gather adds the all-gather that
    leaves the whole buffer on every rank (N RCCL broadcasts of the shards), timed
    separately;
  --scaling weak (opt-in, reported under its own metric name): every rank reconstructs
    its own 7B buffer from the same K=4096 list -- the FedKSeed deployment, where each
    client GPU rebuilds its model from the (seed, sum) list the arbiter broadcasts
    (fedkseed.py:128-141); no collective; value = N buffers / the slowest rank's time.

Under torch.distributed.run (WORLD_SIZE in the environment) the ranks always form a
process group -- RCCL ("nccl") unless FKS_BENCH_SHARE_GPU=1 -- even at WORLD_SIZE=1, so
the timing's max-over-ranks, --gather and the seed-shard all-reduce run through the
collective library on a one-GPU box too (tests/test_gpu_rccl.py).

--mode seed-shard: the north star's C3 variant.  Rank r takes a contiguous 1/N of the
seeds, accumulates its f32 delta over the whole buffer (fks_delta_accumulate), one RCCL
all-reduce sums the deltas over xGMI, every rank applies p = a^K p_0 - delta.  Not the
reference's rounding (DESIGN.md §7 gives its measured deviation).

Rank 0 prints ONE JSON line: the metric, the binding roofline of the dominant kernel
(VALU issue -- the reconstruct draws K*N normals from ~26 GB of traffic), the north
star's HBM roofline next to it, and the reference CPU path timed on this host in the
same run (cpu_baseline).  --selftest runs the launcher / timing / reporting logic on CPU
ranks over gloo with a dummy step (no GPU, no codec): the CPU test of the N > 1 path.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "fate-llm_amd", "python"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

LLAMA7B_PARAMS = 6_738_415_616
HBM_PEAK_GBS = 8000.0  # MI355X spec, /opt/skills/guides/MI355X_MICROARCH.md
# VALU peak (MI355X_MICROARCH.md): 256 CUs x 4 SIMD-32 x 32 lanes x 2.4 GHz = 78.6 T lane-op/s
# (a wave64 instruction every 2 cycles per SIMD).  Measured on this chip
# (profiles/r02_ubench_issue3.log + _pmc.csv, GRBM cycles): only v_mul/v_add/v_fma/v_xor/
# v_add_u32 co-issue two waves; every instruction the slice kernel is made of (v_cvt_pk_bf16_f32,
# v_pk_*_f32, SDWA, v_bitop3, 64-bit shifts) issues alone at 4.43 cycles per wave-instruction
# even at 8 waves per SIMD, so the ceiling for this mix is 1024 x 64 x 2.4e9 / 4.43.
VALU_PEAK_TLANEOPS = 256 * 4 * 32 * 2.4e9 / 1e12
VALU_MIX_CYCLES = 4.43
VALU_MIX_CEILING_TLANEOPS = 1024 * 64 * 2.4e9 / VALU_MIX_CYCLES / 1e12
# per-launch counters of the bf16 slice kernel (fks_apply_bs_kernel), tools/summarize_pmc2.py: the
# weight-decay chain (wd != 0) and the zero-weight-decay chain (kModeUpdateWd0)
PMC_SUMMARIES = {"wd": "pmc_apply_r06_full.json", "wd0": "pmc_apply_r06_wd0.json"}
# the torch_rocm stream's kernel (fks_philox_vec_kernel, 32-seed launches) at wd 0.0
PMC_SUMMARY_PHX = "pmc_apply_r06_phx_wd0.json"


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


def pmc_summary_name(wd):
    return PMC_SUMMARIES["wd0" if wd == 0.0 else "wd"]


def lds_active_frac(pmc):
    """LDS-array cycles (bank conflicts included) per CU-cycle of the dominant kernel:
    rocprofv3 SQ_LDS_IDX_ACTIVE over 256 CUs x GRBM_GUI_ACTIVE / 8 (tools/summarize_pmc2.py);
    beside valu_active_frac, the slice kernel's other co-limit."""
    if pmc.get("lds_active_frac") is not None:
        return round(pmc["lds_active_frac"], 4)
    c, clk = pmc.get("per_launch") or {}, pmc.get("clock_cycles_per_launch")
    if c.get("SQ_LDS_IDX_ACTIVE") and clk:
        return round(c["SQ_LDS_IDX_ACTIVE"] / 256 / clk, 4)
    return None


def load_pmc_summary(wd=None, name=None):
    """Per-launch counters of the dominant kernel from the committed rocprofv3 --pmc
    passes (profiles/PMC_SUMMARIES, written by tools/summarize_pmc2.py)."""
    try:
        with open(os.path.join(ROOT, "profiles", name or pmc_summary_name(wd))) as f:
            return json.load(f)
    except OSError:
        return {}


def alt_stream_leg(codec, views, ks, kv, wd, total, build_id, steps):
    """The same 7B reconstruct drawn from the torch_rocm stream -- the z a reference client
    draws when its model sits on an MI355X (zo_utils.py:47: device=param.data.device), and
    the drop-in's DEFAULT stream on a GPU (codec "auto") -- timed over ``steps`` steps
    (median reported), with the VALU roofline of its kernel (fks_philox_vec_kernel)."""
    specs = [codec.ParamSpec(v, lr=1e-5, weight_decay=wd) for v in views]
    codec.directional_step(specs, ks[:32], kv[:32], stream_mode="torch_rocm")  # the tensor table
    torch.cuda.synchronize()
    times = []
    with codec.profile() as prof:
        for _ in range(steps):
            t0 = time.perf_counter()
            codec.directional_step(specs, ks, kv, stream_mode="torch_rocm")
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
    dt = sorted(times)[len(times) // 2]
    out = {"stream": "torch_rocm", "default_stream": True, "kernel": "fks_philox_vec_kernel", "weight_decay": wd,
           "steps": steps, "ms_per_step": round(dt * 1e3, 1), "ms_per_step_all": [round(t * 1e3, 1) for t in times],
           "value": round(total * 2 / dt / 1e9, 4), "unit": "GB/s",
           "ms_per_seed": round(dt * 1e3 / len(ks), 3), "launches": prof.n_apply,
           "kernel_ms_per_step": round(prof.apply_ms / steps, 1)}
    pmc = load_pmc_summary(name=PMC_SUMMARY_PHX)
    lane_ops = pmc.get("valu_lane_ops_per_seed_param")
    if lane_ops and pmc.get("build_id") == build_id and wd == 0.0:
        ach = total * len(ks) * steps * lane_ops / (prof.apply_ms / 1e3) / 1e12
        out["roofline"] = {"bound": "valu", "achieved": round(ach, 3), "peak": round(VALU_PEAK_TLANEOPS, 2),
                           "unit": "Tlane-op/s", "frac": round(ach / VALU_PEAK_TLANEOPS, 4),
                           "lane_ops_per_unit": round(lane_ops, 3), "build_id": build_id,
                           "counters": {k: pmc.get(k) for k in ("valu_active_frac", "clock_ghz")},
                           "unit_def": f"one seed*param update; lane-ops from profiles/{PMC_SUMMARY_PHX}"}
    else:
        out["roofline"] = None
        out["roofline_withheld"] = (f"profiles/{PMC_SUMMARY_PHX}: build {pmc.get('build_id')} / wd 0.0 only, "
                                    f"this run build {build_id} wd {wd}")
    return out


def hd_leg(codec, flat, specs, ks, kv, stream, host):
    """The north star's path from host memory to host memory: model_0 host -> device (the
    reference's .to(device), fedkseed.py:133, from pinned memory), the reconstruct, and the
    result back to the host (its state dict), timed end to end on one stream, once."""
    sync = torch.cuda.synchronize
    sync()
    t0 = time.perf_counter()
    flat.copy_(host, non_blocking=True)
    sync()
    t1 = time.perf_counter()
    codec.directional_step(specs, ks, kv, stream_mode=stream)
    sync()
    t2 = time.perf_counter()
    host.copy_(flat, non_blocking=True)
    sync()
    t3 = time.perf_counter()
    nbytes = flat.numel() * flat.element_size()
    return {"stream": stream, "h2d_ms": round((t1 - t0) * 1e3, 1), "reconstruct_ms": round((t2 - t1) * 1e3, 1),
            "d2h_ms": round((t3 - t2) * 1e3, 1), "total_ms": round((t3 - t0) * 1e3, 1),
            "value": round(nbytes / (t3 - t0) / 1e9, 4), "unit": "GB/s",
            "h2d_GBps": round(nbytes / (t1 - t0) / 1e9, 1), "d2h_GBps": round(nbytes / (t3 - t2) / 1e9, 1)}


# ------------------------------------------------------------------ CPU baseline
_CPU_CHILD = r'''
import os, sys, time, json, torch
sys.path.insert(0, os.environ["FKS_ROOT"])
torch.set_num_threads(1)
from oracle import torch_replica as R
from bench import synthetic_seeds
n, first, step, budget = (int(os.environ[k]) for k in ("N", "FIRST", "STEP", "BUDGET"))
wd = None if os.environ["WD"] == "none" else float(os.environ["WD"])
s_, g_ = synthetic_seeds(4096)
seeds = [(s, g) for s, g in zip(s_, g_) if g != 0.0]
p = [torch.randn(n, generator=torch.Generator().manual_seed(0)).mul_(0.02).to(torch.bfloat16)]
done, t0 = 0, time.perf_counter()
for i in range(first, len(seeds), step):
    if time.perf_counter() - t0 > budget:
        break
    s, g = seeds[i]
    R.reconstruct(p, [s], [g], 1e-5, wd)
    done += 1
print(json.dumps({"done": done, "s": time.perf_counter() - t0}))
'''


def usable_cpus():
    """CPUs this process may actually run on: its affinity mask, capped by a cgroup CPU
    quota (v2 cpu.max or v1 cfs_quota_us) -- on a GPU box the job's CPU share, which can
    be far below os.cpu_count() (the whole host)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    if quota is not None:
        n = min(n, max(1, int(quota)))
    return max(1, n), quota


def cpu_baseline(budget_s, wd):
    """The reference's CPU path (torch.manual_seed + torch.normal + the update expression
    of zo_utils.py:47-52, re-typed in oracle/torch_replica.py) on bounded samples of the
    same workload, scaled linearly to the 7B buffer x the 4055 non-zero seeds of K=4096:
      * one process at torch's default thread count, at two sizes (2^22 and 2^24 bf16
        params) to check linearity in N;
      * the all-core variant -- reported as `value`: one single-thread process per CPU this
        job may use (affinity mask and cgroup quota, usable_cpus) over disjoint seeds
        (torch.normal holds the generator mutex, so one process draws on one core), the
        fairest CPU upper bound.  `cores` = processes run; `nproc` = the host's CPU count;
        when the job's share is smaller than the host, `all_host_cores_extrapolated`
        scales the measured per-process rate to every host core (not measured)."""
    from oracle import torch_replica as R
    threads = torch.get_num_threads()
    seeds, scalars = synthetic_seeds(4096)
    keep = [(s, g) for s, g in zip(seeds, scalars) if g != 0.0]
    t7b_seeds = len(keep)

    def one_process(n, budget):
        p = [torch.randn(n, generator=torch.Generator().manual_seed(0)).mul_(0.02).to(torch.bfloat16)]
        done, t0 = 0, time.perf_counter()
        while done < len(keep) and time.perf_counter() - t0 < budget:
            s, g = keep[done]
            R.reconstruct(p, [s], [g], 1e-5, wd)
            done += 1
        dt = time.perf_counter() - t0
        return dt / (n * done) * 1e9, done, dt

    ns_small, d_small, _ = one_process(1 << 22, budget_s * 0.2)
    ns_big, d_big, dt_big = one_process(1 << 24, budget_s * 0.3)
    procs, quota = usable_cpus()
    n_all = 1 << 22
    env = dict(os.environ, FKS_ROOT=ROOT, N=str(n_all), WD="none" if wd is None else repr(wd), STEP=str(procs),
               BUDGET=str(int(max(2, budget_s * 0.5))), OMP_NUM_THREADS="1")
    kids = [subprocess.Popen([sys.executable, "-c", _CPU_CHILD], env=dict(env, FIRST=str(i)), stdout=subprocess.PIPE,
                             text=True) for i in range(procs)]
    outs = [json.loads(k.communicate()[0].strip().splitlines()[-1]) for k in kids]
    wall = max(o["s"] for o in outs)
    done_all = sum(o["done"] for o in outs)
    ns_all = wall / (n_all * done_all) * 1e9  # aggregate: ns per seed*param over all processes
    t7b = LLAMA7B_PARAMS * t7b_seeds * ns_all * 1e-9
    t7b_one = LLAMA7B_PARAMS * t7b_seeds * ns_big * 1e-9
    nproc = os.cpu_count() or procs
    value = LLAMA7B_PARAMS * 2 / t7b / 1e9
    out = {
        "value": value, "unit": "GB/s", "cores": procs, "kind": "port",
        "sample": (f"torch CPU replica of zo_utils.directional_derivative_step (oracle/torch_replica.py, "
                   f"weight_decay {wd}), "
                   f"{procs} single-thread processes (one per usable CPU) over disjoint seeds: {done_all} seeds x "
                   f"{n_all} bf16 params in {wall:.1f} s = {ns_all:.3f} ns per seed*param aggregate, scaled linearly "
                   f"to 6.74e9 params x {t7b_seeds} non-zero seeds ({t7b / 3600:.1f} h)"),
        "single_process": {"threads": threads, "ns_per_seed_param_2^22": round(ns_small, 3),
                           "ns_per_seed_param_2^24": round(ns_big, 3), "seeds_2^22": d_small, "seeds_2^24": d_big,
                           "seconds_2^24": round(dt_big, 1), "value_GBps": LLAMA7B_PARAMS * 2 / t7b_one / 1e9,
                           "note": "torch.normal single-threaded under the generator mutex; elementwise ops on "
                                   f"{threads} threads; the two sizes check linearity in N"},
        "nproc": nproc,
        "usable_cpus": {"affinity": len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None,
                        "cgroup_quota_cpus": quota},
    }
    if procs < nproc:
        out["all_host_cores_extrapolated"] = {
            "value": value * nproc / procs, "cores": nproc,
            "note": (f"this job may use {procs} of the host's {nproc} CPUs (affinity / cgroup quota); the measured "
                     "per-process rate x every host core, assuming perfect scaling -- an upper bound, not measured")}
    return out


# ------------------------------------------------------------------ launcher
def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def relaunch(n: int) -> int:
    """Run this script under torch.distributed.run with n ranks, as a child process
    (nothing here has touched the GPU), and return its exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    return subprocess.call(cmd, env=env)


def timed_steps(step, args, world, sync):
    for _ in range(args.warmup):
        step()
    sync()
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    sync()
    if world > 1:
        dist.barrier()
    sync()
    return time.perf_counter() - t0


def max_over_ranks(dt, world, device):
    if not (dist.is_available() and dist.is_initialized()):
        return dt
    t = torch.tensor([dt], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def selftest(args, world, rank):
    """CPU ranks over gloo: the launcher, barrier + max-over-ranks timing and the JSON
    line, with a dummy CPU step in place of the codec."""
    if world > 1:
        dist.init_process_group("gloo")
        world = dist.get_world_size()
    x = torch.ones(1 << 16)

    def step():
        x.mul_(1.0000001)

    dt = max_over_ranks(timed_steps(step, args, world, lambda: None), world, torch.device("cpu"))
    if rank == 0:
        print(json.dumps({"metric": "selftest", "value": args.steps / dt, "unit": "steps/s", "n_gpus": world,
                          "steps": args.steps, "warmup": args.warmup, "selftest": True,
                          "pid": os.getpid()}), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


# ------------------------------------------------------------------ GPU bench
def run(args, world, rank, local):
    # FKS_BENCH_SHARE_GPU=1 (rehearsal on a one-GPU box, tests/test_gpu_bench_ranks.py):
    # the ranks share the visible GPUs and talk over gloo; the measured path is RCCL, one
    # GPU per rank
    share = os.environ.get("FKS_BENCH_SHARE_GPU") == "1"
    if share:
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    distributed = "WORLD_SIZE" in os.environ  # launched by torch.distributed.run (any world size)
    if distributed:
        if share:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
        world = dist.get_world_size()  # what RCCL reports

    from fate_llm.algo.fedkseed import codec, zo_utils

    # the headline draws torch's CPU-generator stream (the oracle-pinned one: a reference
    # client training on the CPU, the tutorial's configuration); the drop-in's default
    # "auto" would draw the torch_rocm stream on a GPU, which alt_stream times beside it
    codec.set_stream_mode(args.stream)
    rocm = args.stream == "torch_rocm"
    dtype = torch.bfloat16
    shapes = [(args.params,)] if args.params else llama7b_shapes()
    total = sum(numel(s) for s in shapes)
    flat = torch.empty(total, dtype=dtype, device=dev)
    flat.normal_(0.0, 0.02, generator=torch.Generator(device=dev).manual_seed(0))
    views, off = [], 0
    for s in shapes:
        views.append(flat[off:off + numel(s)].view(s))
        off += numel(s)
    wd = args.wd
    specs = [codec.ParamSpec(v, lr=1e-5, weight_decay=wd) for v in views]
    seeds, scalars = synthetic_seeds(args.k)
    keep = [(s, g) for s, g in zip(seeds, scalars) if g != 0.0]
    ks, kv = [s for s, _ in keep], [g for _, g in keep]
    seed_shard = args.mode == "seed-shard"
    if seed_shard:
        groups = [{"params": views, "lr": 1e-5, "weight_decay": wd}]
        delta = torch.empty(total, dtype=torch.float32, device=dev)
    weak = not seed_shard and args.scaling == "weak"
    nshards = 1 if weak else world
    shard_words = [codec.shard_range(specs, r, nshards) for r in range(nshards)] if nshards > 1 else [(0, total)]

    def step():
        if seed_shard:
            zo_utils.reconstruct_seed_sharded_(groups, ks, kv, lr=1e-5, weight_decay=wd, delta=delta)
        else:
            codec.directional_step(specs, ks, kv, shard=rank % nshards, nshards=nshards)

    sync = torch.cuda.synchronize
    with codec.profile() as prof:
        dt = timed_steps(step, args, world, sync)
    dt = max_over_ranks(dt, world, dev)
    gather_ms = None
    if args.gather and distributed and not seed_shard and not weak:
        # every rank ends with the whole buffer: one broadcast of each element shard (the
        # bench's buffer is one flat tensor and all its tensors are fast segments, so a
        # shard's stream words are its element range)
        sync()
        dist.barrier()
        t0 = time.perf_counter()
        for r, (lo, hi) in enumerate(shard_words):
            dist.broadcast(flat[lo:hi], src=r)
        sync()
        gather_ms = max_over_ranks(time.perf_counter() - t0, world, dev) * 1e3

    alt = None
    if world == 1 and not seed_shard and args.alt_wd != wd:
        # the same reconstruct at the other weight decay (plan built by a 32-seed call first)
        alt_specs = [codec.ParamSpec(v, lr=1e-5, weight_decay=args.alt_wd) for v in views]
        codec.directional_step(alt_specs, ks[:32], kv[:32])
        sync()
        t0 = time.perf_counter()
        codec.directional_step(alt_specs, ks, kv)
        sync()
        alt_s = time.perf_counter() - t0
        alt = {"weight_decay": args.alt_wd, "ms_per_step": round(alt_s * 1e3, 2),
               "value": round(total * 2 / alt_s / 1e9, 4), "steps": 1}

    from fate_llm.algo.fedkseed import _native
    build_id = _native.build_id()
    alt_stream = None
    if world == 1 and not seed_shard and args.alt_stream == "torch_rocm" and not rocm:
        alt_stream = alt_stream_leg(codec, views, ks, kv, wd, total, build_id, max(1, args.alt_stream_steps))

    hd = None
    if world == 1 and not seed_shard and args.hd:
        # PCIe-inclusive rate for both streams (reported beside value, never as it)
        host = torch.empty(total, dtype=dtype, pin_memory=True)
        host.copy_(flat)
        hd = {s: hd_leg(codec, flat, specs, ks, kv, s, host) for s in ("torch_cpu", "torch_rocm")}
        del host

    ms_per_step = dt / args.steps * 1e3
    buf_bytes = total * 2 * (world if weak else 1)  # weak: one buffer per rank
    value = buf_bytes / (dt / args.steps) / 1e9

    # ---- rooflines of the dominant kernel, this rank: the bf16 slice kernel
    # (fks_apply_bs_kernel, 64 seeds per launch) for every reconstruct of >= 20 seeds
    n_steps_prof = args.steps + args.warmup
    rank_params = total if seed_shard else (shard_words[rank % nshards][1] - shard_words[rank % nshards][0])
    n_apply = max(prof.n_apply, 1)
    avg_apply_s = prof.apply_ms / n_apply / 1e3
    rank_seeds = len(ks) * (rank + 1) // world - len(ks) * rank // world if seed_shard else len(ks)
    seeds_per_launch = rank_seeds * n_steps_prof / n_apply
    units = rank_params * seeds_per_launch  # seed*param updates per launch
    # the dominant kernel's counters: the slice kernel (torch_cpu), or the torch_rocm stream's
    # fks_philox_vec_kernel (profiled at wd 0.0 only)
    pmc = (load_pmc_summary(name=PMC_SUMMARY_PHX) if wd == 0.0 else {}) if rocm else load_pmc_summary(wd)
    lane_ops = pmc.get("valu_lane_ops_per_seed_param")
    valu = None
    withheld = None
    if lane_ops and pmc.get("build_id") != build_id:
        # the committed counters were profiled from other device code: their lane-ops per
        # unit do not describe the kernels timed here
        withheld = (f"profiles/{pmc_summary_name(wd)} was profiled from libfks.so build {pmc.get('build_id')}, "
                    f"this run loaded build {build_id}: VALU roofline withheld (re-run tools/gpu_pmc2.sh)")
        lane_ops = None
    if lane_ops and not seed_shard:
        ach = units * lane_ops / avg_apply_s / 1e12
        valu = {"bound": "valu", "achieved": round(ach, 3), "peak": round(VALU_PEAK_TLANEOPS, 2), "unit": "Tlane-op/s",
                "frac": round(ach / VALU_PEAK_TLANEOPS, 4),
                "mix_ceiling": round(VALU_MIX_CEILING_TLANEOPS, 2),
                "frac_of_mix_ceiling": round(ach / VALU_MIX_CEILING_TLANEOPS, 4),
                # HBM bytes per launch from the PMC passes (FETCH_SIZE + WRITE_SIZE, corrected as
                # MI355X_MICROARCH.md prescribes; tools/summarize_pmc2.py)
                "traffic": (round(pmc["hbm_bytes_per_param_per_launch"] * rank_params)
                            if pmc.get("hbm_bytes_per_param_per_launch") else None),
                "traffic_unit": "HBM bytes per launch",
                "kernel": "fks_philox_vec_kernel" if rocm else "fks_apply_bs_kernel", "launches": prof.n_apply,
                "avg_launch_ms": round(prof.apply_ms / n_apply, 3),
                "units_per_launch": units, "lane_ops_per_unit": round(lane_ops, 3),
                "build_id": build_id,
                "counters": dict({k: pmc.get(k) for k in ("valu_active_frac", "valu_dual_issue_frac", "wait_any_frac",
                                                          "lds_bank_conflict_frac", "clock_ghz")},
                                 lds_active_frac=lds_active_frac(pmc)),
                "unit_def": ("one seed*param update (z draw + update chain); lane-ops = rocprofv3 SQ_INSTS_VALU x 64 "
                             f"per seed*param (profiles/{pmc_summary_name(wd)}); peak = 256 CU x 4 SIMD-32 x 32 lanes x 2.4 GHz "
                             "(MI355X_MICROARCH.md); mix_ceiling = the same chip issuing this kernel's "
                             f"single-issue instruction mix at the measured {VALU_MIX_CYCLES} cycles per "
                             "wave-instruction (profiles/r02_ubench_issue3.log)")}
    # the north star's roof: algorithmic HBM bytes of the WHOLE reconstruct (read + write the
    # buffer once, SURVEY.md §8(d): 2 N elt) over the reconstruct time; the per-pass figure
    # (each 64-seed launch streams its shard once) is reported beside it, named as such.
    # Per GPU, against one GPU's peak: a strong element shard reads + writes its own run
    # once; a weak rank its whole buffer; a seed-shard rank accumulates (and applies) over
    # the whole buffer too
    elt = 4 if seed_shard else 2
    alg_bytes_step = 2 * total * 2 * (world if weak else 1)
    rank_alg_bytes = 2 * rank_params * 2
    hbm_ach = rank_alg_bytes / (dt / args.steps) / 1e9
    traffic = pmc.get("hbm_bytes_per_param_per_launch")
    hbm = {"bound": "hbm", "achieved": round(hbm_ach, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(hbm_ach / HBM_PEAK_GBS, 7),
           "traffic": (round(traffic * rank_params) if traffic and not seed_shard and not withheld else None),
           "alg_bytes_per_step": alg_bytes_step, "alg_bytes_per_step_this_gpu": rank_alg_bytes,
           "per_pass": {"alg_bytes_per_launch": 2 * rank_params * elt,
                        "achieved_GBps": round(2 * rank_params * elt / avg_apply_s / 1e9, 2),
                        "note": f"one launch reads + writes its shard once ({round(seeds_per_launch)} seeds); a reconstruct is "
                                f"{round(n_apply / n_steps_prof)} such passes"}}
    metric = "GB/s param buffer reconstructed from (seed,scalar) list, device-resident"
    if weak and world > 1:
        metric += " [weak scaling: one buffer per GPU]"
    out = {
        "metric": metric,
        "value": round(value, 4), "unit": "GB/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 2), "higher_is_better": True, "scaling": "weak" if weak else "strong",
        "mode": args.mode, "vs_baseline": None, "dtype": "bf16",
        "data": "synthetic (random-init LLaMA-7B shapes, seeded seeds/scalars)",
        "config": {"workload": (f"{world}xMI355X: same 7B / K={args.k}, seeds sharded {len(ks) // world}/GPU, "
                                f"RCCL all-reduce of delta over xGMI") if seed_shard else
                   "1xMI355X: 7B-param bf16 buffer, K=4096 seeds" if world == 1 else
                   (f"{world}xMI355X: one 7B-param bf16 buffer per GPU, K=4096 seeds (each GPU one client's "
                    "reconstruct, no collective)") if weak else
                   f"{world}xMI355X: 7B-param bf16 buffer, K=4096 seeds, element-sharded (bit-exact, no collective)",
                   "params": total, "k": args.k, "k_nonzero": len(ks), "tensors": len(shapes),
                   "lr": 1e-5, "weight_decay": wd, "stream": args.stream,
                   "stream_note": ("value draws torch's CPU-generator stream (the oracle-pinned one; a reference "
                                   "client training on the CPU, FKS_STREAM_MODE=torch_cpu); the drop-in's default "
                                   "on a GPU ('auto') draws torch_rocm, timed as alt_stream") if not rocm else
                                  ("value draws torch's HIP-device generator stream (torch_rocm: the drop-in's "
                                   "default on a GPU, a reference client whose model sits on the GPU)"),
                   "parallelism": (f"seed-shard{world}" if seed_shard else
                                   f"client-per-gpu{world}" if weak else f"element-shard{world}")},
        "roofline": valu if valu else hbm,
        "roofline_hbm": hbm,
        "build_id": build_id,
        "jump_kernel_ms_per_step": round(prof.jump_ms / n_steps_prof, 2),
    }
    if distributed:
        out["backend"] = dist.get_backend()
        if share:
            out["shared_gpu"] = True  # a rehearsal, not a measurement
    if withheld:
        out["valu_roofline_withheld"] = withheld
    if gather_ms is not None:
        out["gather_ms"] = round(gather_ms, 1)
    if alt is not None:
        out["alt_weight_decay"] = alt
    if alt_stream is not None:
        out["alt_stream"] = alt_stream
    if hd is not None:
        out["hd_inclusive"] = hd
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args.cpu_budget, wd)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if distributed:
        dist.destroy_process_group()
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--k", type=int, default=4096)
    ap.add_argument("--params", type=int, default=0, help="override: flat buffer of this many params (dev only)")
    ap.add_argument("--wd", type=lambda v: None if v == "none" else float(v), default=0.0,
                    help="weight decay of every tensor (default 0.0: the HF TrainingArguments default the "
                         "reference's ClientTrainer passes, fedkseed.py:140; 'none' = zo_utils.py:52)")
    ap.add_argument("--alt-wd", type=lambda v: None if v == "none" else float(v), default=0.01,
                    help="N = 1: one more timed reconstruct at this weight decay, reported beside value")
    ap.add_argument("--alt-stream", choices=("torch_rocm", "none"), default="torch_rocm",
                    help="N = 1: one more timed reconstruct drawing the torch_rocm stream (a reference client "
                         "whose model sits on the GPU), with its kernel's VALU roofline")
    ap.add_argument("--alt-stream-steps", type=int, default=3, help="timed steps of the torch_rocm leg (median)")
    ap.add_argument("--stream", choices=("torch_cpu", "torch_rocm"), default="torch_cpu",
                    help="the z stream `value` draws (default torch_cpu, the oracle-pinned stream; torch_rocm is the "
                         "drop-in's default on a GPU, timed beside it as alt_stream)")
    ap.add_argument("--no-hd", dest="hd", action="store_false",
                    help="N = 1: skip the host -> device -> host legs (H2D + reconstruct + D2H, both streams)")
    ap.add_argument("--cpu-budget", type=float, default=24.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--mode", choices=("sequential", "seed-shard"), default="sequential")
    ap.add_argument("--scaling", choices=("weak", "strong"), default="strong",
                    help="sequential mode, N > 1: strong = one buffer element-sharded over the GPUs (default, "
                         "BASELINE's 8xMI355X config); weak = a 7B buffer per GPU (opt-in, own metric name)")
    ap.add_argument("--gather", action="store_true", help="N > 1, strong: all-gather the shards afterwards")
    ap.add_argument("--selftest", action="store_true", help="CPU/gloo check of the launcher and timing logic")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return relaunch(args.gpus)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if args.selftest:
        return selftest(args, world, rank)
    return run(args, world, rank, local)


if __name__ == "__main__":
    sys.exit(main())
