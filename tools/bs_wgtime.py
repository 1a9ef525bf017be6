"""Diagnostic: how unevenly the slice kernel's workgroups finish a pass (the tail a pass
leaves idle).  Needs the FKS_BS_WGTIME variant build (make -C fate-llm_amd variant
NAME=wgtime DEFS=-DFKS_BS_WGTIME=1), which stamps each workgroup's start and each wave's
end with s_memrealtime (100 MHz).  Runs 64-seed passes over the 7B bf16 layout (or
--params P flat) and prints, per pass, the spread of workgroup end times relative to the
pass: the idle CU-time fraction = mean over workgroups of (last end - own end) / span.
python tools/bs_wgtime.py [--passes 3] [--params 0] [--nshards 1]"""
import argparse
import ctypes
import json
import os
os.environ.setdefault("FKS_STREAM_MODE", "torch_cpu")  # the CPU-generator stream these measurements use
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "fate-llm_amd", "ab", "libfks_wgtime.so")
os.environ["FKS_LIB_OVERRIDE"] = LIB
sys.path.insert(0, os.path.join(ROOT, "fate-llm_amd", "python"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--passes", type=int, default=3)
    ap.add_argument("--params", type=int, default=0, help="0: the 7B layout")
    ap.add_argument("--nshards", type=int, default=1, help="time rank 0's shard of N")
    args = ap.parse_args()
    from fate_llm.algo.fedkseed import codec
    dev = torch.device("cuda", 0)
    shapes = bench.llama7b_shapes() if args.params == 0 else [(args.params,)]
    total = sum(bench.numel(s) for s in shapes)
    flat = torch.empty(total, dtype=torch.bfloat16, device=dev).normal_(0.0, 0.02)
    specs, off = [], 0
    for s in shapes:
        specs.append(codec.ParamSpec(flat[off:off + bench.numel(s)].view(s), lr=1e-5, weight_decay=0.0))
        off += bench.numel(s)
    seeds, vals = bench.synthetic_seeds(4096)
    lib = ctypes.CDLL(LIB)
    lib.fks_debug_bs_wgtime.argtypes = [ctypes.c_void_p, ctypes.c_int]
    nblk = 256
    buf = np.zeros((nblk, 16), dtype=np.uint64)
    codec.directional_step(specs, seeds[:64], vals[:64], shard=0, nshards=args.nshards)  # plan + warm-up
    torch.cuda.synchronize()
    for p in range(args.passes):
        s0 = 64 * (p + 1)
        codec.directional_step(specs, seeds[s0:s0 + 64], vals[s0:s0 + 64], shard=0, nshards=args.nshards)
        torch.cuda.synchronize()
        assert lib.fks_debug_bs_wgtime(buf.ctypes.data, nblk) == 0
        start = buf[:, 0].astype(np.int64)
        end = buf[:, 1:13].max(axis=1).astype(np.int64)
        t0, t1 = start.min(), end.max()
        span = (t1 - t0) / 100.0  # us
        idle = float(np.mean(t1 - end)) / 100.0
        print(json.dumps({"pass": p, "nshards": args.nshards, "span_us": round(span, 1),
                          "start_spread_us": round((start.max() - t0) / 100.0, 1),
                          "end_min_us": round((end.min() - t0) / 100.0, 1),
                          "end_p50_us": round((np.percentile(end, 50) - t0) / 100.0, 1),
                          "end_p90_us": round((np.percentile(end, 90) - t0) / 100.0, 1),
                          "mean_idle_us": round(idle, 1), "idle_frac": round(idle / span, 4)}), flush=True)


if __name__ == "__main__":
    main()
