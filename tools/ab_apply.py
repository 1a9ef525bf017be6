"""A/B timing of apply-kernel builds: python tools/ab_apply.py [lib.so ...] (no argument:
the in-tree libfks.so).  Each build runs in its own process (FKS_LIB_OVERRIDE) on the
same workload -- N bf16 params (default 2^28), K seeds (default 95 = 5 full passes),
wd AB_WD (default 0.01, 'none' for None) -- and prints the average apply/jump launch time per pass (AB_SEEDS seeds per
launch for the per-seed figure: 19, or 32 for the bf16 slice kernel).  AB_DT=f32: fp32 params
(FKS_CPU_FP32_FLAVOUR=libm: the libm flavour's kernel)."""
import json
import os
os.environ.setdefault("FKS_STREAM_MODE", "torch_cpu")  # the CPU-generator stream these measurements use
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import os, sys, json, torch
sys.path.insert(0, os.path.join(os.environ["ROOT"], "fate-llm_amd", "python"))
from fate_llm.algo.fedkseed import codec
n, k = int(os.environ["AB_N"]), int(os.environ["AB_K"])
dt = torch.float32 if os.environ.get("AB_DT") == "f32" else torch.bfloat16
buf = torch.empty(n, dtype=dt, device="cuda").normal_(0, 0.02)
wd = os.environ.get("AB_WD", "0.01")
specs = [codec.ParamSpec(buf, lr=1e-5, weight_decay=None if wd == "none" else float(wd))]
g = torch.Generator().manual_seed(1)
seeds = torch.randint(0, 2**32, (k,), generator=g).tolist()
vals = (torch.randn(k, generator=g, dtype=torch.float64) * 20).tolist()
codec.directional_step(specs, seeds[:19], vals[:19]); torch.cuda.synchronize()
best = None
for _ in range(3):
    with codec.profile() as p:
        codec.directional_step(specs, seeds, vals); torch.cuda.synchronize()
    r = p.apply_ms / max(p.n_apply, 1)
    best = r if best is None else min(best, r)
print(json.dumps({"lib": os.environ.get("FKS_LIB_OVERRIDE", "libfks.so"), "dtype": str(dt), "n": n, "k": k, "wd": wd,
                  "fp32_flavour": codec.cpu_fp32_flavour(),
                  "apply_ms_per_launch": round(best, 3),
                  "ps_per_seed_param": round(best * 1e9 / (n * int(os.environ.get("AB_SEEDS", "19"))), 3)}), flush=True)
'''


def main():
    libs = [("" if a == "intree" else a) for a in sys.argv[1:]] or [""]  # "intree": the in-tree libfks.so
    for lib in libs:
        env = dict(os.environ, ROOT=ROOT, AB_N=os.environ.get("AB_N", str(1 << 28)),
                   AB_K=os.environ.get("AB_K", "95"))
        if lib:
            env["FKS_LIB_OVERRIDE"] = os.path.abspath(lib)
        else:
            env.pop("FKS_LIB_OVERRIDE", None)
        r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
        out = [l for l in r.stdout.splitlines() if l.startswith("{")]
        print(out[-1] if out else json.dumps({"lib": lib, "error": r.stderr[-500:]}), flush=True)


if __name__ == "__main__":
    main()
