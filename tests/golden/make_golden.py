"""Generate the golden fixtures under tests/golden/ by IMPORTING the reference.

Run only in the build container, where /root/reference exists:
    PYTHONDONTWRITEBYTECODE=1 python3 tests/golden/make_golden.py

What it imports (read-only, from /root/reference/python):
    fate_llm.algo.fedkseed.zo_utils       (directional_derivative_step, probability_from_amps, ...)
    fate_llm.algo.fedkseed.optimizer      (ZerothOrderOptimizer, KSeedZerothOrderOptimizer)
    fate_llm.algo.fedkseed.pytorch_utils  (get_optimizer_parameters_grouped_with_decay)
    fate_llm.algo.fedkseed.fedkseed       (Trainer; needs a one-symbol stub for fate.arch.context)

The fixtures are DATA only (inputs and the reference's outputs), written as .npz
(no pickles) and .json.  Nothing here travels to the GPU box in runnable form: the
tests read the fixtures, never this script, and never /root/reference.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import types

import numpy as np
import torch

REF = "/root/reference/python"
OUT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REF)

# fedkseed.py:7 imports fate.arch.context.Context for an annotation only.
_fate = types.ModuleType("fate")
_arch = types.ModuleType("fate.arch")
_ctxm = types.ModuleType("fate.arch.context")
_ctxm.Context = object
_fate.arch = _arch
_arch.context = _ctxm
sys.modules.setdefault("fate", _fate)
sys.modules.setdefault("fate.arch", _arch)
sys.modules.setdefault("fate.arch.context", _ctxm)

from fate_llm.algo.fedkseed import zo_utils  # noqa: E402
from fate_llm.algo.fedkseed import optimizer as ref_opt  # noqa: E402
from fate_llm.algo.fedkseed import pytorch_utils  # noqa: E402

try:  # trainer.py imports HF Trainer classes; only Trainer (server) is used here
    from fate_llm.algo.fedkseed import fedkseed as ref_fks  # noqa: E402
except Exception as e:  # pragma: no cover
    ref_fks = None
    print("fedkseed import failed:", e)

DT = {"float32": torch.float32, "bfloat16": torch.bfloat16, "float16": torch.float16, "float64": torch.float64}


def bits(t: torch.Tensor) -> np.ndarray:
    t = t.detach().contiguous().cpu()
    if t.dtype in (torch.bfloat16, torch.float16):
        return t.view(torch.int16).numpy().view(np.uint16).copy()
    return t.numpy().copy()


def meta():
    return {
        "torch": torch.__version__,
        "cpu_capability": torch.backends.cpu.get_cpu_capability(),
        "reference": "FATE-LLM 2.2.0 (python/setup.py:59)",
        "generator": "tests/golden/make_golden.py",
    }


# --------------------------------------------------------------------------- MT19937
def gen_mt():
    seeds = np.array([0, 1, 42, 12345, 2**31, 2**32 - 1, 2**32 + 5, 67280421310721], dtype=np.uint64)
    draws = np.array([0, 1, 623, 624, 625, 1000, 5000, 20000], dtype=np.int64)
    states, lefts, nexts, r64 = [], [], [], []
    for s in seeds:
        for n in draws:
            torch.manual_seed(int(s))
            if n:
                torch.empty(int(n), dtype=torch.float32).uniform_()  # one 32-bit draw per element
            st = torch.get_rng_state().numpy().tobytes()
            lefts.append(np.frombuffer(st[8:12], np.int32)[0])
            nexts.append(np.frombuffer(st[16:24], np.uint64)[0])
            states.append(np.frombuffer(st[24:24 + 624 * 8], np.uint64).astype(np.uint32))
        torch.manual_seed(int(s))
        r64.append(torch.empty(8, dtype=torch.int64).random_().numpy())  # random64 % 2**63
    np.savez(os.path.join(OUT, "mt.npz"), seeds=seeds, draws=draws, states=np.stack(states),
             left=np.array(lefts, np.int32), next=np.array(nexts, np.int64), random64_mod63=np.stack(r64))


# --------------------------------------------------------------------------- z streams
STREAM_SHAPES = [1, 3, 5, 15, 16, 17, 31, 37, 64, 100, 624, 625, 1000, 4103, 2, 7]


def gen_streams():
    out = {"shapes": np.array(STREAM_SHAPES, np.int64), "seeds": np.array([0, 7, 2**32 - 1, 3141592653], np.uint64)}
    for name, dt in DT.items():
        for s in out["seeds"]:
            torch.manual_seed(int(s))
            zs = [bits(torch.normal(mean=0, std=1, size=(n,), dtype=dt)) for n in STREAM_SHAPES]
            out[f"seq_{name}_{int(s)}"] = np.concatenate(zs)
    # long streams (statistics + every bf16 (a, b) table pair)
    torch.manual_seed(2024)
    out["long_float32"] = bits(torch.normal(mean=0, std=1, size=(1 << 18,), dtype=torch.float32))
    torch.manual_seed(2024)
    out["long_bfloat16"] = bits(torch.normal(mean=0, std=1, size=(1 << 20,), dtype=torch.bfloat16))
    torch.manual_seed(2024)
    out["long_float16"] = bits(torch.normal(mean=0, std=1, size=(1 << 18,), dtype=torch.float16))
    # libm flavour of the fp32 kernel (ATEN_CPU_CAPABILITY=default), in a child process
    code = ("import torch,numpy as np,sys;torch.manual_seed(2024);"
            "a=torch.normal(mean=0,std=1,size=(1<<16,),dtype=torch.float32).numpy();"
            "sys.stdout.buffer.write(torch.backends.cpu.get_cpu_capability().encode()+b'\\n'+a.tobytes())")
    env = dict(os.environ, ATEN_CPU_CAPABILITY="default")
    raw = subprocess.run([sys.executable, "-c", code], env=env, check=True, capture_output=True).stdout
    cap, data = raw.split(b"\n", 1)
    assert cap == b"DEFAULT", cap
    out["long_float32_default_capability"] = np.frombuffer(data, np.float32).copy()
    np.savez(os.path.join(OUT, "normal_streams.npz"), **out)


# --------------------------------------------------------------------------- models
class TinyLM(torch.nn.Module):
    """GPT-2-shaped miniature: embeddings, LayerNorms, biased linears (both groups non-empty)."""

    def __init__(self, d=48, v=100, ragged=False):
        super().__init__()
        self.wte = torch.nn.Embedding(v, d)
        self.ln_1 = torch.nn.LayerNorm(d)
        self.attn = torch.nn.Linear(d, 3 * d)
        self.proj = torch.nn.Linear(3 * d, d, bias=False)
        self.ln_f = torch.nn.LayerNorm(d)
        if ragged:
            self.odd = torch.nn.Linear(d, 7)        # weight 336 (%16=0), bias 7 (<16)
            self.odd2 = torch.nn.Linear(5, 37)      # weight 185 (ragged), bias 37 (ragged)
            self.tiny = torch.nn.Parameter(torch.zeros(3))


def build_model(dtype, ragged=False, seed=0):
    torch.manual_seed(seed)
    m = TinyLM(ragged=ragged)
    g = torch.Generator().manual_seed(seed + 1)
    with torch.no_grad():
        for p in m.parameters():
            p.copy_(torch.randn(p.shape, generator=g) * 0.02)
    return m.to(DT[dtype])


def group_layout(model, groups):
    name_of = {id(p): n for n, p in model.named_parameters()}
    return [[name_of[id(p)] for p in g["params"]] for g in groups]


def snapshot(model):
    return {n: bits(p) for n, p in model.named_parameters()}


def gen_reconstruct():
    cases = {}

    def seeds_scalars(k, seed, zeros=0.01, extra=None):
        gg = torch.Generator().manual_seed(seed)
        sd = torch.randint(0, 2**32, (k,), generator=gg, dtype=torch.int64).numpy().astype(np.uint64)
        sc = (torch.randn(k, generator=gg, dtype=torch.float64) * 20.0).numpy()
        nz = max(1, int(k * zeros))
        sc[torch.randperm(k, generator=gg)[:nz].numpy()] = 0.0
        if extra:
            for i, v in extra.items():
                sc[i] = v
        return sd, sc

    specs = [
        # name, dtype, ragged, K, lr, wd (explicit, train_once style), sticky(local-step style), extra scalars
        ("f32_wd", "float32", False, 64, 1e-5, 0.01, False, None),
        ("f32_nowd", "float32", False, 64, 1e-5, 0.0, False, None),
        ("bf16_wd", "bfloat16", False, 64, 1e-3, 0.01, False, None),
        ("bf16_nowd", "bfloat16", False, 64, 1e-5, 0.0, False, None),
        ("f16_wd", "float16", False, 32, 1e-3, 0.01, False, None),
        ("f32_ragged", "float32", True, 24, 1e-4, 0.01, False, None),
        ("bf16_ragged", "bfloat16", True, 24, 1e-3, 0.01, False, None),
        ("f32_sticky", "float32", False, 16, None, None, True, None),
        ("bf16_sticky", "bfloat16", False, 16, None, None, True, None),
        ("f32_edge", "float32", False, 8, 1e-5, 0.01, False, {1: -0.0, 2: 1e40, 3: 1e-45, 5: -3.5e38}),
        ("bf16_nan", "bfloat16", False, 6, 1e-3, 0.01, False, {2: float("nan")}),
        ("f32_k4096", "float32", False, 4096, 1e-5, 0.01, False, None),
        ("bf16_k4096", "bfloat16", False, 4096, 1e-5, 0.01, False, None),
    ]
    for name, dtype, ragged, k, lr, wd, sticky, extra in specs:
        model = build_model(dtype, ragged=ragged, seed=len(cases))
        if name.endswith("k4096"):  # keep the reference run short: 2 small tensors only
            model = torch.nn.Module()
            model.w = torch.nn.Parameter((torch.randn(256, 3, generator=torch.Generator().manual_seed(9)) * 0.02).to(DT[dtype]))
            model.b = torch.nn.Parameter((torch.randn(40, generator=torch.Generator().manual_seed(10)) * 0.02).to(DT[dtype]))
        group_wd = 0.01 if sticky else (wd if wd is not None else 0.0)
        groups = pytorch_utils.get_optimizer_parameters_grouped_with_decay(model, group_wd)
        for g_ in groups:
            g_["lr"] = 3e-4 if sticky else 0.0
        init = snapshot(model)
        sd, sc = seeds_scalars(k, 100 + len(cases), extra=extra)
        for s, g in zip(sd.tolist(), sc.tolist()):
            if g != 0.0:  # fedkseed.py:137
                if sticky:
                    zo_utils.directional_derivative_step(groups, int(s), g)
                else:
                    zo_utils.directional_derivative_step(groups, int(s), g, lr=lr, weight_decay=wd)
        final = snapshot(model)
        layout = group_layout(model, groups)
        case = {"dtype": dtype, "k": k, "lr": lr, "wd": wd, "sticky": sticky,
                "groups": layout, "group_wd": [g_["weight_decay"] for g_ in groups],
                "group_lr": [g_["lr"] for g_ in groups],
                "shapes": {n: list(p.shape) for n, p in model.named_parameters()}}
        arrays = {"seeds": sd, "scalars": sc}
        for n in init:
            arrays[f"init/{n}"] = init[n]
            arrays[f"final/{n}"] = final[n]
        np.savez(os.path.join(OUT, f"reconstruct_{name}.npz"), **arrays)
        cases[name] = case
    # weight_decay None in the groups -> zo_utils.py:52 branch
    model = build_model("float32", seed=77)
    groups = [{"params": list(model.parameters()), "weight_decay": None, "lr": 1e-3}]
    init = snapshot(model)
    sd, sc = seeds_scalars(12, 555)
    for s, g in zip(sd.tolist(), sc.tolist()):
        if g != 0.0:
            zo_utils.directional_derivative_step(groups, int(s), g)
    arrays = {"seeds": sd, "scalars": sc}
    for n in init:
        arrays[f"init/{n}"] = init[n]
        arrays[f"final/{n}"] = snapshot(model)[n]
    np.savez(os.path.join(OUT, "reconstruct_f32_wdnone.npz"), **arrays)
    cases["f32_wdnone"] = {"dtype": "float32", "k": 12, "lr": None, "wd": None, "sticky": True,
                           "groups": [[n for n, _ in model.named_parameters()]], "group_wd": [None],
                           "group_lr": [1e-3], "shapes": {n: list(p.shape) for n, p in model.named_parameters()}}
    return cases


# --------------------------------------------------------------------------- perturb / ZO step
def gen_optimizer():
    cases = {}
    for dtype in ("float32", "bfloat16"):
        model = build_model(dtype, ragged=True, seed=5)
        model.ln_1.weight.requires_grad_(False)  # a frozen tensor inside a group: no z drawn for it
        groups = pytorch_utils.get_optimizer_parameters_grouped_with_decay(model, 0.01)
        groups[1]["params"].append(model.ln_1.weight)  # keep it in the group despite requires_grad=False
        opt = ref_opt.ZerothOrderOptimizer(groups, lr=1e-3, eps=5e-4, weight_decay=0.01, grad_clip=-100.0)
        arrays = {"init": None}
        snaps = [snapshot(model)]
        for sf in (1.0, -2.0, 1.0):
            opt.random_perturb_parameters(987654321, scaling_factor=sf)
            snaps.append(snapshot(model))
        # zeroth_order_step with a device-independent closure (pre-set losses)
        losses = iter([torch.tensor(2.5), torch.tensor(2.375)])
        g, lr_, ll_ = opt.zeroth_order_step(12345678, lambda: next(losses))
        snaps.append(snapshot(model))
        arrays = {}
        for i, s in enumerate(snaps):
            for n, v in s.items():
                arrays[f"s{i}/{n}"] = v
        arrays["g"] = np.array([float(g)])
        np.savez(os.path.join(OUT, f"optimizer_{dtype}.npz"), **arrays)
        cases[dtype] = {"groups": group_layout(model, groups), "requires_grad": {n: p.requires_grad for n, p in model.named_parameters()},
                        "shapes": {n: list(p.shape) for n, p in model.named_parameters()},
                        "perturb_seed": 987654321, "step_seed": 12345678, "losses": [2.5, 2.375],
                        "eps": 5e-4, "lr": 1e-3, "wd": 0.01, "snapshots": ["init", "+1", "-2", "+1", "after zeroth_order_step"]}
    # KSeed optimizer: sampling with the unseeded torch.Generator() (optimizer.py:190)
    model = build_model("float32", seed=6)
    groups = pytorch_utils.get_optimizer_parameters_grouped_with_decay(model, 0.0)
    cand = zo_utils.build_seed_candidates(16, 0, 2**32) if False else torch.arange(1000, 1016, dtype=torch.long) * 7919
    probs = zo_utils.get_even_seed_probabilities(16)
    kopt = ref_opt.KSeedZerothOrderOptimizer(groups, cand, probs, lr=1e-3, eps=5e-4, weight_decay=0.0, grad_clip=-100.0)
    loss_seq = [3.0, 2.9, 2.8, 2.85, float("nan"), 2.7, 2.6, 2.65]
    it = iter([torch.tensor(x) for x in loss_seq])
    rets = [float(kopt.kseed_zeroth_order_step(lambda: next(it))) for _ in range(4)]
    arrays = {f"final/{n}": v for n, v in snapshot(model).items()}
    m0 = build_model("float32", seed=6)
    arrays.update({f"init/{n}": v for n, v in snapshot(m0).items()})
    hist = {str(k): v for k, v in kopt.directional_derivative_history.items() if v}
    np.savez(os.path.join(OUT, "optimizer_kseed.npz"), **arrays)
    cases["kseed"] = {"candidates": cand.tolist(), "losses": loss_seq, "returns": rets, "history": hist,
                      "groups": group_layout(model, groups), "shapes": {n: list(p.shape) for n, p in model.named_parameters()},
                      "lr": 1e-3, "eps": 5e-4, "wd": 0.0}
    return cases


# --------------------------------------------------------------------------- server side
class _FakeClient:
    def __init__(self, name, replies):
        self.name, self.replies, self.sent = name, replies, []

    def put(self, key, value):
        self.sent.append((key, value))

    def get(self, key):
        assert key == "direction_derivative_history"
        return self.replies.pop(0)


class _FakeCtx:
    def __init__(self, guest, hosts):
        self.guest, self.hosts = guest, hosts

    def ctxs_range(self, n):
        for i in range(n):
            yield i, self


def gen_server():
    out = {}
    amps = [[0.5, -2.0, 3.0], [1500.0, -0.1], [0.0], [7.0, 7.0, -7.0]]
    out["probability_from_amps"] = {"amps": amps, "clip": 1000.0,
                                    "probs": zo_utils.probability_from_amps([list(a) for a in amps], 1000.0).tolist()}
    out["even"] = zo_utils.get_even_seed_probabilities(5).tolist()
    if ref_fks is not None:
        seeds = torch.tensor([11, 22, 33, 44], dtype=torch.long)
        rng = np.random.default_rng(0)
        rounds = 3

        def replies():
            return [{int(s): [float(x) for x in rng.normal(0, 5, size=int(rng.integers(0, 3)))] for s in seeds.tolist()}
                    for _ in range(rounds)]
        guest, host = _FakeClient("guest", replies()), _FakeClient("host", replies())
        g_rep = [dict(r) for r in guest.replies]
        h_rep = [dict(r) for r in host.replies]
        args = ref_fks.FedKSeedTrainingArguments(num_aggregations=rounds, k=4)
        ref_fks.Trainer(_FakeCtx(guest, [host]), seeds, None, args).train()

        def enc(payload):
            should_exit, kw = payload
            dd = kw["direction_derivative_sum"]
            return {"should_exit": should_exit, "seed_candidates": kw["seed_candidates"].tolist(),
                    "seed_probabilities": kw["seed_probabilities"].tolist(),
                    "direction_derivative_sum": None if dd is None else {str(k): v for k, v in dd.items()}}
        out["trainer"] = {"seeds": seeds.tolist(), "rounds": rounds,
                          "guest_replies": [{str(k): v for k, v in r.items()} for r in g_rep],
                          "host_replies": [{str(k): v for k, v in r.items()} for r in h_rep],
                          "guest_sent": [enc(v) for _, v in guest.sent], "host_sent": [enc(v) for _, v in host.sent]}
    return out


def main():
    torch.set_num_threads(8)
    gen_mt()
    gen_streams()
    cases = {"meta": meta(), "reconstruct": gen_reconstruct(), "optimizer": gen_optimizer(), "server": gen_server()}
    with open(os.path.join(OUT, "cases.json"), "w") as f:
        json.dump(cases, f, indent=1, sort_keys=True)
    print("wrote fixtures to", OUT)


if __name__ == "__main__":
    main()
