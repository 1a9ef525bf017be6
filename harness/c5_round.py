"""C5 end-to-end FedKSeed round harness (BASELINE config 5).

N clients (one process per GPU) and 1 aggregator process exchange the reference's
round payloads through the drop-in classes:
  * the aggregator runs ``fate_llm.algo.fedkseed.fedkseed.Trainer`` unchanged: seed
    probabilities from the directional-derivative histories (probability_from_amps),
    float64 cumulative sums, one payload per client per round;
  * each client runs ``ClientTrainer.reconstruct`` (the drop-in: deepcopy of model_0,
    .to(device) = the H2D copy, then ONE reconstruct_ of the cumulative (seed, sum)
    list on the MI355X codec) and S local KSeed zeroth-order steps with the drop-in
    ``KSeedZerothOrderOptimizer`` (2 perturbations + 1 fused restore/update per step,
    K=1 codec calls), then returns its history (scalars) to the aggregator.

The FATE transport is out of scope: payloads move as pickled objects
over a torch.distributed gloo group (CPU), the duck-typed context the drop-in Trainer /
ClientTrainer expect.  The closure is synthetic and deterministic (no transformer
forward): the loss is a reduction over one 4096-element slice of the
parameters, so a step's cost is the codec's.  Model: LLaMA-7B-shaped bf16 parameters
(random init, the bench's shapes) -- ``--params`` swaps in a flat buffer for tests.

``--warm`` starts the aggregator from a synthetic steady state in which every one of
the K seeds already has a non-zero cumulative sum, so the first round's reconstruct
replays all K seeds (a late round of a long run); without it round 1 has nothing to
reconstruct, exactly as in the reference.

  python harness/c5_round.py [--clients N] [--rounds R] [--steps S] [--k K] [--warm]
                             [--params P] [--resident] [--backend-device cuda|cpu]

Rank 0 prints one JSON line: per-round wall time and per-phase maxima over clients.
"""
import argparse
import copy
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "fate-llm_amd", "python")):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
from torch import nn  # noqa: E402


# ----------------------------------------------------------------------------- transport
class _Peer:
    """One remote party: put = send a (key, value) object, get = receive one and check
    its key (the reference's ctx.<party>.put/get, in order)."""

    def __init__(self, rank):
        self.rank = rank

    def put(self, key, value):
        dist.send_object_list([(key, value)], dst=self.rank)

    def get(self, key):
        box = [None]
        dist.recv_object_list(box, src=self.rank)
        k, v = box[0]
        if k != key:
            raise RuntimeError(f"expected {key!r} from rank {self.rank}, got {k!r}")
        return v


class _Ctx:
    """Duck-typed federation context: ctxs_range, guest, hosts (aggregator side),
    arbiter (client side)."""

    def __init__(self, clients, arbiter):
        self.guest = _Peer(clients[0]) if clients else None
        self.hosts = [_Peer(r) for r in clients[1:]]
        self.arbiter = _Peer(arbiter) if arbiter is not None else None

    def ctxs_range(self, n):
        for i in range(n):
            yield i, self


# ----------------------------------------------------------------------------- model
def llama7b_shapes():
    h, inter, v, L = 4096, 11008, 32000, 32
    names = [("model.embed_tokens.weight", (v, h))]
    for i in range(L):
        p = f"model.layers.{i}."
        names += [(p + "self_attn.q_proj.weight", (h, h)), (p + "self_attn.k_proj.weight", (h, h)),
                  (p + "self_attn.v_proj.weight", (h, h)), (p + "self_attn.o_proj.weight", (h, h)),
                  (p + "mlp.gate_proj.weight", (inter, h)), (p + "mlp.up_proj.weight", (inter, h)),
                  (p + "mlp.down_proj.weight", (h, inter)), (p + "input_layernorm.weight", (h,)),
                  (p + "post_attention_layernorm.weight", (h,))]
    names += [("model.norm.weight", (h,)), ("lm_head.weight", (v, h))]
    return names


class SyntheticModel(nn.Module):
    """Parameters with LLaMA-7B names and shapes (RMSNorm weights are plain parameters,
    so, as for LlamaRMSNorm, every tensor lands in the decay group)."""

    def __init__(self, shapes, dtype, device):
        super().__init__()
        self._names = []
        for name, shape in shapes:
            mod = self
            parts = name.split(".")
            for part in parts[:-1]:
                if not hasattr(mod, part):
                    mod.add_module(part, nn.Module())
                mod = getattr(mod, part)
            mod.register_parameter(parts[-1], nn.Parameter(torch.empty(shape, dtype=dtype, device=device)))
            self._names.append(name)


def build_model_0(shapes, seed=0):
    """model_0 on the host, values N(0, 0.02^2) drawn on the GPU (setup, not timed)."""
    m = SyntheticModel(shapes, torch.bfloat16, "cpu")
    gen = torch.Generator(device="cuda").manual_seed(seed)
    for p in m.parameters():
        p.data.copy_(torch.empty(p.shape, dtype=torch.bfloat16, device="cuda").normal_(0, 0.02, generator=gen).cpu())
    return m


# ----------------------------------------------------------------------------- client
def run_client(rank, args, arbiter_rank):
    from fate_llm.algo.fedkseed.fedkseed import ClientTrainer, FedKSeedTrainingArguments
    from fate_llm.algo.fedkseed.optimizer import KSeedZerothOrderOptimizer
    from fate_llm.algo.fedkseed.pytorch_utils import get_optimizer_parameters_grouped_with_decay

    ndev = torch.cuda.device_count()
    dev = torch.device("cuda", rank % ndev)
    torch.cuda.set_device(dev)
    shapes = [("flat", (args.params,))] if args.params else llama7b_shapes()
    model_0 = build_model_0(shapes, seed=0)

    class TrainingArgs:
        learning_rate = 1e-5
        weight_decay = 0.0
        device = dev

    fk = FedKSeedTrainingArguments(num_aggregations=args.rounds, k=args.k)
    ctx = _Ctx([], arbiter_rank)
    trainer = ClientTrainer(ctx, model_0, fk, TrainingArgs(), None, None, None, None)
    resident = None
    if args.resident:  # §8(f) row 2: model_0 kept on the device across rounds
        resident = copy.deepcopy(model_0).to(dev)

    timings = []
    for rnd, sub in ctx.ctxs_range(args.rounds):
        should_exit, kw = sub.arbiter.get("train_once")
        if should_exit:
            break
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if resident is None:
            # the drop-in ClientTrainer.reconstruct, phase by phase (deepcopy, H2D, codec)
            model = copy.deepcopy(trainer.model_0)
            t1 = time.perf_counter()
            model.to(dev)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
        else:
            model = copy.deepcopy(resident)  # device-to-device
            torch.cuda.synchronize()
            t1 = t2 = time.perf_counter()
        sums = kw["direction_derivative_sum"]
        n_rec = 0
        if sums is not None:
            from fate_llm.algo.fedkseed.zo_utils import reconstruct_
            groups = get_optimizer_parameters_grouped_with_decay(model, TrainingArgs.weight_decay)
            n_rec = reconstruct_(groups, list(sums.keys()), list(sums.values()), lr=TrainingArgs.learning_rate,
                                 weight_decay=TrainingArgs.weight_decay)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        opt = KSeedZerothOrderOptimizer(
            get_optimizer_parameters_grouped_with_decay(model, TrainingArgs.weight_decay),
            seed_candidates=kw["seed_candidates"], seed_probabilities=kw["seed_probabilities"],
            lr=TrainingArgs.learning_rate, eps=fk.eps, weight_decay=TrainingArgs.weight_decay,
            grad_clip=fk.grad_clip)
        opt.sample_random_generator.manual_seed(1000 * rnd + rank)  # deterministic harness
        probe = next(model.parameters()).view(-1)[:4096]

        @torch.no_grad()
        def closure():
            return probe.float().square().mean() * 1e3

        for _ in range(args.steps):
            opt.kseed_zeroth_order_step(closure)
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        history = {s: v for s, v in opt.directional_derivative_history.items()}
        sub.arbiter.put("direction_derivative_history", history)
        t5 = time.perf_counter()
        timings.append({"round": rnd, "copy_s": t1 - t0, "h2d_s": t2 - t1, "reconstruct_s": t3 - t2,
                        "seeds_reconstructed": n_rec, "local_steps_s": t4 - t3, "send_s": t5 - t4,
                        "client_round_s": t5 - t0})
        del model, opt
    return timings


# ----------------------------------------------------------------------------- aggregator
def run_aggregator(args, clients):
    from fate_llm.algo.fedkseed.fedkseed import FedKSeedTrainingArguments, Trainer
    from fate_llm.algo.fedkseed.zo_utils import build_seed_candidates

    torch.manual_seed(42)
    seeds = build_seed_candidates(args.k)
    fk = FedKSeedTrainingArguments(num_aggregations=args.rounds, k=args.k)
    ctx = _Ctx(clients, None)

    class WarmTrainer(Trainer):
        """Trainer.train with an optional synthetic steady state: every seed already has
        a non-zero cumulative sum and one history entry (--warm)."""

        def train(self):
            if not args.warm:
                return super().train()
            g = torch.Generator().manual_seed(7)
            vals = (torch.randn(self.k, generator=g, dtype=torch.float64) * 20).tolist()
            history = {s.item(): [self.fedkseed_args.grad_initial, v] for s, v in zip(self.seed_candidates, vals)}
            sums = {s.item(): v for s, v in zip(self.seed_candidates, vals)}
            for _, sub in self.ctx.ctxs_range(self.fedkseed_args.num_aggregations):
                probs = self._probabilities(history, first=False)
                payload = {"seed_candidates": self.seed_candidates, "seed_probabilities": probs,
                           "direction_derivative_sum": sums}
                cl = self.get_clients(sub)
                for c in cl:
                    c.put("train_once", (False, payload))
                for c in cl:
                    for seed, values in c.get("direction_derivative_history").items():
                        history.setdefault(int(seed), []).extend(values)
                        sums[int(seed)] += sum(values)

    t0 = time.perf_counter()
    WarmTrainer(ctx, seeds, None, fk).train()
    return time.perf_counter() - t0


def _worker(rank, world, port, args, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        clients = list(range(world - 1))
        arbiter = world - 1
        if rank == arbiter:
            out = {"aggregator_s": run_aggregator(args, clients)}
        else:
            out = {"client": rank, "rounds": run_client(rank, args, arbiter)}
        gathered = [None] * world
        dist.all_gather_object(gathered, out)
        if rank == 0:
            q.put(gathered)
    finally:
        dist.destroy_process_group()


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=1)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--steps", type=int, default=151, help="local ZO steps per round (tutorial notebook :223)")
    ap.add_argument("--k", type=int, default=4096)
    ap.add_argument("--params", type=int, default=0, help="flat buffer of this many params instead of 7B shapes")
    ap.add_argument("--warm", action="store_true")
    ap.add_argument("--resident", action="store_true", help="keep model_0 on the device (no deepcopy/H2D)")
    args = ap.parse_args(argv)
    import torch.multiprocessing as mp

    world = args.clients + 1
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, args, q)) for r in range(world)]
    for p in procs:
        p.start()
    gathered = q.get()
    for p in procs:
        p.join()
        if p.exitcode != 0:
            raise SystemExit(f"a harness process exited with {p.exitcode}")
    clients = [g for g in gathered if "client" in g]
    agg = [g for g in gathered if "aggregator_s" in g][0]
    rounds = []
    for r in range(len(clients[0]["rounds"])):
        per = [c["rounds"][r] for c in clients]
        rounds.append({k: (max(p[k] for p in per) if isinstance(per[0][k], float) else per[0][k]) for k in per[0]})
    nparams = args.params or sum(torch.Size(s).numel() for _, s in llama7b_shapes())
    out = {"harness": "C5 FedKSeed round", "clients": args.clients, "k": args.k, "steps": args.steps,
           "params": nparams, "dtype": "bf16", "warm": args.warm, "resident_model_0": args.resident,
           "transport": "torch.distributed gloo (stand-in for the FATE federation)",
           "rounds": [{k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()} for r in rounds],
           "aggregator_total_s": round(agg["aggregator_s"], 3)}
    print(json.dumps(out), flush=True)
    return out


if __name__ == "__main__":
    main()
