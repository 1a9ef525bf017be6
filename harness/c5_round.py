"""C5 end-to-end FedKSeed round harness (BASELINE config 5).

N clients (one process per GPU) and 1 aggregator process exchange the reference's
round payloads through the drop-in classes:
  * the aggregator runs ``fate_llm.algo.fedkseed.fedkseed.Trainer`` unchanged: seed
    probabilities from the directional-derivative histories (probability_from_amps),
    float64 cumulative sums, one payload per client per round;
  * each client runs the drop-in ``ClientTrainer``: ``reconstruct`` (model_0 onto the
    device -- ``--placement`` host: staged H2D through pinned buffers, pinned: model_0
    pinned once, device: a resident copy -- then ONE reconstruct_ of the cumulative
    (seed, sum) list on the MI355X codec) and S local KSeed zeroth-order steps, then
    returns its history (scalars) to the aggregator.  ``--driver trainer`` runs the
    whole ``ClientTrainer.train`` loop as the reference does, the local steps through
    ``KSeedZOExtendedTrainer.training_step`` in the transformers training loop;
    ``--driver optimizer`` (default) drives the drop-in ``KSeedZerothOrderOptimizer``
    directly (2 perturbations + 1 fused restore/update per step, K=1 codec calls).
  * ``--wire``: both ends wrap their context in payload.WireContext, so the round
    payloads travel in the compact binary format; bytes per round are reported.
  * ``--record`` (parity instrumentation, tests/test_gpu_c5_harness.py): each client also
    returns its model_0 prefix, and per round the payload it received, the first 4096
    parameters after the reconstruct and after the local steps, and its local steps in
    order (sampled seed, g, group-0 lr), so every client's round can be replayed through
    the oracle.

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
                             [--params P] [--placement host|pinned|device] [--driver optimizer|trainer]
                             [--wire]

Each client process sees one GPU (HIP_VISIBLE_DEVICES = client index mod GPU count), so
several clients can share one GPU in tests.

Rank 0 prints one JSON line: per-round wall time and per-phase maxima over clients.
"""
import argparse
import json
import pickle
import os
os.environ.setdefault("FKS_STREAM_MODE", "torch_cpu")  # the CPU-generator stream these measurements use
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

    def __init__(self, rank, meter):
        self.rank = rank
        self.meter = meter  # bytes sent / received per key, as pickled by the transport

    def put(self, key, value):
        self.meter[key + ".sent"] = self.meter.get(key + ".sent", 0) + len(pickle.dumps((key, value)))
        dist.send_object_list([(key, value)], dst=self.rank)

    def get(self, key):
        box = [None]
        dist.recv_object_list(box, src=self.rank)
        k, v = box[0]
        self.meter[key + ".recv"] = self.meter.get(key + ".recv", 0) + len(pickle.dumps((k, v)))
        if k != key:
            raise RuntimeError(f"expected {key!r} from rank {self.rank}, got {k!r}")
        return v


class _Ctx:
    """Duck-typed federation context: ctxs_range, guest, hosts (aggregator side),
    arbiter (client side)."""

    def __init__(self, clients, arbiter):
        self.meter = {}
        self.guest = _Peer(clients[0], self.meter) if clients else None
        self.hosts = [_Peer(r, self.meter) for r in clients[1:]]
        self.arbiter = _Peer(arbiter, self.meter) if arbiter is not None else None

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
    so, as for LlamaRMSNorm, every tensor lands in the decay group).  forward() is the
    synthetic closure: a loss from one 4096-element slice of the first tensor (no
    transformer forward), returned as the transformers loss output."""

    def forward(self, input_ids=None, labels=None, **_):
        probe = next(self.parameters()).view(-1)[:4096]
        return {"loss": probe.float().square().mean() * 1e3}

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
class _Steps(torch.utils.data.Dataset):
    """S dummy batches for the transformers loop (the synthetic model ignores them)."""

    def __init__(self, n):
        self.n = n

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        return {"input_ids": torch.zeros(1, dtype=torch.long)}


PREFIX = 4096  # parameters of the first tensor a --record client reports (--record-prefix)


def _prefix_bits(model, n=PREFIX):
    """The first n elements (0: all) of the model's first parameter, as raw bits (bf16: u16)."""
    t = next(model.parameters()).detach().reshape(-1)
    t = t[:n] if n else t
    return t.view(torch.int16).cpu().numpy().view("u2").tolist()


def run_client(rank, args, arbiter_rank):
    from fate_llm.algo.fedkseed import fedkseed as F
    from fate_llm.algo.fedkseed import optimizer as OPT
    from fate_llm.algo.fedkseed.optimizer import KSeedZerothOrderOptimizer
    from fate_llm.algo.fedkseed.payload import WireContext
    from fate_llm.algo.fedkseed.pytorch_utils import get_optimizer_parameters_grouped_with_decay
    from fate_llm.algo.fedkseed.zo_utils import reconstruct_

    dev = torch.device("cuda", 0)  # the one GPU this client process sees
    torch.cuda.set_device(dev)
    shapes = [("flat", (args.params,))] if args.params else llama7b_shapes()
    model_0 = build_model_0(shapes, seed=0)
    fk = F.FedKSeedTrainingArguments(num_aggregations=args.rounds, k=args.k)
    raw = _Ctx([], arbiter_rank)
    ctx = WireContext(raw) if args.wire else raw
    timings, received_all, histories = [], [], []
    records = {"model_0": _prefix_bits(model_0, args.record_prefix), "rounds": []} if args.record else None
    steps = []  # this round's local steps: (seed, g as returned -- a device or host value --, group-0 lr)
    if args.record:
        orig_step = OPT.ZerothOrderOptimizer.zeroth_order_step

        def recorded_step(self, seed, closure):
            lr = self.param_groups[0]["lr"]  # the sticky lr of the step's update (zo_utils.py:44-45)
            out = orig_step(self, seed, closure)
            steps.append((int(seed), out[0], float(lr)))
            return out

        OPT.ZerothOrderOptimizer.zeroth_order_step = recorded_step

    if args.driver == "trainer":
        import tempfile

        import transformers
        training_args = transformers.TrainingArguments(
            output_dir=tempfile.mkdtemp(prefix="c5_"), per_device_train_batch_size=1, max_steps=args.steps,
            learning_rate=1e-5, weight_decay=0.0, report_to=[], save_strategy="no", logging_strategy="no",
            max_grad_norm=0.0, dataloader_num_workers=0, disable_tqdm=True)
    else:
        class training_args:  # noqa: N801 -- the attributes ClientTrainer reads
            learning_rate = 1e-5
            weight_decay = 0.0
            device = dev

    class TimedClient(F.ClientTrainer):
        """The drop-in ClientTrainer with per-phase clocks (no behavioural change)."""

        def reconstruct(self, sums):
            received_all.append(None if sums is None else {int(k): float(v) for k, v in sums.items()})
            steps.clear()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            model = self.materialize()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            n = 0
            if sums is not None:
                groups = get_optimizer_parameters_grouped_with_decay(model, self.weight_decay)
                n = reconstruct_(groups, list(sums.keys()), list(sums.values()),
                                 lr=self.training_args.learning_rate, weight_decay=self.training_args.weight_decay)
            torch.cuda.synchronize()
            self._t = {"t0": t0, "materialize_s": t1 - t0, "reconstruct_s": time.perf_counter() - t1,
                       "seeds_reconstructed": n}
            if records is not None:
                self._model = model
                self._after_reconstruct = _prefix_bits(model, args.record_prefix)
            return model

        def train_once(self, seed_candidates, seed_probabilities, direction_derivative_sum):
            if args.driver == "trainer":
                hist = super().train_once(seed_candidates, seed_probabilities, direction_derivative_sum)
            else:
                model = self.reconstruct(direction_derivative_sum)
                t = time.perf_counter()
                opt = KSeedZerothOrderOptimizer(
                    get_optimizer_parameters_grouped_with_decay(model, self.weight_decay),
                    seed_candidates=seed_candidates, seed_probabilities=seed_probabilities,
                    lr=self.training_args.learning_rate, eps=fk.eps, weight_decay=self.weight_decay,
                    grad_clip=fk.grad_clip)
                opt.sample_random_generator.manual_seed(1000 * len(timings) + rank)  # deterministic harness

                @torch.no_grad()
                def closure():
                    return model(input_ids=None)["loss"]

                for _ in range(args.steps):
                    opt.kseed_zeroth_order_step(closure)
                hist = opt.directional_derivative_history
                if args.d2h:
                    # the path ends in host memory (the north star's H<->D clause): the trained
                    # parameters back into pinned host buffers, timed on their own
                    torch.cuda.synchronize()
                    td = time.perf_counter()
                    if not hasattr(self, "_host"):  # one pinned buffer per parameter, kept across rounds
                        self._host = [torch.empty(p.shape, dtype=p.dtype, pin_memory=True) for p in model.parameters()]
                    for buf, p in zip(self._host, model.parameters()):
                        buf.copy_(p.detach(), non_blocking=True)
                    torch.cuda.synchronize()
                    self._t["d2h_s"] = time.perf_counter() - td
                del model, opt
            torch.cuda.synchronize()
            end = time.perf_counter()
            rec = dict(self._t)
            t0 = rec.pop("t0")
            rec["local_steps_s"] = end - t0 - rec["materialize_s"] - rec["reconstruct_s"] - rec.get("d2h_s", 0.0)
            rec["client_round_s"] = end - t0
            rec["round"] = len(timings)
            timings.append(rec)
            hist = {int(s): list(v) for s, v in hist.items()}
            histories.append(hist)
            if records is not None:
                records["rounds"].append({
                    "sums": received_all[-1],
                    "candidates": [int(x) for x in seed_candidates],
                    "probabilities": torch.as_tensor(seed_probabilities).float().tolist(),
                    "after_reconstruct": self._after_reconstruct,
                    "steps": [(sd, float(torch.as_tensor(g).reshape(()).item()), lr) for sd, g, lr in steps],
                    "after_steps": _prefix_bits(self._model, args.record_prefix),
                    "history": hist})
                self._model = None
            return hist

    trainer = TimedClient(ctx, model_0, fk, training_args, _Steps(args.steps) if args.driver == "trainer" else None,
                       None, None, None, model_0_placement=args.placement)
    trainer.train()
    small = args.k <= 256
    return {"rounds": timings, "received_sums": received_all if small else None,
            "histories": histories if small else None, "bytes": raw.meter, "records": records}


# ----------------------------------------------------------------------------- aggregator
def run_aggregator(args, clients):
    from fate_llm.algo.fedkseed.fedkseed import FedKSeedTrainingArguments, Trainer
    from fate_llm.algo.fedkseed.zo_utils import build_seed_candidates

    torch.manual_seed(42)
    seeds = build_seed_candidates(args.k)
    fk = FedKSeedTrainingArguments(num_aggregations=args.rounds, k=args.k)
    raw = _Ctx(clients, None)
    if args.wire:
        from fate_llm.algo.fedkseed.payload import WireContext
        ctx = WireContext(raw)
    else:
        ctx = raw
    replies = []

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
    return {"aggregator_s": time.perf_counter() - t0, "bytes": raw.meter, "seeds": seeds.tolist()}


def _worker(rank, world, port, args, ndev, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if rank < world - 1:  # a client sees one GPU (transformers would otherwise DataParallel over all)
        os.environ["HIP_VISIBLE_DEVICES"] = os.environ["CUDA_VISIBLE_DEVICES"] = str(rank % max(ndev, 1))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        clients = list(range(world - 1))
        arbiter = world - 1
        if rank == arbiter:
            out = run_aggregator(args, clients)
        else:
            out = {"client": rank, **run_client(rank, args, arbiter)}
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
    ap.add_argument("--resident", action="store_true", help="alias of --placement device")
    ap.add_argument("--placement", choices=("host", "pinned", "device"), default="host",
                    help="ClientTrainer model_0_placement")
    ap.add_argument("--driver", choices=("optimizer", "trainer"), default="optimizer")
    ap.add_argument("--wire", action="store_true", help="round payloads in the compact binary format")
    ap.add_argument("--d2h", action="store_true",
                    help="optimizer driver: copy the trained parameters back to pinned host memory, timed (d2h_s)")
    ap.add_argument("--record", action="store_true", help="return every client's round for an oracle replay")
    ap.add_argument("--record-prefix", type=int, default=PREFIX,
                    help="parameters of the first tensor --record reports (0: the whole tensor)")
    args = ap.parse_args(argv)
    if args.resident:
        args.placement = "device"
    import torch.multiprocessing as mp

    world = args.clients + 1
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ndev = torch.cuda.device_count()  # counting devices does not initialise the GPU
    procs = [ctx.Process(target=_worker, args=(r, world, port, args, ndev, q)) for r in range(world)]
    for p in procs:
        p.start()
    gathered = q.get()
    for p in procs:
        p.join()
        if p.exitcode != 0:
            raise SystemExit(f"a harness process exited with {p.exitcode}")
    clients = [g for g in gathered if "client" in g]
    agg = [g for g in gathered if "aggregator_s" in g][0]
    nrounds = max(len(clients[0]["rounds"]), 1)
    rounds = []
    for r in range(len(clients[0]["rounds"])):
        per = [c["rounds"][r] for c in clients]
        rounds.append({k: (max(p[k] for p in per) if isinstance(per[0][k], float) else per[0][k]) for k in per[0]})
    nparams = args.params or sum(torch.Size(s).numel() for _, s in llama7b_shapes())
    out = {"harness": "C5 FedKSeed round", "clients": args.clients, "k": args.k, "steps": args.steps,
           "params": nparams, "dtype": "bf16", "warm": args.warm, "placement": args.placement,
           "driver": args.driver, "wire": args.wire,
           "transport": "torch.distributed gloo (stand-in for the FATE federation)",
           "rounds": [{k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()} for r in rounds],
           "aggregator_total_s": round(agg["aggregator_s"], 3),
           "bytes_per_round_per_client": {k: v // (nrounds * args.clients) for k, v in agg["bytes"].items()},
           "seeds": agg["seeds"] if args.k <= 256 else None,
           "client_received_sums": {c["client"]: c["received_sums"] for c in clients} if args.k <= 256 else None,
           "client_histories": {c["client"]: c["histories"] for c in clients} if args.k <= 256 else None}
    print(json.dumps(out), flush=True)
    if args.record:  # returned, not printed (8 clients x 3 rounds x 3 prefixes)
        out["client_records"] = {c["client"]: c["records"] for c in clients}
    return out


if __name__ == "__main__":
    main()
