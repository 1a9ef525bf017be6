"""Drop-in for python/fate_llm/algo/fedkseed/fedkseed.py (FATE-LLM 2.2.0).

Arbiter side (``Trainer``, reference :17-85): per round, recompute the seed-sampling
probabilities from every seed's directional-derivative history, send
``(should_exit, {seed_candidates, seed_probabilities, direction_derivative_sum})`` to
every client, then fold the clients' histories into the history and the cumulative
float64 sums.  Only K-sized scalars move; nothing here touches parameters.

Client side (``ClientTrainer``, reference :88-158): per round, rebuild the model from
``model_0`` plus the cumulative (seed, sum) list -- the K-seed reconstruct, one
``zo_utils.reconstruct_`` call on the MI355X codec instead of K Python-level
``directional_derivative_step`` calls -- then run local KSeedZO training and return
the directional-derivative history.

The federation context is duck-typed (``ctxs_range``, ``guest``, ``hosts``,
``arbiter.put/get``), so ``fate.arch`` is not a dependency of this package.

The z stream (codec.py) is part of the round: a client logs the stream it draws and,
over a ``payload.WireContext``, tags its histories with it; the arbiter rejects a
history drawn from another stream than the rest of the federation's
(``payload.StreamMismatchError``), since the reference's parties would otherwise apply
one (seed, scalar) list along different directions without noticing.

Round pipeline.  The reference rebuilds the model every round
as ``copy.deepcopy(model_0).to(device)`` (fedkseed.py:132-133): a host copy of the
whole buffer, then a pageable H2D copy.  The drop-in builds the device model directly:
the module structure is deep-copied with every parameter and buffer already replaced by
a device tensor, and the bytes move host -> device once, through pinned staging buffers
on a side stream (a host-side memcpy of chunk i+1 overlaps the DMA of chunk i).  Two
opt-in placements of ``model_0`` go further (``model_0_placement``): "pinned" pins
model_0's host tensors once, so every round is one DMA at PCIe speed; "device" keeps a
copy of model_0 on the device, so every round is a device-to-device copy.  All three
give the reference's values bit for bit (copies only).
"""
import copy
import logging
import threading
from dataclasses import dataclass, field
from typing import Dict, List, Mapping, Optional

import torch

from . import codec
from .args import KSeedTrainingArguments
from .payload import WireContext, check_stream
from .pytorch_utils import get_optimizer_parameters_grouped_with_decay
from .zo_utils import get_even_seed_probabilities, probability_from_amps, reconstruct_

logger = logging.getLogger(__name__)


class Trainer:
    """FedKSeed arbiter (reference fedkseed.py:17-85)."""

    def __init__(self, ctx, seed_candidates: torch.LongTensor, args, fedkseed_args):
        self.ctx = ctx
        self.args = args
        self.fedkseed_args = fedkseed_args
        self.seed_candidates = seed_candidates
        self.k = len(seed_candidates)
        self.model = None
        # the federation's z stream (and torch_rocm grid cap): what a WireContext declared,
        # else the first tagged client history's; every later tagged history must match it,
        # and once known it is declared into the arbiter's own WireContext, so that the
        # "train_once" records it sends from then on carry it to the clients
        wire = isinstance(ctx, WireContext)
        self.stream_mode = ctx.stream_mode if wire else None
        self.stream_grid = ctx.stream_grid if wire else None

    @staticmethod
    def get_clients(ctx) -> list:
        """The guest, then every host (a context without hosts has only the guest)."""
        clients = [ctx.guest]
        hosts = getattr(ctx, "hosts", None)
        if hosts:
            clients.extend(hosts)
        return clients

    def load_model(self):
        raise NotImplementedError

    def _probabilities(self, history: Dict[int, List[float]], first: bool):
        if first:
            return get_even_seed_probabilities(self.k)
        return probability_from_amps([history[s.item()] for s in self.seed_candidates],
                                     self.fedkseed_args.bias_loss_clip)

    def train(self):
        history: Dict[int, List[float]] = {s.item(): [self.fedkseed_args.grad_initial] for s in self.seed_candidates}
        # one dict object for the whole run, updated in place after every round (the
        # reference hands the same object to every put)
        sums: Optional[Dict[int, float]] = None
        probs = None
        for _, sub_ctx in self.ctx.ctxs_range(self.fedkseed_args.num_aggregations):
            probs = self._probabilities(history, first=probs is None)
            payload = {"seed_candidates": self.seed_candidates, "seed_probabilities": probs,
                       "direction_derivative_sum": sums}
            clients = self.get_clients(sub_ctx)
            for client in clients:
                client.put("train_once", (False, payload))
            if sums is None:
                sums = {s.item(): 0.0 for s in self.seed_candidates}
            tagged = untagged = 0
            for i, client in enumerate(clients):
                hist = client.get("direction_derivative_history")
                stream = getattr(hist, "stream_mode", None)  # payload.History of a tagged record
                grid = getattr(hist, "stream_grid", None)
                check_stream(self.stream_mode, stream, f"client {i} (guest first, then hosts)", self.stream_grid, grid)
                if stream is None:
                    untagged += 1
                else:
                    tagged += 1
                    self._adopt_stream(stream, grid)
                for seed, values in hist.items():
                    seed = int(seed)
                    history.setdefault(seed, []).extend(values)
                    # python float sum of the new values, then one float64 add; a seed
                    # outside the candidates raises KeyError, as in the reference
                    sums[seed] += sum(values)
            if tagged and untagged:
                logger.warning(f"FedKSeed arbiter: {untagged} of {tagged + untagged} clients sent untagged histories "
                               f"(reference parties?) beside clients drawing {self.stream_mode}; their z stream "
                               "cannot be checked")
            if self.should_stop():
                break

    def _adopt_stream(self, stream: str, grid) -> None:
        """Take the first tagged history's stream as the federation's and declare it into
        the arbiter's WireContext (its later "train_once" records carry it)."""
        changed = False
        if self.stream_mode is None:
            self.stream_mode, changed = stream, True
        if self.stream_mode == "torch_rocm" and self.stream_grid is None and grid is not None:
            self.stream_grid, changed = grid, True
        if changed and isinstance(self.ctx, WireContext):
            self.ctx.declare_stream_mode(self.stream_mode, self.stream_grid)

    def should_stop(self) -> bool:
        return False

    def evaluate(self):
        pass


_STAGE_BYTES = 64 << 20
_STAGES = 3


def _h2d_staged(pairs, device) -> None:
    """dst.copy_(src) for every (device dst, source) pair, through _STAGES pinned
    buffers on a side stream; pinned and device sources go straight to the DMA.  The side
    stream first waits for the current stream (the destinations were allocated there, and
    their memory's previous owner or a device source's producer may still have work
    queued on it); the current stream then waits for the copies (the caller's next kernels
    see the data)."""
    cur = torch.cuda.current_stream(device)
    stream = torch.cuda.Stream(device)
    stream.wait_stream(cur)
    bufs, ready = [], [None] * _STAGES
    i = 0
    with torch.cuda.stream(stream):
        for dst, src in pairs:
            if src.numel() == 0:
                continue
            if src.is_pinned() or src.device.type == "cuda":
                dst.copy_(src, non_blocking=True)
                continue
            s = src.contiguous().view(-1).view(torch.uint8)
            d = dst.view(-1).view(torch.uint8)
            for off in range(0, s.numel(), _STAGE_BYTES):
                n = min(_STAGE_BYTES, s.numel() - off)
                slot = i % _STAGES
                if len(bufs) <= slot:
                    bufs.append(torch.empty(_STAGE_BYTES, dtype=torch.uint8, pin_memory=True))
                if ready[slot] is not None:
                    ready[slot].synchronize()  # the DMA that last read this buffer is done
                bufs[slot][:n].copy_(s[off:off + n])  # host memcpy (parallel), overlaps the previous DMA
                d[off:off + n].copy_(bufs[slot][:n], non_blocking=True)
                ready[slot] = torch.cuda.Event()
                ready[slot].record(stream)
                i += 1
    cur.wait_stream(stream)
    stream.synchronize()  # the staging buffers are released on return


def _device_copy(module, device):
    """copy.deepcopy(module).to(device) without the host copy: every parameter and
    buffer is replaced by a device tensor of the same values (tied tensors stay tied)."""
    memo, pairs = {}, []
    tensors = list(module.named_parameters(remove_duplicate=True)) + list(module.named_buffers(remove_duplicate=True))
    for _, t in tensors:
        if id(t) in memo:
            continue
        data = torch.empty(t.shape, dtype=t.dtype, device=device)
        pairs.append((data, t.detach()))
        if isinstance(t, torch.nn.Parameter):
            new = torch.nn.Parameter(data, requires_grad=t.requires_grad)
        else:
            new = data
        memo[id(t)] = new
    out = copy.deepcopy(module, memo)
    if any(dst.device.type == "cuda" for dst, _ in pairs):
        _h2d_staged(pairs, device)
    else:
        for dst, src in pairs:
            dst.copy_(src)
    return out


class ClientTrainer:
    """FedKSeed client (reference fedkseed.py:88-158).

    ``model_0_placement`` (keyword, not in the reference): "host" (default; model_0
    stays as given, each round materialises it on the device through pinned staging),
    "pinned" (model_0's host tensors are pinned once; each round is one DMA) or
    "device" (a device copy of model_0 is kept; each round is a device-to-device copy)."""

    def __init__(self, ctx, model, fedkseed_args, training_args, train_dataset, eval_dataset, data_collator,
                 tokenizer, model_0_placement: str = "host"):
        self.ctx = ctx
        self.fedkseed_args = fedkseed_args
        self.training_args = training_args
        self.data_collator = data_collator
        self.train_dataset = train_dataset
        self.eval_dataset = eval_dataset
        self.tokenizer = tokenizer
        self.weight_decay = training_args.weight_decay
        self.model_0 = model
        if model_0_placement not in ("host", "pinned", "device"):
            raise ValueError(f"model_0_placement must be host, pinned or device, not {model_0_placement!r}")
        self.model_0_placement = model_0_placement
        self._model_0_device = None
        self._pinned = False
        self._lock = threading.Lock()

    @property
    def stream_mode(self) -> str:
        """The z stream this client's reconstruct and local steps draw: the process-wide
        codec setting resolved for the training device (FKS_STREAM_MODE unset = "auto":
        torch_rocm on an MI355X, what an unmodified reference client there draws), as
        codec.stream_identity names it ("torch_cpu_libm": the CPU stream under ATen's DEFAULT
        capability, for a model with fp32 tensors of >= 16 elements)."""
        mode = codec.resolve_stream_mode(getattr(self.training_args, "device", None))
        return codec.stream_identity(mode, self.model_0.parameters() if self.model_0 is not None else None)

    @property
    def stream_grid(self):
        """torch_rocm only: the grid cap of the training device (codec.rocm_grid_cap), part of
        the stream's identity -- torch draws every tensor above 256 x cap / 4 elements in a
        grid of cap blocks (DistributionTemplates.h:50-62); None for torch_cpu."""
        if self.stream_mode != "torch_rocm":
            return None
        return self._device_grid_cap()

    def _device_grid_cap(self) -> int:
        return codec.rocm_grid_cap(getattr(self.training_args, "device", None))

    def train(self):
        stream, grid = self.stream_mode, self.stream_grid
        logger.info(f"FedKSeed client: z stream {stream}" + (f", grid cap {grid}" if grid is not None else "") +
                    f" (codec setting {codec.get_stream_mode()!r})")
        if isinstance(self.ctx, WireContext):
            self.ctx.declare_stream_mode(stream, grid)  # tags the histories this client sends
        for i, sub_ctx in self.ctx.ctxs_range(self.fedkseed_args.num_aggregations):
            logger.info(f"training loop started: {i}")
            should_exit, kwargs = sub_ctx.arbiter.get("train_once")
            check_stream(stream, kwargs.get("stream_mode"), "the arbiter", grid, kwargs.get("stream_grid"))
            if should_exit:
                break
            history = self.train_once(kwargs["seed_candidates"], kwargs["seed_probabilities"],
                                      kwargs["direction_derivative_sum"])
            sub_ctx.arbiter.put("direction_derivative_history", history)

    def materialize(self, device=None):
        """A fresh copy of model_0 on ``device`` (the training device by default): the
        reference's copy.deepcopy(model_0).to(device) (fedkseed.py:132-133)."""
        device = torch.device(device if device is not None else self.training_args.device)
        if device.type != "cuda":
            return copy.deepcopy(self.model_0).to(device)
        with self._lock:
            if self.model_0_placement == "device":
                if self._model_0_device is None:
                    self._model_0_device = _device_copy(self.model_0, device)
                return copy.deepcopy(self._model_0_device)
            if self.model_0_placement == "pinned" and not self._pinned:
                for t in list(self.model_0.parameters()) + list(self.model_0.buffers()):
                    if t.device.type == "cpu" and not t.is_pinned():
                        t.data = t.data.pin_memory()
                self._pinned = True
        return _device_copy(self.model_0, device)

    def reconstruct(self, direction_derivative_sum: Optional[Mapping[int, float]]):
        """model_0 + every accumulated (seed, sum) step, in the dict's insertion order,
        zero sums skipped (reference :130-141), on the training device."""
        model = self.materialize()
        if direction_derivative_sum is not None:
            groups = get_optimizer_parameters_grouped_with_decay(model, self.weight_decay)
            reconstruct_(groups, list(direction_derivative_sum.keys()), list(direction_derivative_sum.values()),
                         lr=self.training_args.learning_rate, weight_decay=self.training_args.weight_decay)
        return model

    def train_once(self, seed_candidates, seed_probabilities, direction_derivative_sum) -> Mapping[int, List[float]]:
        from .trainer import KSeedZOExtendedTrainer  # needs transformers; the codec does not

        model = self.reconstruct(direction_derivative_sum)
        trainer = KSeedZOExtendedTrainer(
            model=model, training_args=self.training_args, kseed_args=self.fedkseed_args, tokenizer=self.tokenizer,
            data_collator=self.data_collator, train_dataset=self.train_dataset, eval_dataset=self.eval_dataset)
        trainer.configure_seed_candidates(seed_candidates, seed_probabilities)
        trainer.train()
        if self.eval_dataset is not None:
            logger.info(f"evaluate: {trainer.evaluate()}")
        return trainer.get_directional_derivative_history()


@dataclass
class FedKSeedTrainingArguments(KSeedTrainingArguments):
    """KSeed options plus the federation's (same fields and defaults as the reference)."""

    num_aggregations: int = field(default=10, metadata={"help": "The number of aggregations to perform."})
    bias_loss_clip: float = field(default=1000.0, metadata={"help": "The bias loss clip value."})
    grad_initial: float = field(
        default=0.0, metadata={"help": "The initial value for the directional derivative history."}
    )
