"""Drop-in for python/fate_llm/algo/fedkseed/zo_utils.py (FATE-LLM 2.2.0).

``directional_derivative_step`` (reference :23-54) runs on the MI355X codec;
``reconstruct_`` is the batched form ClientTrainer.train_once uses (one device pass
for all K seeds instead of K Python-level passes).  The scalar helpers
(``probability_from_amps`` :6-20, ``build_seed_candidates`` :57-61,
``get_even_seed_probabilities`` :64-68) operate on K-sized vectors and stay in torch.
"""
from typing import List, Sequence

import torch

from . import codec


def probability_from_amps(amps: List[List[float]], clip):
    """Seed-sampling distribution from each seed's directional-derivative history.

    amp_i = mean(|clamp(history_i, -clip, clip)|), min-max normalised, then softmax.
    Same arithmetic as the reference (fp32 torch ops, +1e-10 in the denominator).
    """
    per_seed = []
    for history in amps:
        h = torch.tensor(history, dtype=torch.float32)
        per_seed.append(h.clamp(-clip, clip).abs().mean())
    amp = torch.stack(per_seed)
    lo, hi = amp.min(), amp.max()
    return ((amp - lo) / (hi - lo + 1e-10)).softmax(0)


def _value_kind(value, specs=(), stream_mode=None):
    """(g as a python float, whether it is a tensor): a tensor g is cast to each
    parameter's dtype by the reference's ``g * z`` (zo_utils.py:49).  A 1-element tensor
    that is not 0-dim takes part in type promotion and broadcasting as a dimensioned
    tensor: that is the same update when the promoted dtype is the parameter's own and
    the parameter has a dimension; otherwise the reference rebinds ``param.data`` to a
    tensor of another dtype or shape, which an in-place update cannot be -- raised.

    Where z lives decides the cast: on the CPU (the torch_cpu stream) TensorIterator
    promotes the 0-dim g to the parameter dtype before the f32 multiply; with z on a GPU
    (the torch_rocm stream) a 0-dim g on the GPU is cast the same way (the kernel's
    dynamic-cast load), but a 0-dim g on the CPU is a "CPU scalar" whose f32 value enters
    the kernel unrounded (gpu_kernel_with_scalars: scalar_value<opmath_t>) -- the same
    multiply as a python number -- and a dimensioned CPU g is torch's device-mismatch
    error."""
    if isinstance(value, torch.Tensor) and value.device.type == "cpu" and specs:
        dev = specs[0].tensor.device
        if dev.type == "cuda" and codec.resolve_stream_mode(dev, stream_mode) == "torch_rocm":
            if value.dim() != 0:
                raise RuntimeError("Expected all tensors to be on the same device, but found at least two devices, "
                                   f"{dev} and cpu! (a {tuple(value.shape)} directional_derivative_value on the CPU "
                                   "times z on the GPU, zo_utils.py:49)")
            return float(value.item()), False
    if isinstance(value, torch.Tensor):
        if value.dim() != 0:
            if value.numel() != 1:
                raise ValueError("directional_derivative_value must be a python number or a 1-element tensor")
            for sp in specs:
                t = sp.tensor
                if torch.promote_types(value.dtype, t.dtype) != t.dtype or t.dim() == 0:
                    raise NotImplementedError(
                        f"a {tuple(value.shape)} {value.dtype} directional_derivative_value would turn a "
                        f"{tuple(t.shape)} {t.dtype} parameter into {torch.promote_types(value.dtype, t.dtype)} "
                        "of the broadcast shape (the reference rebinds param.data); pass a 0-dim tensor")
        return float(value.reshape(()).item()), True
    return float(value), False


def directional_derivative_step(
    param_groups: List[dict],
    directional_derivative_seed: int,
    directional_derivative_value: torch.FloatTensor,
    lr: float = None,
    weight_decay: float = None,
) -> torch.FloatTensor:
    """p <- p - lr * (value * z + weight_decay * p) along z = N(0, 1) drawn from
    ``directional_derivative_seed``, for every parameter of every group in order
    (or p <- p - lr * value * z when the resolved weight_decay is None).

    lr / weight_decay default to the first group's values and then stick for every
    later group, exactly as the reference resolves them.  Parameters are updated in
    place on the GPU, and torch's generators are left where the reference's
    torch.manual_seed and draws leave them (the generator of the parameters' device past
    this seed's z).
    """
    torch.manual_seed(directional_derivative_seed)
    specs = codec.resolve_groups(param_groups, lr=lr, weight_decay=weight_decay)
    v, is_tensor = _value_kind(directional_derivative_value, specs)
    codec.directional_step(specs, [directional_derivative_seed], [v], value_is_tensor=is_tensor)
    codec.mark_rebound(p for g in param_groups for p in g["params"])  # zo_utils.py:49 rebinds param.data
    return directional_derivative_value


def reconstruct_(param_groups: List[dict], seeds: Sequence[int], values: Sequence[float], lr: float,
                 weight_decay: float) -> int:
    """The reconstruct loop of ClientTrainer.train_once (fedkseed.py:136-141) in one pass:
    for (seed, value) in order, skip exact zeros (NaN is applied, as in the reference),
    then directional_derivative_step(param_groups, seed, value, lr=lr, weight_decay=weight_decay).
    Returns the number of seeds applied."""
    keep = [(int(s), float(g)) for s, g in zip(seeds, values) if float(g) != 0.0]
    if not keep:
        return 0
    specs = codec.resolve_groups(param_groups, lr=lr, weight_decay=weight_decay)
    # the same list comes back every round (the arbiter's fixed seed candidates): keep the
    # jumped generator windows for the next reconstruct (codec.jwin_reserve, a speed cache).
    # torch's generators end where the last applied seed's draws leave them (codec._leave).
    codec.directional_step(specs, [s for s, _ in keep], [g for _, g in keep], value_is_tensor=False,
                           cache_windows=True)
    codec.mark_rebound(p for g in param_groups for p in g["params"])
    return len(keep)


def seed_shard_coefficients(values: Sequence[float], lr: float, weight_decay, rank: int = 0, world: int = 1):
    """Seed-sharded variant (BASELINE config C3): the K sequential steps
    p <- p - lr*(g_k*z_k + wd*p) of the reconstruct sum to
    p_K = a^K p_0 - sum_k lr g_k a^(K-1-k) z_k with a = 1 - lr*wd (a = 1 without the
    decay term).  Returns (first, last) -- the seed index range [first, last) rank
    ``rank`` of ``world`` accumulates, a contiguous 1/world of the K seeds -- the
    coefficients lr g_k a^(K-1-k) of that range (float64), and a^K.
    lr and wd enter as the fp32 values the reference's opmath sees."""
    import math

    import numpy as np

    k = len(values)
    first, last = k * rank // world, k * (rank + 1) // world
    lr32 = float(np.float32(lr))
    if weight_decay is None:
        log_a = 0.0
    else:
        log_a = math.log1p(-lr32 * float(np.float32(weight_decay)))
    coefs = [lr32 * float(values[i]) * math.exp((k - 1 - i) * log_a) for i in range(first, last)]
    return first, last, coefs, math.exp(k * log_a)


def reconstruct_seed_sharded_(param_groups: List[dict], seeds: Sequence[int], values: Sequence[float], lr: float,
                              weight_decay: float, process_group=None, delta: torch.Tensor = None) -> int:
    """The reconstruct of ClientTrainer.train_once as the north star's seed-sharded
    variant: every rank of ``process_group`` (torch.distributed, RCCL on MI355X) takes a
    contiguous 1/world of the non-zero seeds, accumulates its part of the f32 delta on
    its GPU, one all-reduce sums the parts, and every rank applies p = a^K p_0 - delta.

    NOT bit-equal to ``reconstruct_`` / the reference (which rounds every op of every
    seed to the parameter dtype): see DESIGN.md §7 for the measured deviation.  All
    tensors must share one (lr, wd) -- train_once passes them explicitly, so the sticky
    rule makes them uniform.  ``delta``: optional preallocated f32 buffer (the
    parameters' concatenation), zeroed here.  Returns the number of seeds applied."""
    import torch.distributed as dist

    keep = [(int(s), float(g)) for s, g in zip(seeds, values) if float(g) != 0.0]
    if not keep:
        return 0
    specs = codec.resolve_groups(param_groups, lr=lr, weight_decay=weight_decay)
    classes = {(sp.lr, sp.weight_decay) for sp in specs}
    if len(classes) != 1:
        raise ValueError("seed-sharded reconstruct needs one (lr, weight_decay) for every tensor")
    distributed = process_group is not None or (dist.is_available() and dist.is_initialized())
    rank = dist.get_rank(process_group) if distributed else 0
    world = dist.get_world_size(process_group) if distributed else 1
    sp0 = specs[0]
    first, last, coefs, decay = seed_shard_coefficients([g for _, g in keep], sp0.lr, sp0.weight_decay, rank, world)
    total = sum(sp.tensor.numel() for sp in specs)
    dev = sp0.tensor.device
    if delta is None:
        delta = torch.zeros(total, dtype=torch.float32, device=dev)
    else:
        delta.zero_()
    codec.delta_accumulate(specs, [s for s, _ in keep[first:last]], coefs, delta)
    if distributed:  # also at world size 1: the group's collective library sums (an identity)
        dist.all_reduce(delta, op=dist.ReduceOp.SUM, group=process_group)
    codec.delta_apply(specs, delta, [decay] * len(specs))
    codec.leave_generators(specs, keep[-1][0])  # where the reference's last seed leaves them
    return len(keep)


def build_seed_candidates(k, low=0, high=2**32):
    """K seed candidates drawn from the global torch generator."""
    return torch.randint(low, high, size=(k,), dtype=torch.long)


def get_even_seed_probabilities(k):
    """Uniform sampling probabilities 1/k."""
    return torch.ones(k) / k
