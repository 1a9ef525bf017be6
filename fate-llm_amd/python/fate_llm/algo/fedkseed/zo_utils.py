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


def _value_kind(value):
    if isinstance(value, torch.Tensor):
        if value.dim() != 0:
            raise ValueError("directional_derivative_value must be a python number or a 0-dim tensor")
        return float(value.item()), True
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
    place on the GPU; ``torch.manual_seed`` is still called for its global side effect.
    """
    torch.manual_seed(directional_derivative_seed)
    specs = codec.resolve_groups(param_groups, lr=lr, weight_decay=weight_decay)
    v, is_tensor = _value_kind(directional_derivative_value)
    codec.directional_step(specs, [directional_derivative_seed], [v], value_is_tensor=is_tensor)
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
    codec.directional_step(specs, [s for s, _ in keep], [g for _, g in keep], value_is_tensor=False)
    torch.manual_seed(keep[-1][0])  # the global generator was last seeded with the last applied seed
    return len(keep)


def build_seed_candidates(k, low=0, high=2**32):
    """K seed candidates drawn from the global torch generator."""
    return torch.randint(low, high, size=(k,), dtype=torch.long)


def get_even_seed_probabilities(k):
    """Uniform sampling probabilities 1/k."""
    return torch.ones(k) / k
