"""Drop-in for python/fate_llm/algo/fedkseed/pytorch_utils.py (FATE-LLM 2.2.0).

The grouping defines the z-stream order: group 0 (no decay) tensors are drawn
first, then group 1, each in ``named_parameters`` order.
"""
from typing import List

from transformers.pytorch_utils import ALL_LAYERNORM_LAYERS
from transformers.trainer_pt_utils import get_parameter_names


def get_decay_parameter_names(model) -> List[str]:
    """Names of the parameters weight decay applies to: everything outside LayerNorm
    modules (isinstance check, so RMSNorm-style custom norms DO decay) except names
    containing "bias" -- the HF Trainer convention the reference follows."""
    return [name for name in get_parameter_names(model, ALL_LAYERNORM_LAYERS) if "bias" not in name]


def get_optimizer_parameters_grouped_with_decay(model, weight_decay: float) -> List[dict]:
    """[{params: no-decay, weight_decay: 0.0}, {params: decay, weight_decay: weight_decay}],
    trainable parameters only."""
    decay_names = set(get_decay_parameter_names(model))
    no_decay, decay = [], []
    for name, p in model.named_parameters():
        if not p.requires_grad:
            continue
        (decay if name in decay_names else no_decay).append(p)
    return [
        {"params": no_decay, "weight_decay": 0.0},
        {"params": decay, "weight_decay": weight_decay},
    ]
