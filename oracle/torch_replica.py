"""The reference's reconstruct arithmetic re-typed with plain torch CPU calls.

TEST/BASELINE INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg).  It repeats the exact
torch calls of zo_utils.directional_derivative_step (python/fate_llm/algo/fedkseed/
zo_utils.py:42-52) -- torch.manual_seed, torch.normal on the CPU generator, and the
elementwise update expression -- so timing it on the GPU box's host measures the
reference's own CPU path without shipping the reference file.
"""
import torch


def directional_step(params, seed: int, g: float, lr: float, weight_decay):
    torch.manual_seed(seed)
    for p in params:
        z = torch.normal(mean=0, std=1, size=p.data.size(), device=p.data.device, dtype=p.data.dtype)
        if weight_decay is not None:  # zo_utils.py:48-49
            p.data = p.data - lr * (g * z + weight_decay * p.data)
        else:  # zo_utils.py:50-52
            p.data = p.data - lr * (g * z)


def reconstruct(params, seeds, scalars, lr: float, weight_decay: float) -> int:
    """ClientTrainer.train_once's loop (fedkseed.py:136-141); returns seeds applied."""
    n = 0
    for s, g in zip(seeds, scalars):
        if g != 0.0:
            directional_step(params, int(s), float(g), lr, weight_decay)
            n += 1
    return n
