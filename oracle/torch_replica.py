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


def random_perturb_parameters(param_groups, seed: int, scaling_factor: float):
    """ZerothOrderOptimizer.random_perturb_parameters (optimizer.py:165-173)."""
    torch.manual_seed(seed)
    for group in param_groups:
        eps = group["eps"]
        for p in group["params"]:
            if p.requires_grad:
                z = torch.normal(mean=0, std=1, size=p.data.size(), device=p.data.device, dtype=p.data.dtype)
                p.data = p.data + scaling_factor * eps * z


def directional_derivative_step(param_groups, seed: int, value, lr=None, weight_decay=None):
    """zo_utils.directional_derivative_step (zo_utils.py:42-54), sticky lr / weight decay."""
    torch.manual_seed(seed)
    for group in param_groups:
        weight_decay = group["weight_decay"] if weight_decay is None else weight_decay
        lr = group["lr"] if lr is None else lr
        for p in group["params"]:
            z = torch.normal(mean=0, std=1, size=p.data.size(), device=p.data.device, dtype=p.data.dtype)
            if weight_decay is not None:
                p.data = p.data - lr * (value * z + weight_decay * p.data)
            else:
                p.data = p.data - lr * (value * z)
    return value


def zeroth_order_step(param_groups, seed: int, closure, eps: float, grad_clip: float = 0.0):
    """ZerothOrderOptimizer.zeroth_order_step (optimizer.py:127-150) with
    RandomWalkOptimizer.directional_derivative_step's clip (:84-92)."""
    random_perturb_parameters(param_groups, seed, 1.0)
    loss_right = closure()
    random_perturb_parameters(param_groups, seed, -2.0)
    loss_left = closure()
    random_perturb_parameters(param_groups, seed, 1.0)
    if torch.isnan(loss_right):
        return loss_right, loss_right, loss_left
    if torch.isnan(loss_left):
        return loss_left, loss_right, loss_left
    g = (loss_right - loss_left) / (2 * eps)
    if grad_clip > 0.0 and abs(g) > grad_clip:
        return torch.FloatTensor([torch.nan]), loss_right, loss_left
    directional_derivative_step(param_groups, seed, g)
    return g, loss_right, loss_left
