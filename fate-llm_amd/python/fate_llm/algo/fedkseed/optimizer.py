"""Drop-in for python/fate_llm/algo/fedkseed/optimizer.py (FATE-LLM 2.2.0).

MeZO-style zeroth-order optimizers with the K-seed sampler of FedKSeed.  Class
names, constructor arguments, methods and return conventions follow the reference
(RandomWalkOptimizer :55-99, ZerothOrderOptimizer :102-173,
KSeedZerothOrderOptimizer :176-235).  The two N-sized operations -- the +-eps*z
perturbations and the directional update -- run on the MI355X codec.
"""
import math
from typing import Callable, List, Mapping, Optional, Tuple

import torch
from torch.optim import Optimizer

from . import codec
from .pytorch_utils import get_optimizer_parameters_grouped_with_decay
from .zo_utils import _value_kind, directional_derivative_step


class RandomWalkOptimizer(Optimizer):
    """Updates parameters along a seeded random direction (no gradients)."""

    def __init__(self, params, lr, weight_decay, grad_clip, defaults=None):
        self.lr = lr
        self.weight_decay = weight_decay
        self.grad_clip = grad_clip
        merged = dict(defaults) if defaults is not None else {}
        merged.update(lr=lr, weight_decay=weight_decay)
        super().__init__(params, merged)

    @classmethod
    def from_model(cls, model, lr, weight_decay, grad_clip, **kwargs):
        groups = get_optimizer_parameters_grouped_with_decay(model, weight_decay)
        kwargs.update(lr=lr, weight_decay=weight_decay, grad_clip=grad_clip)
        return cls(groups, **kwargs)

    def directional_derivative_step(
        self, directional_derivative_seed: int, directional_derivative_value: torch.FloatTensor
    ) -> torch.FloatTensor:
        """Apply the update unless |value| exceeds a positive grad_clip (then NaN, no update)."""
        if self.grad_clip > 0.0 and abs(directional_derivative_value) > self.grad_clip:
            return torch.FloatTensor([torch.nan])
        directional_derivative_step(self.param_groups, directional_derivative_seed, directional_derivative_value)
        return directional_derivative_value

    def step(self, closure: Optional[Callable[[], float]] = None) -> Optional[float]:
        raise NotImplementedError(
            "use random_step instead of step for RandomWalkOptimizer "
            "since we need pass the `seed` and `grad_projected_value`"
        )


class ZerothOrderOptimizer(RandomWalkOptimizer):
    """Two-point (SPSA / MeZO) estimate of the directional derivative along z."""

    # device_step: when the losses are device tensors on the parameters' device and the
    # restore and update walk the same tensors, g, the NaN checks and the clip decision
    # stay on the device and the fused restore + update reads them there
    # (codec.perturb_step_device): no host synchronisation inside zeroth_order_step
    device_step = True

    def __init__(self, params, lr, eps, weight_decay, grad_clip):
        self.eps = eps
        self._last_step_on_device = False
        super().__init__(params, lr, weight_decay, grad_clip, dict(eps=eps))

    def zeroth_order_step(
        self, directional_derivative_seed: int, closure: Callable[[], torch.FloatTensor]
    ) -> Tuple[torch.FloatTensor, torch.FloatTensor, torch.FloatTensor]:
        """x+eps*z -> loss_right; x-eps*z -> loss_left; back to x; then the update with
        g = (loss_right - loss_left) / (2 eps).  Returns (g, loss_right, loss_left); a NaN
        loss short-circuits before the update, as in the reference (optimizer.py:108-150).

        The restore perturbation and the update use the same z, so when they walk the
        same tensors (every grouped parameter requires grad) they run as ONE device pass
        (codec.perturb_step); the values are those of the two separate steps."""
        self.random_perturb_parameters(directional_derivative_seed, scaling_factor=1.0)
        loss_right = closure()
        self.random_perturb_parameters(directional_derivative_seed, scaling_factor=-2.0)
        loss_left = closure()

        self._last_step_on_device = self._on_device(loss_right, loss_left)
        if self._last_step_on_device:
            return self._device_tail(directional_derivative_seed, loss_right, loss_left)
        right_nan, left_nan = bool(torch.isnan(loss_right)), bool(torch.isnan(loss_left))
        if right_nan or left_nan:
            self.random_perturb_parameters(directional_derivative_seed, scaling_factor=1.0)
            return (loss_right if right_nan else loss_left), loss_right, loss_left

        g = (loss_right - loss_left) / (2 * self.eps)
        clipped = self.grad_clip > 0.0 and abs(g) > self.grad_clip
        if clipped or not self._fusable():
            self.random_perturb_parameters(directional_derivative_seed, scaling_factor=1.0)
            g = self.directional_derivative_step(directional_derivative_seed, g)
            return g, loss_right, loss_left
        specs = codec.resolve_groups(self.param_groups)
        try:
            # the same value rules as the unfused directional step (a g that would rebind
            # param.data to another dtype or shape is rejected), checked before any update
            v, is_tensor = _value_kind(g, specs)
        except NotImplementedError:
            self.random_perturb_parameters(directional_derivative_seed, scaling_factor=1.0)
            raise
        torch.manual_seed(directional_derivative_seed)
        scales = [1.0 * group["eps"] for group in self.param_groups for _ in group["params"]]
        codec.perturb_step(specs, directional_derivative_seed, scales, v, value_is_tensor=is_tensor, update=True)
        codec.mark_rebound(p for group in self.param_groups for p in group["params"])
        return g, loss_right, loss_left

    # loss dtypes whose g reaches the kernels exactly as an f32 (then rounded to each
    # parameter's dtype there, as the host path's 0-dim tensor value is)
    _DEVICE_LOSS_DTYPES = (torch.float32, torch.bfloat16, torch.float16)

    def _on_device(self, loss_right, loss_left) -> bool:
        """The device tail takes exactly the losses the host path treats as a 0-dim tensor
        value (zo_utils._value_kind): 0-dim f32 / bf16 / f16 tensors on the parameters'
        device.  Anything else (a shape-(1,) loss, an f64 loss) goes through the host
        path, which accepts and rejects the same inputs as the reference."""
        if not (self.device_step and self._fusable()):
            return False
        dev = next((p.device for group in self.param_groups for p in group["params"]), None)
        return (dev is not None and dev.type == "cuda" and all(
            isinstance(x, torch.Tensor) and x.device == dev and x.dim() == 0 and x.dtype in self._DEVICE_LOSS_DTYPES
            for x in (loss_right, loss_left)))

    def _device_tail(self, seed, loss_right, loss_left):
        """optimizer.py:136-148 without leaving the device: g = (loss_right - loss_left) /
        (2 eps) as the reference computes it; the update applies unless a loss is NaN or a
        positive grad_clip is exceeded; the restore perturbation always.  The returned g is
        NaN where the reference returns a NaN tensor (a NaN loss or a clipped g)."""
        g = (loss_right - loss_left) / (2 * self.eps)
        ok = ~(torch.isnan(loss_right) | torch.isnan(loss_left))
        if self.grad_clip > 0.0:
            ok = ok & ~(torch.abs(g) > self.grad_clip)
        torch.manual_seed(seed)
        specs = codec.resolve_groups(self.param_groups)
        scales = [1.0 * group["eps"] for group in self.param_groups for _ in group["params"]]
        codec.perturb_step_device(specs, seed, scales, g, ok)
        codec.mark_rebound(p for group in self.param_groups for p in group["params"])
        return torch.where(ok, g, torch.full_like(g, math.nan)), loss_right, loss_left

    def _fusable(self) -> bool:
        """restore and update walk the same tensors: no frozen parameter in the groups"""
        return all(p.requires_grad for group in self.param_groups for p in group["params"])

    def random_perturb_parameters(self, directional_derivative_seed: int, scaling_factor: float):
        """p <- p + scaling_factor*eps*z for every parameter that requires grad; frozen
        parameters draw no z (their stream slot is skipped, as in the reference)."""
        torch.manual_seed(directional_derivative_seed)
        tensors, scales, params = [], [], []
        for group in self.param_groups:
            scale = scaling_factor * group["eps"]  # python double, cast to fp32 at the multiply
            for p in group["params"]:
                if p.requires_grad:
                    tensors.append(p.data)
                    scales.append(scale)
                    params.append(p)
        codec.perturb(tensors, directional_derivative_seed, scales, fresh=[codec.is_rebound(p) for p in params])
        codec.mark_rebound(params)  # optimizer.py:173 rebinds param.data


class KSeedZerothOrderOptimizer(ZerothOrderOptimizer):
    """Zeroth-order optimizer that samples its direction seed from K candidates and
    records the directional derivative observed for each seed."""

    def __init__(self, params, seed_candidates: torch.LongTensor, seed_probabilities: torch.FloatTensor,
                 lr, eps, weight_decay, grad_clip):
        self.seed_candidate = seed_candidates
        self.seed_probabilities = seed_probabilities
        self._pending = []  # (seed, device g) of device-side steps, not yet in the history
        self.directional_derivative_history: Mapping[int, List[float]] = {s.item(): [] for s in seed_candidates}
        self.sample_random_generator = torch.Generator()  # unseeded, as in the reference (optimizer.py:190)
        super().__init__(params, lr, eps, weight_decay, grad_clip)

    @property
    def directional_derivative_history(self) -> Mapping[int, List[float]]:
        """seed -> the g values recorded for it, in step order (optimizer.py:189, :233).
        Device-side steps record g lazily: reading the history brings every pending g to
        the host in one transfer (one synchronisation per read, none per step)."""
        if self._pending:
            pend, self._pending = self._pending, []
            vals = torch.stack([g.reshape(()) for _, g in pend]).tolist()
            for (seed, _), v in zip(pend, vals):
                if not math.isnan(v):
                    self._history[seed].append(v)
        return self._history

    @directional_derivative_history.setter
    def directional_derivative_history(self, value) -> None:
        self._pending = []
        self._history = value

    def sample(self) -> int:
        idx = torch.multinomial(input=self.seed_probabilities, num_samples=1,
                                generator=self.sample_random_generator)[0].item()
        return self.seed_candidate[idx].item()

    def step(self, closure: Callable[[], torch.FloatTensor] = None) -> torch.FloatTensor:
        if closure is None:
            # HF Trainer calls step() without a closure after training_step; no-op (NaN)
            return torch.FloatTensor([torch.nan])
        return self.kseed_zeroth_order_step(closure)

    def kseed_zeroth_order_step(self, closure: Callable[[], torch.FloatTensor]) -> torch.FloatTensor:
        """Sample a seed, run the zeroth-order step, record g for that seed; returns loss_right."""
        if closure is None:
            raise ValueError("closure must not be None")
        seed = self.sample()
        g, loss_right, loss_left = self.zeroth_order_step(seed, closure)
        if self._last_step_on_device:
            # g stays on the device: recorded when the history is read; the returned value
            # is g where it is NaN, else loss_right (optimizer.py:229-235), as a device tensor
            self._pending.append((seed, g))
            return torch.where(torch.isnan(g), g, loss_right)
        if math.isnan(g):
            return g
        self.directional_derivative_history[seed].append(g.item())
        return loss_right
