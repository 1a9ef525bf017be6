"""Drop-in for python/fate_llm/algo/fedkseed/trainer.py (FATE-LLM 2.2.0).

``KSeedZOExtendedTrainer`` (reference :20-153) is a transformers ``Trainer`` whose
optimizer is ``KSeedZerothOrderOptimizer`` and whose ``training_step`` runs one
K-seed zeroth-order step (two closure forwards around the +-eps*z perturbations,
then the directional update) instead of backprop.  The perturbations and the update
run on the MI355X codec through the optimizer; this class only wires it into the
HF training loop.

The reference pins transformers 4.37.2 (python/setup.py:35), whose ``Trainer`` takes
``tokenizer=`` and calls ``training_step(model, inputs)``; 5.x renamed the keyword to
``processing_class=`` and passes ``num_items_in_batch``.  The constructor keeps the
reference's ``tokenizer`` keyword and forwards it under whichever name the installed
``Trainer`` accepts; ``training_step`` takes both call forms.
"""
import inspect
import logging
from typing import Any, Callable, Dict, List, Optional, Tuple, Union

import torch
from torch import nn
from transformers import Trainer, TrainingArguments
from transformers.optimization import SchedulerType, get_scheduler

from .args import KSeedTrainingArguments
from .optimizer import KSeedZerothOrderOptimizer
from .pytorch_utils import get_optimizer_parameters_grouped_with_decay

logger = logging.getLogger(__name__)

# the keyword the installed transformers.Trainer takes the tokenizer under
_TOKENIZER_KW = "processing_class" if "processing_class" in inspect.signature(Trainer.__init__).parameters \
    else "tokenizer"
_STEP_TAKES_NUM_ITEMS = "num_items_in_batch" in inspect.signature(Trainer.training_step).parameters


class KSeedZOExtendedTrainer(Trainer):
    def __init__(
        self,
        model: Optional[nn.Module] = None,
        training_args: Optional[TrainingArguments] = None,
        kseed_args: Optional[KSeedTrainingArguments] = None,
        data_collator=None,
        train_dataset=None,
        eval_dataset=None,
        tokenizer=None,
        model_init: Optional[Callable] = None,
        compute_metrics: Optional[Callable] = None,
        callbacks: Optional[List] = None,
        optimizers: Tuple[Optional[torch.optim.Optimizer], Optional[Any]] = (None, None),
        preprocess_logits_for_metrics: Optional[Callable] = None,
    ):
        kw = dict(model=model, args=training_args, data_collator=data_collator, train_dataset=train_dataset,
                  eval_dataset=eval_dataset, model_init=model_init, compute_metrics=compute_metrics,
                  callbacks=callbacks, optimizers=optimizers,
                  preprocess_logits_for_metrics=preprocess_logits_for_metrics)
        kw[_TOKENIZER_KW] = tokenizer
        super().__init__(**kw)
        self.kseed_args = kseed_args
        self._kseed_optimizer: Optional[KSeedZerothOrderOptimizer] = None
        self._seed_candidates = None
        self._seed_probabilities = None

    def configure_seed_candidates(self, seed_candidates: torch.LongTensor, seed_probabilities: torch.FloatTensor):
        self._seed_candidates = seed_candidates
        self._seed_probabilities = seed_probabilities

    def get_directional_derivative_history(self):
        """{seed: [g, ...]} recorded by the optimizer during training."""
        if not self.k_seed_zo_mode(self.kseed_args) or self._kseed_optimizer is None:
            raise ValueError("KSeedZerothOrderOptimizer is not configured")
        return self._kseed_optimizer.directional_derivative_history

    @staticmethod
    def k_seed_zo_mode(args) -> bool:
        return bool(getattr(args, "zo_optim", False))

    def training_step(self, model: nn.Module, inputs: Dict[str, Union[torch.Tensor, Any]],
                      num_items_in_batch=None) -> torch.Tensor:
        """One KSeedZO step: loss = closure at x+eps*z (the reference returns loss_right).

        As in the reference (trainer.py:85-90) the closure is only DEFINED inside
        compute_loss_context_manager(); it runs outside it, under torch.no_grad()."""
        if not self.k_seed_zo_mode(self.kseed_args):
            if _STEP_TAKES_NUM_ITEMS:
                return super().training_step(model, inputs, num_items_in_batch)
            return super().training_step(model, inputs)
        if self._kseed_optimizer is None:
            raise ValueError("KSeedZerothOrderOptimizer is not configured")
        model.eval()
        inputs = self._prepare_inputs(inputs)

        with self.compute_loss_context_manager():
            def closure() -> torch.FloatTensor:
                with torch.no_grad():
                    return self.compute_loss(model, inputs, return_outputs=False).detach()

        with torch.no_grad():
            loss = self._kseed_optimizer.kseed_zeroth_order_step(closure=closure)
        return loss.detach() if isinstance(loss, torch.Tensor) else torch.tensor(loss)

    def create_optimizer_and_scheduler(self, num_training_steps: int):
        """The reference's hook (trainer.py:101-132; transformers 4.37 calls it)."""
        if not self.k_seed_zo_mode(self.kseed_args):
            return super().create_optimizer_and_scheduler(num_training_steps)
        self.create_optimizer()
        self.create_scheduler(num_training_steps, self.optimizer)

    # transformers 5.x calls these two directly instead of create_optimizer_and_scheduler
    def create_optimizer(self, model=None):
        if not self.k_seed_zo_mode(self.kseed_args):
            return super().create_optimizer(model) if model is not None else super().create_optimizer()
        if self._kseed_optimizer is not None:
            return self.optimizer
        if self._seed_candidates is None or self._seed_probabilities is None:
            raise ValueError("Seed candidates and probabilities are not configured.")
        groups = get_optimizer_parameters_grouped_with_decay(self.model, self.args.weight_decay)
        self.optimizer = KSeedZerothOrderOptimizer(
            groups, seed_candidates=self._seed_candidates, seed_probabilities=self._seed_probabilities,
            lr=self.args.learning_rate, eps=self.kseed_args.eps, weight_decay=self.args.weight_decay,
            grad_clip=self.kseed_args.grad_clip)
        self._kseed_optimizer = self.optimizer
        return self.optimizer

    def create_scheduler(self, num_training_steps: int, optimizer=None):
        if not self.k_seed_zo_mode(self.kseed_args):
            return super().create_scheduler(num_training_steps, optimizer)
        # constant schedule: the aggregated update replays each seed with the base lr
        self.lr_scheduler = get_scheduler(name=SchedulerType.CONSTANT, optimizer=optimizer or self.optimizer,
                                          num_warmup_steps=self.args.warmup_steps,
                                          num_training_steps=num_training_steps)
        return self.lr_scheduler
