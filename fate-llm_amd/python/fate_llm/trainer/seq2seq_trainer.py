"""Drop-in for the training-argument classes of python/fate_llm/trainer/seq2seq_trainer.py
(FATE-LLM 2.2.0): the arguments FedKSeedRunner builds its ClientTrainer and arbiter
Trainer from (runner/fedkseed_runner.py:95,120).

FATE changes a handful of HF defaults (seq2seq_trainer.py:42-58): no checkpoints, a
constant learning rate, per-epoch logging, no tqdm, info-level logs, no safetensors,
pipeline-controlled output dir; and it switches the hub off (:60-70).  Those defaults
matter off the ZO path too (checkpoint saving, logging, ``zo_optim=False`` training), so
the drop-in runner takes its arguments from here, not from transformers directly.

The federated HF trainer of that module (HomoSeq2SeqTrainerClient, fate.ml's
HomoTrainerMixin) is FATE federation plumbing and out of scope.
"""
import copy
from dataclasses import dataclass, field
from typing import Optional

from transformers import Seq2SeqTrainingArguments as _HFSeq2SeqTrainingArguments


@dataclass
class _S2STrainingArguments(_HFSeq2SeqTrainingArguments):
    """HF Seq2SeqTrainingArguments with FATE's defaults."""

    output_dir: str = field(default="./")  # the pipeline sets the real one
    disable_tqdm: bool = field(default=True)
    save_strategy: str = field(default="no")
    logging_strategy: str = field(default="epoch")
    logging_steps: int = field(default=1)
    evaluation_strategy: str = field(default="no")
    logging_dir: str = field(default=None)
    checkpoint_idx: int = field(default=None)
    lr_scheduler_type: str = field(default="constant")  # FATE-1.x behaviour
    log_level: str = field(default="info")
    deepspeed: Optional[str] = field(default=None)
    save_safetensors: bool = field(default=False)
    use_cpu: bool = field(default=False)

    def __post_init__(self):
        # never push to a hub from a federation party
        self.push_to_hub = False
        self.hub_model_id = None
        self.hub_strategy = "every_save"
        self.hub_token = None
        self.hub_private_repo = False
        self.push_to_hub_model_id = None
        self.push_to_hub_organization = None
        self.push_to_hub_token = None
        super().__post_init__()


DEFAULT_ARGS = _S2STrainingArguments().to_dict()


@dataclass
class Seq2SeqTrainingArguments(_S2STrainingArguments):
    """FATE's arguments; ``to_dict`` lists only what differs from FATE's defaults."""

    def to_dict(self):
        defaults = copy.deepcopy(DEFAULT_ARGS)
        return {k: v for k, v in super().to_dict().items() if v != defaults.get(k)}
