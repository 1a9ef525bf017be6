"""Drop-in for python/fate_llm/runner/fedkseed_runner.py (FATE-LLM 2.2.0).

``FedKSeedRunner`` wires the FedKSeed arbiter (``Trainer``) and client
(``ClientTrainer``) from pipeline confs, as the reference runner does (:37-123):
same constructor, ``client_setup`` / ``server_setup`` and the ``fedkseed`` algo
check.  The reference subclasses FATE's ``DefaultRunner`` (fate.components), which
is not part of this build.  The only pieces of it this runner uses are restated
here:
* the context (``set_context`` / ``get_context``);
* the ``{"module_name", "item_name", "kwargs"}`` conf loader.

Pass a live FATE context (or any object with the same duck type) through
``set_context``.
"""
import importlib
import logging
from typing import Dict, Literal, Optional

from fate_llm.algo.fedkseed.fedkseed import ClientTrainer, FedKSeedTrainingArguments, Trainer
from fate_llm.algo.fedkseed.zo_utils import build_seed_candidates

logger = logging.getLogger(__name__)

SUPPORTED_ALGO = ["fedkseed"]


def loader_load_from_conf(conf: Optional[Dict]):
    """Instantiate ``module_name.item_name(**kwargs)`` (FATE's Loader conf format)."""
    if conf is None:
        return None
    module = importlib.import_module(conf["module_name"])
    item = getattr(module, conf["item_name"])
    kwargs = conf.get("kwargs", {}) or {}
    return item(**kwargs) if callable(item) else item


def maybe_loader_load_from_conf(conf):
    """Load a model from its conf; HF wrappers exposing ``load()`` are materialised."""
    model = loader_load_from_conf(conf)
    if model is not None and hasattr(model, "load") and not hasattr(model, "parameters"):
        model = model.load()
    return model


class FedKSeedRunner:
    def __init__(
        self,
        algo: str = "fedkseed",
        model_conf: Optional[Dict] = None,
        dataset_conf: Optional[Dict] = None,
        optimizer_conf: Optional[Dict] = None,
        training_args_conf: Optional[Dict] = None,
        fed_args_conf: Optional[Dict] = None,
        data_collator_conf: Optional[Dict] = None,
        tokenizer_conf: Optional[Dict] = None,
        task_type: Literal["causal_lm", "other"] = "causal_lm",
        local_mode: bool = False,
        save_trainable_weights_only: bool = False,
    ) -> None:
        self.algo = algo
        self.model_conf = model_conf
        self.dataset_conf = dataset_conf
        self.optimizer_conf = optimizer_conf
        self.training_args_conf = training_args_conf or {}
        self.fed_args_conf = fed_args_conf or {}
        self.data_collator_conf = data_collator_conf
        self.local_mode = local_mode
        self.tokenizer_conf = tokenizer_conf
        self.task_type = task_type
        self.save_trainable_weights_only = save_trainable_weights_only
        if self.algo not in SUPPORTED_ALGO:
            raise ValueError(f"algo should be one of {SUPPORTED_ALGO}")
        if self.task_type not in ["causal_lm", "others"]:
            raise ValueError("task_type should be one of [binary, multi, regression, others]")
        assert isinstance(self.local_mode, bool), "local should be bool"
        self.trainer = None
        self.training_args = None
        self._ctx = None

    # ---- the part of FATE's runner base this runner needs
    def set_context(self, ctx) -> None:
        self._ctx = ctx

    def get_context(self):
        if self._ctx is None:
            raise RuntimeError("FedKSeedRunner: no federation context; call set_context(ctx) first")
        return self._ctx

    @staticmethod
    def _training_args(conf: Dict, output_dir: Optional[str] = None):
        """FATE's Seq2SeqTrainingArguments (trainer/seq2seq_trainer.py: no checkpoints,
        constant lr, per-epoch logging, ...) as the reference runner builds them
        (fedkseed_runner.py:95,120); the client's output dir is set afterwards (:97)."""
        from fate_llm.trainer.seq2seq_trainer import Seq2SeqTrainingArguments

        args = Seq2SeqTrainingArguments(**conf)
        if output_dir is not None:
            args.output_dir = output_dir
        return args

    def client_setup(self, train_set=None, validate_set=None, output_dir=None, saved_model=None, stage="train"):
        if self.algo != "fedkseed":
            raise ValueError(f"algo {self.algo} not supported")
        import transformers

        ctx = self.get_context()
        model = maybe_loader_load_from_conf(self.model_conf)
        if model is None:
            raise ValueError(f"model is None, cannot load model from conf {self.model_conf}")
        tokenizer = transformers.AutoTokenizer.from_pretrained(**self.data_collator_conf["kwargs"]["tokenizer_params"])
        data_collator = transformers.DataCollatorForLanguageModeling(tokenizer=tokenizer, mlm=False)
        training_args = self._training_args(self.training_args_conf, output_dir or "./")
        self.training_args = training_args
        fedkseed_args = FedKSeedTrainingArguments(**self.fed_args_conf)
        logger.debug(f"training_args: {training_args}")
        logger.debug(f"fedkseed_args: {fedkseed_args}")
        return ClientTrainer(ctx=ctx, model=model, training_args=training_args, fedkseed_args=fedkseed_args,
                             data_collator=data_collator, tokenizer=tokenizer, train_dataset=train_set,
                             eval_dataset=validate_set)

    def server_setup(self, stage="train"):
        if self.algo != "fedkseed":
            raise ValueError(f"algo {self.algo} not supported")
        ctx = self.get_context()
        fedkseed_args = FedKSeedTrainingArguments(**self.fed_args_conf)
        training_args = self._training_args(self.training_args_conf)
        seed_candidates = build_seed_candidates(fedkseed_args.k, low=0, high=2**32)
        return Trainer(ctx=ctx, seed_candidates=seed_candidates, args=training_args, fedkseed_args=fedkseed_args)
