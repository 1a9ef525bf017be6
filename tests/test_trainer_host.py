"""KSeedZOExtendedTrainer (trainer.py) on the CPU: construction on a locally built tiny
GPT-2 (no download) under the installed transformers, the tokenizer keyword shim
(4.37's ``tokenizer=`` / 5.x's ``processing_class=``), the optimizer/scheduler hook
and the non-ZO training_step fallback.  The ZO training_step runs on the GPU
(tests/test_gpu_trainer.py)."""
import inspect

import pytest
import torch

transformers = pytest.importorskip("transformers")

from fate_llm.algo.fedkseed import trainer as T  # noqa: E402
from fate_llm.algo.fedkseed.args import KSeedTrainingArguments  # noqa: E402
from fate_llm.algo.fedkseed.optimizer import KSeedZerothOrderOptimizer  # noqa: E402


def tiny_gpt2():
    cfg = transformers.GPT2Config(n_embd=32, n_layer=2, n_head=2, vocab_size=64, n_positions=32)
    torch.manual_seed(0)
    return transformers.GPT2LMHeadModel(cfg)


class Toks(torch.utils.data.Dataset):
    def __init__(self, n=8, length=12):
        g = torch.Generator().manual_seed(1)
        self.x = torch.randint(0, 64, (n, length), generator=g)

    def __len__(self):
        return len(self.x)

    def __getitem__(self, i):
        return {"input_ids": self.x[i], "labels": self.x[i].clone()}


def targs(tmp_path, **kw):
    base = dict(output_dir=str(tmp_path), per_device_train_batch_size=2, max_steps=2, learning_rate=1e-5,
                weight_decay=0.0, report_to=[], save_strategy="no", logging_strategy="no", use_cpu=True,
                max_grad_norm=0.0)
    base.update(kw)
    return transformers.TrainingArguments(**base)


def test_tokenizer_keyword_matches_installed_trainer():
    params = inspect.signature(transformers.Trainer.__init__).parameters
    assert T._TOKENIZER_KW in params
    assert T._TOKENIZER_KW == ("processing_class" if "processing_class" in params else "tokenizer")


def test_construct_and_optimizer_hook(tmp_path):
    model = tiny_gpt2()
    tr = T.KSeedZOExtendedTrainer(model=model, training_args=targs(tmp_path), kseed_args=KSeedTrainingArguments(),
                                  train_dataset=Toks(), tokenizer=None)
    assert tr.k_seed_zo_mode(tr.kseed_args)
    with pytest.raises(ValueError):
        tr.create_optimizer_and_scheduler(2)  # seeds not configured yet
    tr.configure_seed_candidates(torch.arange(16) * 7919, torch.ones(16) / 16)
    tr.create_optimizer_and_scheduler(2)
    assert isinstance(tr.optimizer, KSeedZerothOrderOptimizer)
    names = {id(p): n for n, p in model.named_parameters()}
    no_decay = [names[id(p)] for p in tr.optimizer.param_groups[0]["params"]]
    assert no_decay and all(("bias" in n) or ("ln" in n) for n in no_decay)
    assert tr.get_directional_derivative_history() == {int(s): [] for s in torch.arange(16) * 7919}


def test_non_zo_mode_trains_with_backprop(tmp_path):
    model = tiny_gpt2()
    before = model.transformer.h[0].attn.c_attn.weight.detach().clone()
    tr = T.KSeedZOExtendedTrainer(model=model, training_args=targs(tmp_path, learning_rate=1e-2),
                                  kseed_args=KSeedTrainingArguments(zo_optim=False), train_dataset=Toks(),
                                  tokenizer=None)
    tr.train()
    assert not torch.equal(before, model.transformer.h[0].attn.c_attn.weight.detach())
    with pytest.raises(ValueError):
        tr.get_directional_derivative_history()
