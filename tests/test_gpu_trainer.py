"""KSeedZOExtendedTrainer.training_step end to end on the GPU (trainer.py:74-99 of the
reference): a locally built tiny GPT-2 (fp32, no download) trained for a few steps by the
HF training loop with the K-seed ZO optimizer; every step's sampled seed and recorded g
are replayed through the oracle -- perturb +eps, -2 eps, +eps, then the update with the
sticky group-0 lr / weight decay (zo_utils.py:44-45) -- and the model's final
parameters must equal the replay bit for bit."""
import pytest
import torch

from conftest import assert_bitwise
from oracle import fks_oracle as O
from test_gpu_parity import _dev, to_np
from test_trainer_host import Toks, tiny_gpt2

transformers = pytest.importorskip("transformers")
pytestmark = pytest.mark.gpu


def test_training_step_replays_through_oracle(tmp_path):
    from fate_llm.algo.fedkseed import optimizer as OPT
    from fate_llm.algo.fedkseed import trainer as T
    from fate_llm.algo.fedkseed.args import KSeedTrainingArguments
    _dev()
    model = tiny_gpt2()
    args = transformers.TrainingArguments(
        output_dir=str(tmp_path), per_device_train_batch_size=2, max_steps=4, learning_rate=1e-3, weight_decay=0.01,
        report_to=[], save_strategy="no", logging_strategy="no", max_grad_norm=0.0, dataloader_num_workers=0)
    kargs = KSeedTrainingArguments(zo_optim=True, eps=5e-4, grad_clip=-100.0)
    tr = T.KSeedZOExtendedTrainer(model=model, training_args=args, kseed_args=kargs, train_dataset=Toks(),
                                  tokenizer=None)
    cands = torch.arange(1, 17) * 104729
    tr.configure_seed_candidates(cands, torch.ones(16) / 16)
    groups = None
    init = None
    sampled = []
    orig_sample = OPT.KSeedZerothOrderOptimizer.sample

    def sample(self):
        nonlocal groups, init
        if init is None:  # first step: the optimizer's groups, in z-stream order, before any update
            groups = self.param_groups
            init = [to_np(p.data) for g in groups for p in g["params"]]
        s = orig_sample(self)
        sampled.append(s)
        return s

    OPT.KSeedZerothOrderOptimizer.sample = sample
    try:
        tr.train()
    finally:
        OPT.KSeedZerothOrderOptimizer.sample = orig_sample
    torch.cuda.synchronize()
    assert len(sampled) == 4
    hist = tr.get_directional_derivative_history()
    gs = {s: list(v) for s, v in hist.items()}
    arrays = [a.copy() for a in init]
    n = len(arrays)
    eps = 5e-4
    for s in sampled:
        for sf in (1.0, -2.0, 1.0):
            O.perturb_params(arrays, [O.F32] * n, s, sf * eps)
        g = gs[s].pop(0)
        # sticky rule: group 0's lr and weight decay (0.0) for every tensor
        O.reconstruct(arrays, [O.F32] * n, [1e-3] * n, [0.0] * n, [s], [g])
    final = [to_np(p.data) for g in groups for p in g["params"]]
    for i, (got, want) in enumerate(zip(final, arrays)):
        assert_bitwise(got.reshape(-1), want.reshape(-1), "float32", f"param {i}")
