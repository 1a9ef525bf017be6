"""Drop-in for python/fate_llm/algo/fedkseed/args.py (FATE-LLM 2.2.0)."""
from dataclasses import dataclass, field


@dataclass
class KSeedTrainingArguments:
    """FedKSeed / KSeedZO options (same fields and defaults as the reference).

    zo_optim: use KSeedZerothOrderOptimizer (suppresses `optim`).
    k: number of seed candidates.
    eps: perturbation scale of the two-point estimate.
    grad_clip: reject updates with |g| > grad_clip when positive.
    """

    zo_optim: bool = field(
        default=True,
        metadata={"help": "Whether to use KSeedZerothOrderOptimizer. This suppress `optim` argument when True."},
    )
    k: int = field(
        default=4096,
        metadata={"help": "The number of seed candidates to use. This suppress `seed_candidates` argument when > 1."},
    )
    eps: float = field(default=0.0005, metadata={"help": "Epsilon value for KSeedZerothOrderOptimizer."})
    grad_clip: float = field(default=-100.0, metadata={"help": "Gradient clip value for KSeedZerothOrderOptimizer."})
