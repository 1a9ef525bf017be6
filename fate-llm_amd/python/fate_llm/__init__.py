"""fate_llm -- MI355X-native drop-in for FATE-LLM's FedKSeed path.

Only the FedKSeed subsystem (fate_llm.algo.fedkseed, fate_llm.runner.fedkseed_runner)
is provided; see DESIGN.md for scope.  Mirrors the package layout of the reference
(python/fate_llm/ in FATE-LLM 2.2.0).
"""
__version__ = "2.2.0+mi355x.1"
