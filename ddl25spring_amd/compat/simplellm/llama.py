"""``simplellm.llama`` names (reference ``intro_DP_GA.py:1``, ``intro_PP_1F1B_MB.py:1``)."""
from ...models.llama import CausalLLama, LLama, LLamaFirstStage, LLamaLastStage, LLamaStage  # noqa: F401

__all__ = ["CausalLLama", "LLama", "LLamaFirstStage", "LLamaStage", "LLamaLastStage"]
