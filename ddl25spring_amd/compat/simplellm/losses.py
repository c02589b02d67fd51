"""``simplellm.losses`` names (reference ``intro_DP_GA.py:4``); fused vocabulary CE kernel."""
from ...models.llama import causalLLMLoss  # noqa: F401

__all__ = ["causalLLMLoss"]
