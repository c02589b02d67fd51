"""``simplellm.tokenizers`` names (reference ``intro_DP_GA.py:2``)."""
from ...data.text import SPTokenizer  # noqa: F401

__all__ = ["SPTokenizer"]
