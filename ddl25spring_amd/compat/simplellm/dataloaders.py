"""``simplellm.dataloaders`` names (reference ``intro_DP_GA.py:3``); synthetic TinyStories stream."""
from ...data.text import TinyStories  # noqa: F401

__all__ = ["TinyStories"]
