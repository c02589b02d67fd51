"""Drop-in for the external ``simplellm`` package the tutorial_1b DP/PP scripts import.

Reference imports (``lab/tutorial_1b/DP/*/intro_DP_*.py:1-4``, ``PP/*/intro_PP_*.py:1-10``)::

    from simplellm.llama import CausalLLama, LLama, LLamaFirstStage, LLamaStage, LLamaLastStage
    from simplellm.tokenizers import SPTokenizer
    from simplellm.dataloaders import TinyStories
    from simplellm.losses import causalLLMLoss

Each submodule re-exports the MI355X-native implementation (``models/llama.py`` on the
``llama.hip`` kernels, ``data/text.py``). ``ddl25spring_amd.compat.install_aliases()`` registers
this package as top-level ``simplellm`` so those scripts run unchanged. The architecture internals
of the external package are not available here (no network): parity unpinned, see docs/PARITY.md M8.
"""
from . import dataloaders, llama, losses, tokenizers  # noqa: F401
