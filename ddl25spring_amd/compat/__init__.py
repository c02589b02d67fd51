"""Reference-API compatibility modules, one per reference module.

| reference module                              | here                                   |
|-----------------------------------------------|----------------------------------------|
| ``lab/tutorial_1a/hfl_complete.py``           | ``compat.hfl_complete``                |
| ``lab/tutorial_2a/centralized.py``            | ``compat.centralized``                 |
| ``lab/tutorial_2a/generative-modeling.py``    | ``compat.generative_modeling``         |
| ``lab/tutorial_2b/vfl.py`` / ``exercise_1,2`` | ``compat.vfl``                         |
| ``lab/tutorial_2b/exercise_3.py``             | ``compat.exercise_3``                  |
| external ``simplellm.{llama,tokenizers,dataloaders,losses}`` | ``compat.simplellm.*``  |

``install_aliases()`` registers them under the reference's own import names (``hfl_complete``,
``centralized``, ``vfl``, ``simplellm``, ``simplellm.llama``, ...) in ``sys.modules`` so the lab
scripts' import lines resolve to this framework without edits. Modules are imported lazily: nothing
here touches the GPU or the data at import time (Q11).
"""
from __future__ import annotations

import importlib
import sys

_ALIASES = {
    "hfl_complete": "hfl_complete",
    "centralized": "centralized",
    "generative_modeling": "generative_modeling",
    "vfl": "vfl",
    "exercise_3": "exercise_3",
    "simplellm": "simplellm",
    "simplellm.llama": "simplellm.llama",
    "simplellm.tokenizers": "simplellm.tokenizers",
    "simplellm.dataloaders": "simplellm.dataloaders",
    "simplellm.losses": "simplellm.losses",
}


def install_aliases(overwrite: bool = False) -> list[str]:
    """Make ``import simplellm.llama`` / ``from vfl import VFLNetwork`` / ... resolve here.

    Existing ``sys.modules`` entries are kept unless ``overwrite``. Returns the names installed."""
    done = []
    for name, sub in _ALIASES.items():
        if name in sys.modules and not overwrite:
            continue
        sys.modules[name] = importlib.import_module(f"{__name__}.{sub}")
        done.append(name)
    return done


__all__ = ["install_aliases"]
