"""Names of ``lab/tutorial_2b/vfl.py`` (and ``exercise_1.py`` / ``exercise_2.py``, which redefine
the same three classes): ``BottomModel`` (vfl.py:11), ``TopModel`` (:25), ``VFLNetwork`` (:43).

The classes are the framework's (``models/tabular.py``): fused ``tabular.hip`` layers on the GPU,
bottom models registered and ``zero_grad`` per batch by default; ``VFLNetwork(..., parity=True)``
reproduces the reference's quirks Q5/Q6/Q8. Data helpers for the heart table
(``data/heart.py``) are re-exported for the exercises' partitioning code.
"""
from ..data.heart import (centralized_split, load_heart, partition_balanced,  # noqa: F401
                          partition_random, partition_raw_columns, row_split, vfl_frame)
from ..models.tabular import BottomModel, TopModel, VFLNetwork  # noqa: F401

__all__ = ["BottomModel", "TopModel", "VFLNetwork", "load_heart", "vfl_frame", "row_split",
           "centralized_split", "partition_raw_columns", "partition_random", "partition_balanced"]
