"""Names of ``lab/tutorial_2a/centralized.py``: ``HeartDiseaseNN`` (:13) and the centralized
training loop (:40-75) as ``train_centralized`` (keeps a deep copy of the best weights — Q9)."""
from ..data.heart import centralized_split, load_heart  # noqa: F401
from ..models.tabular import HeartDiseaseNN, train_centralized  # noqa: F401

__all__ = ["HeartDiseaseNN", "train_centralized", "load_heart", "centralized_split"]
