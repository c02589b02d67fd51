"""Names of ``lab/tutorial_2a/generative-modeling.py`` (the file name is not importable as-is):
``Autoencoder`` (:13, ``train_with_settings`` / ``sample`` — Q10 batch-posterior sampling kept) and
``customLoss`` (:121, MSE(sum)+KL, fused ``loss.hip::ddl_mse_kl`` kernel on the GPU)."""
from ..models.tabular import Autoencoder, customLoss  # noqa: F401

__all__ = ["Autoencoder", "customLoss"]
