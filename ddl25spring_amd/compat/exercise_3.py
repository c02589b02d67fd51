"""Names of ``lab/tutorial_2b/exercise_3.py`` (VFL-VAE): ``ClientEncoder`` (:10), ``ClientDecoder``
(:33), ``ServerVAE`` (:56), ``VFLVAE`` (:115), ``combined_loss`` (:140) — from ``models/tabular.py``
(fused MSE+KL ``loss.hip::ddl_mse_kl`` on the GPU). The distributed one-party-per-rank variant is
``vfl/splitnn.py::VAEParty`` / ``VAEServer``."""
from ..models.tabular import ClientDecoder, ClientEncoder, ServerVAE, VFLVAE, combined_loss  # noqa: F401

__all__ = ["ClientEncoder", "ClientDecoder", "ServerVAE", "VFLVAE", "combined_loss"]
