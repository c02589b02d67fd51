"""Vertical federated learning: split-NN and VFL-VAE, single-process (reference semantics, see
``ddl25spring_amd.models.tabular``) and distributed one-party-per-rank (``splitnn``)."""
from ..models.tabular import (BottomModel, ClientDecoder, ClientEncoder, ServerVAE, TopModel,  # noqa: F401
                              VFLNetwork, VFLVAE, combined_loss)
from .splitnn import SplitNNParty, SplitNNServer, VAEParty, VAEServer  # noqa: F401
