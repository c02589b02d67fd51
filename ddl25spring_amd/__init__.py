"""ddl25spring_amd — an MI355X-native distributed & federated learning lab framework.

Capabilities of the DDL25Spring course labs (horizontal FL: FedSGD/FedAvg + robust aggregation,
vertical FL split-NN / VFL-VAE, tabular VAE, DP/PP/DPxPP LLaMA training) built on hand-written
CDNA4 HIP kernels, a C++ host runtime and RCCL collectives over xGMI.
"""
__version__ = "0.1.0"
