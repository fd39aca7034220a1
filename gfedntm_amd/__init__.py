"""gfedntm_amd -- MI355X-native federated neural topic models.

ProdLDA / NeuralLDA (AVITM) and CombinedTM / ZeroShotTM (CTM) trained as a
federation of one client per GPU: the local minibatch step runs as fused
CDNA4 HIP kernels, and the per-round sample-weighted FedAvg is one RCCL
all-reduce over xGMI.  See README.md and SURVEY.md.
"""
__version__ = "0.1.0"
