from .networks import (DecoderNetwork, CTMDecoderNetwork, InferenceNetwork,
                       CombinedInferenceNetwork, ContextualInferenceNetwork)
from .avitm import AVITM
from .ctm import CTM, ZeroShotTM, CombinedTM

__all__ = ["DecoderNetwork", "CTMDecoderNetwork", "InferenceNetwork",
           "CombinedInferenceNetwork", "ContextualInferenceNetwork", "AVITM", "CTM",
           "ZeroShotTM", "CombinedTM"]
