from .backbones import build_trunk, fold_frozen_bn
from .immatchnet import (FeatureCorrelation, FeatureExtraction, ImMatchNet, MutualMatching, NeighConsensus,
                         featureL2Norm, maxpool4d)

__all__ = ["build_trunk", "fold_frozen_bn", "FeatureCorrelation", "FeatureExtraction", "ImMatchNet",
           "MutualMatching", "NeighConsensus", "featureL2Norm", "maxpool4d"]
