"""Tensor primitives of NC-Net: HIP kernels on GPU, PyTorch oracles on CPU."""
from . import reference
from ._ext import available as hip_available
from .conv4d import Conv4d, conv4d
from .correlation import correlation, correlation_pool2, l2norm_pack, maxpool4d
from .loss import match_score, weak_loss_from_corr
from .mutual import mutual_matching
from .neigh_consensus import neigh_consensus

__all__ = ["reference", "hip_available", "Conv4d", "conv4d", "correlation", "correlation_pool2", "l2norm_pack",
           "maxpool4d", "match_score", "weak_loss_from_corr", "mutual_matching", "neigh_consensus"]
