"""ncnet_amd: an MI355X-native Neighbourhood Consensus Network framework.

Layers:
  ncnet_amd.ops       HIP-kernel-backed tensor primitives (+ PyTorch oracles)
  ncnet_amd.models    backbones, Conv4d, NeighConsensus, ImMatchNet
  ncnet_amd.data      pair datasets, transforms, synthetic pairs
  ncnet_amd.parallel  RCCL data parallelism
  ncnet_amd.engine    trainer, checkpoints, reference-algorithm baseline
  ncnet_amd.eval      match extraction, PCK, InLoc export
"""
__version__ = "0.1.0"
