from .dist import (DistContext, GradBucket, all_reduce_mean, barrier, broadcast_module, broadcast_parameters,
                   init_distributed,
                   shard_indices)

__all__ = ["DistContext", "GradBucket", "all_reduce_mean", "barrier", "broadcast_module", "broadcast_parameters", "init_distributed",
           "shard_indices"]
