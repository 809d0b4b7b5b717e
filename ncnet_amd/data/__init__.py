from .datasets import ImagePairDataset, PFPascalDataset, SyntheticPairDataset, synthetic_batch
from .transforms import AffineTnf, NormalizeImageDict, normalize_image, resize_bilinear

__all__ = ["ImagePairDataset", "PFPascalDataset", "SyntheticPairDataset", "synthetic_batch", "AffineTnf",
           "NormalizeImageDict", "normalize_image", "resize_bilinear"]
