from .checkpoint import load_checkpoint, save_checkpoint, str_to_bool
from .trainer import Trainer, weak_loss

__all__ = ["load_checkpoint", "save_checkpoint", "str_to_bool", "Trainer", "weak_loss"]
