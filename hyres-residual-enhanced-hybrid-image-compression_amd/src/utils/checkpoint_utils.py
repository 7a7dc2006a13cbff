"""src/utils/checkpoint_utils.py:7-28 (same checkpoint dict layout; safe loading)."""
import os
from pathlib import Path
from typing import Dict

import torch

__all__ = ["DelfileList", "load_checkpoint", "save_checkpoint"]


def DelfileList(path, filestarts="checkpoint_last"):
    for root, dirs, files in os.walk(path):
        for file in files:
            if file.startswith(filestarts):
                os.remove(os.path.join(root, file))


def load_checkpoint(filepath: Path) -> Dict[str, torch.Tensor]:
    checkpoint = torch.load(filepath, map_location="cpu", weights_only=True)
    if "network" in checkpoint:
        return checkpoint["network"]
    if "state_dict" in checkpoint:
        return checkpoint["state_dict"]
    return checkpoint


def save_checkpoint(state, filename="checkpoint.pth.tar"):
    torch.save(state, filename)
