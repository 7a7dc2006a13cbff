"""src/utils/dataset_utils.py: ImageFolder (host I/O, kept) and the data-parallel wrapper.

The reference's ``CustomDataParallel(nn.DataParallel)`` (:76-82) is single-process, disabled by
``CUDA_VISIBLE_DEVICES=gpu_id`` and broken when forced.  Data parallelism here is one
process per GPU (torchrun) with the RCCL FlatGradReducer (hyres_hip.ddp); ``CustomDataParallel`` is kept
as a transparent attribute-forwarding wrapper so reference code that wraps the model still runs."""
from pathlib import Path

import torch.nn as nn
from PIL import Image
from torch.utils.data import Dataset

__all__ = ["ImageFolder", "CustomDataParallel"]


class ImageFolder(Dataset):
    """rootdir/{train,test}/*.png (src/utils/dataset_utils.py:8-73)."""

    def __init__(self, root, transform=None, split="train"):
        splitdir = Path(root) / split
        if not splitdir.is_dir():
            raise RuntimeError(f'Invalid directory "{root}"')
        self.samples = sorted(f for f in splitdir.iterdir() if f.is_file())
        self.transform = transform

    def __getitem__(self, index):
        img = Image.open(self.samples[index]).convert("RGB")
        if self.transform and hasattr(self.transform, "transforms"):
            crop_size = None
            for t in self.transform.transforms:
                if hasattr(t, "size") and t.__class__.__name__ in ("RandomCrop", "CenterCrop"):
                    crop_size = tuple(t.size) if hasattr(t.size, "__iter__") else (t.size, t.size)
                    break
            if crop_size and (img.width < crop_size[0] or img.height < crop_size[1]):
                scale = max(crop_size[0] / img.width, crop_size[1] / img.height) * 1.01
                new_width = max(int(img.width * scale), crop_size[0])
                new_height = max(int(img.height * scale), crop_size[1])
                img = img.resize((new_width, new_height), Image.BILINEAR)
        if self.transform:
            return self.transform(img)
        return img

    def __len__(self):
        return len(self.samples)


class CustomDataParallel(nn.Module):
    """Attribute-forwarding wrapper (no replication: one process per GPU does the data parallelism)."""

    def __init__(self, module):
        super().__init__()
        self.module = module

    def forward(self, *args, **kwargs):
        return self.module(*args, **kwargs)

    def __getattr__(self, key):
        try:
            return super().__getattr__(key)
        except AttributeError:
            return getattr(self.module, key)
