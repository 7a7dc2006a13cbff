"""Minimal RandomCrop / CenterCrop / ToTensor / Compose (torchvision is not part of this image).

Same semantics as torchvision for PIL inputs: crops take (h, w) sizes, ToTensor gives float [0,1] CHW."""
import random

import numpy as np
import torch


class Compose:
    def __init__(self, transforms):
        self.transforms = list(transforms)

    def __call__(self, img):
        for t in self.transforms:
            img = t(img)
        return img


def _size(size):
    return tuple(size) if hasattr(size, "__iter__") else (size, size)


class RandomCrop:
    def __init__(self, size):
        self.size = _size(size)

    def __call__(self, img):
        th, tw = self.size
        w, h = img.size
        i = random.randint(0, h - th) if h > th else 0
        j = random.randint(0, w - tw) if w > tw else 0
        return img.crop((j, i, j + tw, i + th))


class CenterCrop:
    def __init__(self, size):
        self.size = _size(size)

    def __call__(self, img):
        th, tw = self.size
        w, h = img.size
        i = int(round((h - th) / 2.0))
        j = int(round((w - tw) / 2.0))
        return img.crop((j, i, j + tw, i + th))


class ToTensor:
    def __call__(self, img):
        a = np.asarray(img, dtype=np.uint8)
        if a.ndim == 2:
            a = a[:, :, None]
        return torch.from_numpy(a.copy()).permute(2, 0, 1).float().div(255.0)
