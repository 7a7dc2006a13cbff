"""src/losses (src/losses/__init__.py:1-16): RateDistortionLoss (HIP reductions) + AverageMeter."""
from hyres_hip.loss import RateDistortionLoss  # noqa: F401


class AverageMeter:
    """Compute running average."""

    def __init__(self):
        self.val = 0
        self.avg = 0
        self.sum = 0
        self.count = 0

    def update(self, val, n=1):
        self.val = val
        self.sum += val * n
        self.count += n
        self.avg = self.sum / self.count
