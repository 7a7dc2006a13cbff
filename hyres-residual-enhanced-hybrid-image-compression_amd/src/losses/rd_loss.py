"""src/losses/rd_loss.py — RateDistortionLoss on HIP reductions (see hyres_hip.loss)."""
from hyres_hip.loss import RateDistortionLoss  # noqa: F401
