"""src/utils/optimizers.py:4-35 — main/aux optimisers, as fused HIP Adam over flat buffers."""
from hyres_hip.optim import FusedAdam, configure_optimizers  # noqa: F401

__all__ = ["configure_optimizers", "FusedAdam"]
