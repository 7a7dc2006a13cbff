"""models/layers/common.py:4-11 — conv helper factories (HIP implicit-GEMM convolutions)."""
from hyres_hip.layers import conv1x1, conv3x3  # noqa: F401

__all__ = ["conv1x1", "conv3x3"]
