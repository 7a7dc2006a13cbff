"""AttentionBlock (models/layers/attention.py:7-47) on HIP.

out = conv_a(x) * sigmoid(conv_b(x)) + x, conv_a = 3 ResidualUnits, conv_b = 3 ResidualUnits + 1x1.
ResidualUnit = relu(x + 1x1(relu(3x3(relu(1x1(x)))))): the residual add and final ReLU are fused into
the last 1x1 conv's epilogue; the gate is one elementwise kernel."""
from __future__ import annotations

import torch.nn as nn

from hyres_hip import _lib as L
from hyres_hip import ops as O
from hyres_hip.layers import HipModule, ReLU, Sequential, conv1x1, conv3x3

__all__ = ["AttentionBlock", "ResidualUnit"]


class ResidualUnit(HipModule):
    """Simple residual unit (the reference defines it inside AttentionBlock.__init__, :11-30)."""

    def __init__(self, N: int):
        super().__init__()
        self.conv = Sequential(
            conv1x1(N, N // 2),
            ReLU(inplace=True),
            conv3x3(N // 2, N // 2),
            ReLU(inplace=True),
            conv1x1(N // 2, N),
        )
        self.relu = ReLU(inplace=True)

    def hip(self, tape, x):
        y = O.residual_unit_fused(tape, x, self.conv[0], self.conv[2], self.conv[4], final_relu=True)
        if y is not None:  # autocast with fp16 activations: one launch, t1 / t2 on chip (csrc/ru_fused.hip)
            return y
        t = self.conv[0].hip(tape, x, act=L.ACT_RELU)
        t = self.conv[2].hip(tape, t, act=L.ACT_RELU)
        return self.conv[4].hip(tape, t, act=L.ACT_RELU, res=x)


class AttentionBlock(HipModule):
    def __init__(self, N: int):
        super().__init__()
        self.conv_a = nn.Sequential(ResidualUnit(N), ResidualUnit(N), ResidualUnit(N))
        self.conv_b = nn.Sequential(ResidualUnit(N), ResidualUnit(N), ResidualUnit(N), conv1x1(N, N))

    def hip(self, tape, x):
        def branch_a(tape, a):
            for ru in self.conv_a:
                a = ru.hip(tape, a)
            return a

        def branch_b(tape, b):
            for ru in list(self.conv_b)[:3]:
                b = ru.hip(tape, b)
            return self.conv_b[3].hip(tape, b)

        # the two branches are independent: run them on two HIP streams (forward and backward)
        a, b = O.run_branches(tape, x, [branch_a, branch_b])
        return O.attn_gate(tape, a, b, x)
