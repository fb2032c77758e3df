"""Drop-in ``Decoder_model`` / ``ObjectnessHead`` / ``BboxesHead``
(reference: models/regression_head.py:3-62).

Same constructors, reference initialisation (N(0, 0.01) weights, zero bias,
:17-24) and state_dict keys (``layer.<2i>.weight``, ``head.0.weight``).
``Decoder_model`` runs on the split 16-bit-MFMA implicit-GEMM kernel
(tmr_split_conv; ``precision`` "fp32" = 3-term fp16 split, the fp32
1e-5 contract; "bf16" = config C), the 1x1 heads on the same kernel at
ks = 1 (3-term split, fp32 contract).  Inside ``matching_net`` the decoders
and heads are not called one by one: the fused kernel (tmr_split_conv with heads)
consumes their parameters directly.
"""
from __future__ import annotations

from torch import nn

from .engine import conv2d_split


class Decoder_model(nn.Module):
    def __init__(self, in_channels, num_layers=1, kernel_size=3):
        super().__init__()
        layer = []
        for _ in range(num_layers):
            layer.append(nn.Conv2d(in_channels, in_channels, kernel_size=kernel_size,
                                   padding=(kernel_size - 1) // 2))
            layer.append(nn.LeakyReLU())
        self.layer = nn.Sequential(*layer)
        self.out_channels = in_channels
        self.precision = "fp32"
        self.reset_parameters()

    def convs(self):
        return [m for m in self.layer if isinstance(m, nn.Conv2d)]

    def forward(self, x):
        for conv in self.convs():
            x = conv2d_split(x, conv.weight, conv.bias, True, self.precision)
        return x

    def reset_parameters(self):
        for module in self.modules():
            if isinstance(module, nn.Conv2d):
                nn.init.normal_(module.weight, std=0.01)
                if module.bias is not None:
                    nn.init.constant_(module.bias, 0)


class _Head1x1(nn.Module):
    OUT = 1

    def __init__(self, in_channels):
        super().__init__()
        self.head = nn.Sequential(nn.Conv2d(in_channels, self.OUT, kernel_size=1))
        self.reset_parameters()

    def forward(self, x):
        conv = self.head[0]
        return conv2d_split(x, conv.weight, conv.bias, False, "fp32")

    def reset_parameters(self):
        for module in self.modules():
            if isinstance(module, nn.Conv2d):
                nn.init.normal_(module.weight, std=0.01)
                if module.bias is not None:
                    nn.init.constant_(module.bias, 0)


class ObjectnessHead(_Head1x1):
    """1x1 conv -> 1 objectness logit (regression_head.py:26-43)."""
    OUT = 1


class BboxesHead(_Head1x1):
    """1x1 conv -> 4 box regressions (regression_head.py:45-62)."""
    OUT = 4
