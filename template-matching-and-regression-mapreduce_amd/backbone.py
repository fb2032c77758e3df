"""Backbone hook of ``build_model(args)`` (reference: models/backbone/__init__.py:4-24,
models/__init__.py:4-10).

The reference's ``build_backbone(args)`` picks a frozen SAM / ResNet encoder by
``args.backbone``.  Those encoders are outside the accelerated path
(BASELINE.json north_star: "the frozen SAM/SAM-HQ backbone stays on stock
PyTorch-ROCm ops"), so this module is a registry: the caller registers the
stock-PyTorch encoder under the reference's name once, and
``build_model(args)`` then works exactly as the reference's does
(trainer.py:21, demo.py:58).  Two encoders are built in:

  * ``"features"`` -- identity: the input already IS the backbone feature map
    ``[B, args.num_channels (default 256), h, w]`` (precomputed SAM features,
    extract_feature.py:103-108 / the mapper's .npy cache, mapper.py:116-118);
  * any name registered with :func:`register_backbone`.
"""
from __future__ import annotations

from typing import Callable, Dict

from torch import nn

from ._lib import TMRError

_REGISTRY: Dict[str, Callable] = {}

# the reference's backbone names (models/backbone/__init__.py:5-22)
REFERENCE_BACKBONES = ("resnet50", "resnet50_layer1", "resnet50_layer2", "resnet50_layer3",
                       "resnet50_layer1_FRZ", "resnet50_layer2_FRZ", "resnet50_layer3_FRZ", "sam")


class FeatureInput(nn.Module):
    """Identity encoder over precomputed backbone features (SAM: 256 channels,
    sam.py:33,93)."""

    def __init__(self, num_channels: int = 256):
        super().__init__()
        self.num_channels = num_channels

    def forward(self, x):
        return x


def register_backbone(name: str, factory: Callable) -> None:
    """Register ``factory(args) -> nn.Module`` (with a ``num_channels``
    attribute, like the reference's encoders) under ``args.backbone == name``,
    e.g. ``register_backbone("sam", lambda a: Sam_Backbone(requires_grad=False,
    model_type="vit_h"))`` with the reference's own stock-PyTorch SAM module."""
    if not callable(factory):
        raise TypeError("factory must be callable: factory(args) -> nn.Module")
    _REGISTRY[name] = factory


def unregister_backbone(name: str) -> None:
    _REGISTRY.pop(name, None)


def build_backbone(args) -> nn.Module:
    """models/backbone/__init__.py:4-24 over the registry."""
    name = getattr(args, "backbone", "features")
    if name in _REGISTRY:
        bb = _REGISTRY[name](args)
    elif name == "features":
        bb = FeatureInput(getattr(args, "num_channels", 256))
    else:
        known = sorted(set(_REGISTRY) | {"features"})
        hint = (" (a reference backbone: it runs on stock PyTorch-ROCm, outside this package;"
                " register it with tmr_amd.register_backbone)") if name in REFERENCE_BACKBONES else ""
        raise TMRError(f"backbone {name!r} is not registered{hint}; available: {known}")
    if not hasattr(bb, "num_channels"):
        raise TMRError(f"backbone {name!r} must expose num_channels (models/encoders.py:13)")
    return bb
