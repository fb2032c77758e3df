"""Drop-in ``matching_net`` / ``build_model`` / ``Backbone_Encoder``
(reference: models/matching_net.py:9-81, models/__init__.py:4-10,
models/encoders.py:6-18).

Construction, submodule names and therefore state_dict keys match the
reference, so Lightning checkpoints load unchanged.  The
backbone is whatever module the caller passes (the frozen SAM encoder stays on
stock PyTorch-ROCm, out of scope); everything after it runs in libtmr.so:
upsample+projection, templates, cross-correlation and the fused
decoder+head kernel.
"""
from __future__ import annotations

import torch
from torch import nn

from .backbone import build_backbone
from .engine import PathConfig, TMREngine
from .regression_head import BboxesHead, Decoder_model, ObjectnessHead
from .template_matching import TemplateMatching, _box_host


class Backbone_Encoder(nn.Module):
    """models/encoders.py:9-18: passthrough around the backbone."""

    def __init__(self, backbone, emb_dim):
        super().__init__()
        self.backbone = backbone
        self.num_channels = backbone.num_channels

    def forward(self, x):
        return self.backbone(x)


def build_encoder(args):
    if args.encoder == "original":
        return Backbone_Encoder
    raise KeyError(args.encoder)


class matching_net(nn.Module):
    def __init__(self, backbone, args):
        super().__init__()
        self.args = args
        self.emb_dim = args.emb_dim
        self.fusion = args.fusion
        self.box_reg = not args.ablation_no_box_regression
        self.encoder = build_encoder(args)(backbone, args.emb_dim)
        self.decoder_model = Decoder_model
        self.feature_upsample = args.feature_upsample
        self.matcher = None if args.no_matcher else TemplateMatching(args.template_type, args.squeeze)
        if isinstance(self.encoder.num_channels, list):
            raise NotImplementedError("multi-level encoders are not on the scripted path")
        self.input_proj = nn.ModuleList([nn.Conv2d(self.encoder.num_channels, self.emb_dim, 1)])
        nl, ks = args.decoder_num_layer, args.decoder_kernel_size
        if args.squeeze:
            ch = 1 + self.emb_dim if self.fusion else 1
        else:
            ch = 2 * self.emb_dim if self.fusion else self.emb_dim
        self.decoder_o = self.decoder_model(ch, nl, ks)
        self.decoder_b = self.decoder_model(ch, nl, ks) if self.box_reg else None
        self.objectness_head = ObjectnessHead(self.decoder_o.out_channels)
        self.ltrbs_head = BboxesHead(self.decoder_b.out_channels) if self.box_reg else None
        self._engine = None

    def _param_slots(self):
        """(edges, slots) of the module tree: edges (parent, name, child) of
        every registered submodule and each module's parameter count; slots
        (key, module, name) of every parameter outside the encoder.  Built by
        one walk, reused while every edge and count still holds (a submodule
        or parameter added or replaced re-runs the walk)."""
        c = getattr(self, "_pslots", None)
        if c is not None and all(p._modules.get(n) is m for p, n, m in c[0]) and \
                all(len(m._parameters) == k for m, k in c[1]):
            return c[2]
        edges, counts, slots = [], [], []
        for pre, m in self.named_modules():
            counts.append((m, len(m._parameters)))
            for n, ch in m._modules.items():
                if ch is not None:
                    edges.append((m, n, ch))
            if pre == "encoder" or pre.startswith("encoder."):
                continue
            for n, v in m._parameters.items():
                if v is not None:
                    slots.append((f"{pre}.{n}" if pre else n, m, n))
        object.__setattr__(self, "_pslots", (edges, counts, slots))
        return slots

    def path_params(self):
        """The hot-path parameters under their reference state_dict keys
        (the parameters read through their slots: a parameter re-bound by
        to() / load_state_dict(assign=True) / setattr is the one returned)."""
        P = {k: m._parameters[n] for k, m, n in self._param_slots()}
        if self.matcher is None:
            P["matcher.scale"] = torch.ones(1, device=P["input_proj.0.weight"].device)
        return P

    def engine(self) -> TMREngine:
        P = self.path_params()
        if self._engine is None:
            self._engine = TMREngine(P, PathConfig.from_args(self.args))
            # the callers run one forward per exemplar on the same features
            # (demo.py:111, trainer.py:96): reuse the image's projection and
            # decoder fp half across those calls (same values, fp32 contract)
            self._engine.reuse_image_work = True
        else:
            self._engine.P = P
        return self._engine

    def forward(self, sample, exemplars, **kwargs):
        f = self.encoder(sample)
        if isinstance(f, list):
            if len(f) != 1:
                raise NotImplementedError("one feature level on the path (matching_net.py:54)")
            f = f[0]
        B = f.shape[0]
        eng = self.engine()
        if self.matcher is None:
            boxes = [[0.0, 0.0, 1.0, 1.0]] * B
        else:
            boxes = [_box_host(exemplars[b][0]) for b in range(B)]
        r = eng.forward_units(f, list(range(B)), boxes, want_aux=True)
        return [r["o"]], [r["b"]], [r["f_tm_relu"]], r["f0"]


def build_model(args, backbone=None):
    """models/__init__.py:4-10: ``build_model(args)`` with the reference's
    signature; the backbone comes from ``build_backbone(args)`` (the registry
    in backbone.py: the frozen encoder stays on stock PyTorch-ROCm).  The
    optional ``backbone`` module (extension) bypasses the registry."""
    if backbone is None:
        backbone = build_backbone(args)
    if args.modeltype == "matching_net":
        return matching_net(backbone, args)
    raise KeyError(args.modeltype)
