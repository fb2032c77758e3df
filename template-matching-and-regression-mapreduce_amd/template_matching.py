"""Drop-in ``TemplateMatching`` (reference: models/template_matching.py:8-99).

Same constructor, parameters (``scale``), state_dict keys and forward
signature; the template extraction (RoIAlign / prototype) and the depthwise
cross-correlation run in libtmr.so (tmr_templates, tmr_xcorr).
"""
from __future__ import annotations

import numpy as np
import torch
from torch import nn

from . import host
from ._lib import require_gpu
from .engine import PathConfig, TMREngine


def _box_host(exemplar_coord) -> np.ndarray:
    if isinstance(exemplar_coord, torch.Tensor):
        return exemplar_coord.detach().float().cpu().numpy().reshape(4)
    return np.asarray(exemplar_coord, np.float32).reshape(4)


class TemplateMatching(nn.Module):
    def __init__(self, template_type, squeeze=False):
        super().__init__()
        if template_type not in host.TEMPLATE_TYPES:
            raise KeyError(template_type)  # template_types[...] lookup, :16-20
        self.template_type = template_type
        self.squeeze = squeeze
        self.scale = nn.Parameter(torch.tensor([1.0], dtype=torch.float32))
        self.avg_pool = nn.AdaptiveAvgPool2d((1, 1))  # parameter-free, kept for parity

    def _engine(self, C: int) -> TMREngine:
        cfg = PathConfig(emb_dim=C, squeeze=self.squeeze, template_type=self.template_type)
        return TMREngine({"matcher.scale": self.scale}, cfg)

    def matcher(self, sample, exemplars):
        """Per-image template + xcorr (:79-93); returns the *scaled* map."""
        require_gpu(sample, "feature")
        B, C, H, W = sample.shape
        boxes = np.stack([_box_host(exemplars[b][0]) for b in range(B)])
        out, _ = self._engine(C).match(sample.float().contiguous(), list(range(B)), boxes)
        return out

    def forward(self, feature, exemplars):
        # the kernel applies `* self.scale` (:97) in its epilogue
        return self.matcher(feature, exemplars)

    def extract_template(self, f, exemplar_coord):
        """roi_align template [1,C,Ht,Wt] (:55-76)."""
        return self._templates(f, exemplar_coord, "roi_align")

    def extract_prototype(self, f, exemplar_coord):
        """AdaptiveAvgPool2d(1) prototype [1,C,1,1] (:43-53)."""
        return self._templates(f, exemplar_coord, "prototype")

    def _templates(self, f, exemplar_coord, ttype):
        from ._lib import call, ptr, stream
        from .engine import _units_to_device

        require_gpu(f, "feature")
        f = f.float().contiguous()
        _, C, H, W = f.shape
        units, tfl, mh, mw = host.build_units(_box_host(exemplar_coord)[None], [0], H, W, C, ttype)
        t = torch.empty(tfl, device=f.device, dtype=torch.float32)
        ud = _units_to_device(units, f.device)
        call("tmr_templates", ptr(f), 1, C, H, W, ptr(ud), 1, mh, mw, ptr(t), stream())
        return t.view(1, C, int(units["ht"][0]), int(units["wt"][0]))
