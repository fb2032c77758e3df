"""tmr_amd -- MI355X-native TMR hot path (template matching + regression +
peaks/NMS), a drop-in for the reference's models/ and utils/TM_utils.py API.

Import name ``tmr_amd`` (see tmr_import.py; the directory name is not a
Python identifier).  All compute runs in libtmr.so (csrc/, hand-written HIP
for gfx950); there is no CPU fallback.
"""
from . import host, synth  # noqa: F401
from ._lib import LIB_PATH, TMRError, load  # noqa: F401
from .backbone import FeatureInput, build_backbone, register_backbone, unregister_backbone  # noqa: F401
from .engine import PathConfig, TMREngine, conv2d_split  # noqa: F401
from .matching_net import Backbone_Encoder, build_encoder, build_model, matching_net  # noqa: F401
from .regression_head import BboxesHead, Decoder_model, ObjectnessHead  # noqa: F401
from .template_matching import TemplateMatching  # noqa: F401
from .tm_utils import (NMS, Get_pred_boxes, Make_Template_size_predictions,  # noqa: F401
                       NMS_process, adaptive_kernel_generater, calc_area, custom_shape_3x3_maxpool2d,
                       map_normalization)

__all__ = [
    "TemplateMatching", "Decoder_model", "ObjectnessHead", "BboxesHead", "matching_net",
    "build_model", "Backbone_Encoder", "build_encoder", "Get_pred_boxes", "NMS", "NMS_process",
    "adaptive_kernel_generater", "Make_Template_size_predictions", "custom_shape_3x3_maxpool2d",
    "calc_area", "map_normalization", "TMREngine", "PathConfig",
    "TMRError", "build_backbone", "register_backbone", "unregister_backbone", "FeatureInput",
]
