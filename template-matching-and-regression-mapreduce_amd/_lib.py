"""ctypes binding of libtmr.so (include/tmr.h).

The library is the ONLY compute path: there is no CPU / PyTorch fallback.  A
missing or unloadable library, or a CPU tensor handed to a compute entry
point, raises immediately.
"""
from __future__ import annotations

import ctypes
import os
import threading

import numpy as np
import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libtmr.so")
if os.environ.get("TMR_LIB_VARIANT"):  # profiling only: an experiment build next to libtmr.so
    LIB_PATH = os.path.join(_HERE, "libtmr_%s.so" % os.environ["TMR_LIB_VARIANT"])
HEADER = os.path.join(os.path.dirname(_HERE), "include", "tmr.h")

_lock = threading.Lock()
_lib = None

# ABI structs (must match include/tmr.h)
UNIT_DTYPE = np.dtype({
    "names": ["image", "type", "ht", "wt", "roi", "pbox", "tmpl_offset", "row_offset", "out_unit"],
    "formats": [np.int32, np.int32, np.int32, np.int32, (np.float32, 4), (np.int32, 4), np.int64,
                np.int32, np.int32],
    "offsets": [0, 4, 8, 12, 16, 32, 48, 56, 60],
    "itemsize": 64,
})
PEAK_DTYPE = np.dtype({
    "names": ["thr", "scale_w", "scale_h", "mask", "mode", "pad_"],
    "formats": [np.float32, np.float32, np.float32, np.int32, np.int32, np.int32],
    "offsets": [0, 4, 8, 12, 16, 20],
    "itemsize": 24,
})

TEMPLATE_ROI_ALIGN = 0
TEMPLATE_PROTOTYPE = 1

# decoder-conv precision modes of the split 16-bit-MFMA kernel (include/tmr.h)
PREC_CODES = {"fp32": 0, "bf16": 1, "f16": 2}
SPLIT_TILED_OUT, SPLIT_TILED_INIT, SPLIT_INIT_BCAST = 1, 2, 4
SPLIT_OUT_BF16, SPLIT_INIT_BF16 = 8, 16  # one-term precisions: bf16 acc0 slabs
SPLIT_XMAX_PER_UNIT = 32  # xmax is float[U]: one activation scale per unit / output slab
SPLIT_XMAX_PER_PIXEL = 64  # 1x1 stores: xmax is float[U][H][W], one scale per output pixel
PEAKS_PROB_SCRATCH = 2  # tmr_peaks_decode: prob is scratch (low logits hold -1)
SPLIT_UNITS_PER_IMAGE_SHIFT = 8  # flags bits 8..15: E units per image -> image-major heads order
# correlation kernel choice (tmr_xcorr_algo)
XCORR_ALGOS = {"auto": 0, "valu": 1, "mfma": 2}

_P = ctypes.c_void_p
_I = ctypes.c_int
_L = ctypes.c_int64
_D = ctypes.c_double

# name -> (restype, argtypes)
SIGNATURES = {
    "tmr_version": (_I, []),
    "tmr_strerror": (ctypes.c_char_p, [_I]),
    "tmr_upsample2x": (_I, [_P, _I, _I, _I, _P, _P]),
    "tmr_templates": (_I, [_P, _I, _I, _I, _I, _P, _I, _I, _I, _P, _P]),
    "tmr_xcorr": (_I, [_P, _I, _I, _I, _I, _P, _P, _P, _I, _I, _I, _P, _I, _P, _P, _P, _P, _P]),
    "tmr_xcorr_algo": (_I, [_P, _I, _I, _I, _I, _P, _P, _P, _I, _I, _I, _P, _I, _P, _P, _P, _P, _P, _L,
                            _I, _I, _P]),
    "tmr_xcorr_prec": (_I, [_P, _I, _I, _I, _I, _P, _P, _P, _I, _I, _I, _P, _I, _P, _P, _P, _P, _P, _L,
                            _I, _I, _I, _P]),
    "tmr_xcorr_out": (_I, [_P, _I, _I, _I, _I, _P, _P, _P, _I, _I, _I, _P, _I, _P, _P, _P, _P, _P, _L,
                           _I, _I, _I, _I, _P]),
    "tmr_template_split_size": (_L, [_I, _I, _L]),
    "tmr_template_split": (_I, [_P, _P, _I, _I, _L, _P, _P]),  # (..., total_rows, out, stream)
    "tmr_template_split_prec": (_I, [_P, _P, _I, _I, _L, _I, _P, _P]),  # (..., total_rows, prec, out, stream)
    "tmr_heads_partials_size": (_L, [_I, _I, _I, _I]),
    "tmr_heads_reduce": (_I, [_P, _I, _I, _I, _I, _I, _P, _P, _P, _P]),
    "tmr_absmax": (_I, [_P, _L, _I, _P, _P]),
    "tmr_absmax_rows": (_I, [_P, _I, _L, _I, _P, _P]),
    "tmr_scale_merge": (_I, [_P, _P, _P, _I, _I, _P, _P, _P]),
    "tmr_pixel_absmax": (_I, [_P, _I, _I, _L, _P, _P]),
    "tmr_split_xpack_size": (_L, [_I, _I, _I, _I, _I, _I]),
    "tmr_split_xpack": (_I, [_P, _I, _I, _I, _I, _I, _I, _P, _I, _P, _P]),
    "tmr_split_xpack16": (_I, [_P, _I, _I, _I, _I, _I, _I, _P, _P]),
    "tmr_split_xpack_ring": (_I, [_P, _I, _I, _I, _I, _I, _I, _P]),
    "tmr_split_xpack_up": (_I, [_P, _I, _I, _I, _I, _I, _I, _I, _I, _P, _I, _P, _P]),
    "tmr_split_fold_proj": (_I, [_P, _I, _I, _I, _I, _P, _P, _I, _P, _P]),
    "tmr_split_wpack_size": (_L, [_I, _I, _I, _I, _I]),
    "tmr_split_wpack": (_I, [_P, _I, _I, _I, _I, _I, _P, _P, _P]),
    "tmr_split_acc_size": (_L, [_I, _I, _I, _I]),
    "tmr_split_conv_store": (_I, [_P, _I, _P, _P, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _I, _I,
                                  _P, _P, _I, _P]),
    "tmr_split_conv_heads": (_I, [_P, _I, _P, _P, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _I, _I,
                                  _P, _P, _P, _I, _P]),
    "tmr_peaks_decode": (_I, [_P, _I, _P, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P]),
    "tmr_maxpool3x3": (_I, [_P, _L, _I, _I, _I, _P, _P]),
    "tmr_nms_work_size": (_L, [_L, _L, _L, _I]),
    "tmr_nms": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _I, _L, _L, _L, _D, _P, _P, _P, _P, _P, _P, _P]),
    "tmr_nms_small": (_I, [_P, _P, _P, _P, _P, _P, _I, _D, _P, _P, _P, _P, _P, _P]),
    "tmr_feature_stats_work_size": (_L, [_I]),
    "tmr_feature_stats": (_I, [_P, _I, _L, _P, _P, _P]),
    "tmr_exp_table_encode": (_L, [_P, _L, _P, _L]),
    "tmr_exp_table_decode": (_L, [_P, _L, _P, _L]),
}


class TMRError(RuntimeError):
    pass


def load() -> ctypes.CDLL:
    """Load libtmr.so (once).  Raises TMRError when it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise TMRError(
                f"libtmr.so not found at {LIB_PATH}; build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.tmr_version() != 2:
            raise TMRError("libtmr.so ABI version mismatch")
        _lib = lib
        return lib


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = load().tmr_strerror(rc).decode()
        raise TMRError(f"{what}: {msg} (rc={rc})" if what else msg)


def ptr(t) -> int | None:
    """Device pointer of a tensor (None -> NULL).  CPU tensors are rejected."""
    if t is None:
        return None
    if not t.is_cuda:
        raise TMRError("tmr_amd kernels run on the GPU only; got a CPU tensor")
    if not t.is_contiguous():
        raise TMRError("tmr_amd kernels need contiguous tensors")
    return t.data_ptr()


def stream(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def call(name: str, *args) -> None:
    check(getattr(load(), name)(*args), name)


def require_gpu(t: torch.Tensor, name: str = "input") -> None:
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise TMRError(f"{name} must be a tensor on a HIP device (MI355X); no CPU path exists")
