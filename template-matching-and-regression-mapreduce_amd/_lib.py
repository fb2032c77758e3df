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
    "names": ["image", "type", "ht", "wt", "roi", "pbox", "tmpl_offset", "row_offset", "pad_"],
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
# correlation kernel choice (tmr_xcorr_args_t.algo)
XCORR_ALGOS = {"auto": 0, "valu": 1, "mfma": 2}
XPACK_UPSAMPLE, XPACK_ONES = 1, 2  # tmr_split_xpack `up` bits
# tmr_size kinds
SIZE_KINDS = {"template_split": 1, "heads_partials": 2, "xpack": 3, "wpack": 4, "acc": 5, "nms_work": 6,
              "stats_work": 7}
ABI_VERSION = 3

_P = ctypes.c_void_p
_I = ctypes.c_int
_L = ctypes.c_int64
_D = ctypes.c_double


class XcorrArgs(ctypes.Structure):
    """tmr_xcorr_args_t (include/tmr.h)."""
    _fields_ = [("f", _P), ("templates", _P), ("units", _P), ("img_units", _P), ("scale", _P), ("out", _P),
                ("relu_out", _P), ("work", _P), ("out_absmax", _P), ("tmpl_split", _P), ("total_rows", _L),
                ("B", ctypes.c_int32), ("C", ctypes.c_int32), ("H", ctypes.c_int32), ("W", ctypes.c_int32),
                ("U", ctypes.c_int32), ("max_ht", ctypes.c_int32), ("max_wt", ctypes.c_int32),
                ("squeeze", ctypes.c_int32), ("algo", ctypes.c_int32), ("min_k", ctypes.c_int32),
                ("prec", ctypes.c_int32), ("out_bf16", ctypes.c_int32)]

# name -> (restype, argtypes)
SIGNATURES = {
    "tmr_version": (_I, []),
    "tmr_strerror": (ctypes.c_char_p, [_I]),
    "tmr_upsample2x": (_I, [_P, _I, _I, _I, _P, _P]),
    "tmr_templates": (_I, [_P, _I, _I, _I, _I, _P, _I, _I, _I, _P, _P]),
    "tmr_size": (_L, [_I, _L, _L, _L, _L, _L, _L]),
    "tmr_xcorr": (_I, [ctypes.POINTER(XcorrArgs), _P]),
    "tmr_template_split": (_I, [_P, _P, _I, _I, _L, _I, _P, _P]),  # (..., total_rows, prec, out, stream)
    "tmr_heads_reduce": (_I, [_P, _I, _I, _I, _I, _I, _P, _P, _P, _P]),
    "tmr_absmax_rows": (_I, [_P, _I, _L, _I, _P, _P]),
    "tmr_scale_merge": (_I, [_P, _P, _P, _I, _I, _P, _P, _P]),
    "tmr_pixel_absmax": (_I, [_P, _I, _I, _L, _P, _P]),
    "tmr_split_xpack": (_I, [_P, _I, _I, _I, _I, _I, _I, _I, _P, _I, _P, _P]),
    "tmr_split_xpack16": (_I, [_P, _I, _I, _I, _I, _I, _I, _P, _P]),
    "tmr_split_fold_proj": (_I, [_P, _I, _I, _I, _I, _P, _P, _I, _P, _P]),
    "tmr_split_wpack": (_I, [_P, _I, _I, _I, _I, _I, _P, _P, _P]),
    "tmr_split_conv": (_I, [_P, _I, _P, _P, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _I, _I, _P, _P, _P, _I,
                            _P]),
    "tmr_peaks_decode": (_I, [_P, _I, _P, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P]),
    "tmr_maxpool3x3": (_I, [_P, _L, _I, _I, _I, _P, _P]),
    "tmr_nms": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _I, _L, _L, _L, _D, _P, _P, _P, _P, _P, _P, _P]),
    "tmr_nms_small": (_I, [_P, _P, _P, _P, _P, _P, _I, _D, _P, _P, _P, _P, _P, _P]),
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
        if lib.tmr_version() != ABI_VERSION:
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


def size(kind: str, *dims) -> int:
    """tmr_size: bytes (or floats) of a caller-provided buffer; raises on
    invalid dimensions."""
    d = [int(x) for x in dims] + [0] * (6 - len(dims))
    n = int(load().tmr_size(SIZE_KINDS[kind], *d))
    if n < 0:
        raise TMRError(f"tmr_size({kind}, {dims}): invalid dimensions")
    return n


def xcorr(**fields) -> None:
    """tmr_xcorr with a tmr_xcorr_args_t built from keyword fields (pointer
    fields take ptr(...) values or None; omitted fields are 0 / NULL)."""
    a = XcorrArgs()
    for k, v in fields.items():
        if k == "stream":
            continue
        setattr(a, k, v if v is not None else (None if k in _XPTR else 0))
    check(load().tmr_xcorr(ctypes.byref(a), fields.get("stream")), "tmr_xcorr")


_XPTR = {"f", "templates", "units", "img_units", "scale", "out", "relu_out", "work", "out_absmax", "tmpl_split"}


def require_gpu(t: torch.Tensor, name: str = "input") -> None:
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise TMRError(f"{name} must be a tensor on a HIP device (MI355X); no CPU path exists")
