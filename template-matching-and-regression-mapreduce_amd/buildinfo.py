"""Which sources build each profiled kernel role, and their digest.

A rocprofv3 PMC record (profiles/pmc_by_config.json, profiles/pmc_assemble.py)
stores the digest of the sources of the kernel it measured; bench.py prints
the record's counters (``roofline.traffic``, ``mfma_busy_pmc``) only when the
current tree's digest is the same, so a counter figure can never outlive the
kernel it was collected on.
"""
from __future__ import annotations

import hashlib
import os

_CSRC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "csrc")
_COMMON = ("tmr_common.h", "Makefile")
# kernel role (pmc_assemble.ROLES) -> the csrc files its code object depends on
KERNEL_SOURCES = {
    "heads": ("conv_split.hip",) + _COMMON,
    "store": ("conv_split.hip",) + _COMMON,
    "xcorr": ("xcorr.hip",) + _COMMON,
}


def source_digest(role: str) -> str:
    """SHA-256 (hex, first 16 digits) over the role's source files."""
    h = hashlib.sha256()
    for name in KERNEL_SOURCES[role]:
        h.update(name.encode() + b"\0")
        with open(os.path.join(_CSRC, name), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]
