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
import re

_CSRC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "csrc")
_COMMON = ("tmr_common.h", "Makefile")
# kernel role (pmc_assemble.ROLES) -> the csrc files its code object depends on
KERNEL_SOURCES = {
    "heads": ("conv_split.hip",) + _COMMON,
    "store": ("conv_split.hip",) + _COMMON,
    "xcorr": ("xcorr.hip",) + _COMMON,
}


def _code(name: str, text: bytes) -> bytes:
    """The code of a source file: C/C++ comments (and Makefile comment lines)
    removed and whitespace runs collapsed, so a comment-only edit keeps the
    digest and any code edit changes it."""
    if name == "Makefile":
        text = re.sub(rb"(?m)^\s*#[^\n]*$", b"", text)
    else:
        text = re.sub(rb"//[^\n]*|/\*.*?\*/", b" ", text, flags=re.S)
    return b" ".join(text.split())


def source_digest(role: str) -> str:
    """SHA-256 (hex, first 16 digits) over the code of the role's source
    files (comments and whitespace layout excluded)."""
    h = hashlib.sha256()
    for name in KERNEL_SOURCES[role]:
        h.update(name.encode() + b"\0")
        with open(os.path.join(_CSRC, name), "rb") as fh:
            h.update(_code(name, fh.read()))
    return h.hexdigest()[:16]
