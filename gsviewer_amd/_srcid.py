"""Digest of the sources libgsr.so is built from.

``build.py`` compiles it into the library (``gsr_source_digest()``) and
``_lib.load`` compares it with the tree's, so a library older than its
sources fails to load instead of being tested, benchmarked and profiled as
if it were the current tree (the GPU box runs the in-tree ``.so`` without
building).  Only the in-tree library is checked; ``GSR_LIB_PATH`` variants
(A/B builds of other trees) are not.
"""
from __future__ import annotations

import hashlib
import os

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(ROOT, "include")


def source_files():
    """Every file the library's objects are compiled from: csrc/*.hip|cpp|h and include/*.h."""
    out = []
    for d, exts in ((CSRC, (".hip", ".cpp", ".h")), (INCLUDE, (".h",))):
        out += [os.path.join(d, f) for f in sorted(os.listdir(d)) if f.endswith(exts)]
    return out


def source_digest() -> str:
    h = hashlib.sha256()
    for p in source_files():
        h.update(os.path.relpath(p, ROOT).encode())
        h.update(b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()[:16]
