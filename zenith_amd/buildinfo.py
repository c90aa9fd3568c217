"""Identity of a libzenith_raster build: a hash of the sources it is compiled from.

Profiles collected on the GPU box (rocprofv3 kernel traces, PMC traffic
summaries under profiles/) record the hash of the tree they ran on, and bench.py
only quotes a profile whose hash is the current tree's: a kernel change after the
last profiling pass makes its numbers stale, and they are dropped rather than
reported beside a different build (tests/test_bench.py checks the committed ones).
"""
from __future__ import annotations

import glob
import hashlib
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SOURCES = ("zenith_amd/csrc/*", "include/zenith_raster.h", "zenith_amd/Makefile")


def source_files(root: str = ROOT) -> list[str]:
    files = []
    for pat in SOURCES:
        files += [f for f in glob.glob(os.path.join(root, pat)) if os.path.isfile(f)]
    return sorted(files)


def source_hash(root: str = ROOT) -> str:
    """sha256 (first 16 hex digits) over the library's source files, path and bytes."""
    h = hashlib.sha256()
    for f in source_files(root):
        h.update(os.path.relpath(f, root).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()[:16]
