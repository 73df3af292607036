"""Helpers for the extended-format tests (compressed pages, DATA_PAGE_V2;
SURVEY §8f rank 4): the committed pyarrow fixtures and their manifest."""
from __future__ import annotations

import hashlib
import json
import os

from pqgpu import capi

EXT_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ext")
EXT_ALL = capi.EXT_CODECS | capi.EXT_PAGE_V2


def manifest() -> dict:
    with open(os.path.join(EXT_DIR, "manifest.json")) as fh:
        return json.load(fh)


def load(name: str) -> bytes:
    with open(os.path.join(EXT_DIR, name), "rb") as fh:
        return fh.read()


def ext_chunks(file: bytes, col: int, flags: int = EXT_ALL):
    F = capi.File(file)
    out = []
    for rg in range(F.num_row_groups):
        d = F.chunk(rg, col)
        d.ext_flags = flags
        out.append(d)
    return out


def sha(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()
