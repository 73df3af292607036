"""The real-world dictionary fixtures (tests/golden/dict_shapes, written by
make_dict_shapes.py with pyarrow 25): chunks mixing dictionary and PLAIN data
pages, and dictionaries over 64 KiB / 65,535 entries."""
from __future__ import annotations

import hashlib
import json
import os

DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "dict_shapes")
NAMES = ["fallback_opt.parquet", "fallback_req.parquet", "big_dict.parquet", "wide_dict.parquet"]


def manifest() -> dict:
    with open(os.path.join(DIR, "manifest.json")) as fh:
        return json.load(fh)


def load(name: str) -> bytes:
    with open(os.path.join(DIR, name), "rb") as fh:
        return fh.read()


def sha(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()
