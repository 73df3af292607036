"""The repeated-column fixtures (tests/golden/lists, written by make_lists.py
with pyarrow 25): LIST columns whose V1 pages hold repetition levels, which
the reference reads in its own order (column_reader.cpp:146-164)."""
from __future__ import annotations

import hashlib
import json
import os

DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "lists")
NAMES = ["list_int64_req.parquet", "list_str_req_dict.parquet", "list_str_opt_plain.parquet",
         "list_int64_opt_plain.parquet", "list_double_opt_plain.parquet"]
STRING_NAMES = [n for n in NAMES if "_str_" in n]


def manifest() -> dict:
    with open(os.path.join(DIR, "manifest.json")) as fh:
        return json.load(fh)


def load(name: str) -> bytes:
    with open(os.path.join(DIR, name), "rb") as fh:
        return fh.read()


def sha(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()
