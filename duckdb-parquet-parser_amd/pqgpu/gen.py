"""Deterministic synthetic Parquet inputs — ctypes over libpqgen.so.

The generator is C++ (csrc/gen/pqgen.cpp); this module only describes the
benchmark configurations and calls it.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field

from . import _paths

BOOLEAN, INT32, INT64, INT96, FLOAT, DOUBLE, BYTE_ARRAY, FLBA = range(8)
DICT_STRINGS, COMMENT, UNIFORM, DOUBLE_RANGE, SMALL_INT = range(5)
REF_LAYOUT, ARROW_LAYOUT = 0, 1


class _Col(C.Structure):
    _fields_ = [
        ("name", C.c_char_p),
        ("kind", C.c_int32),
        ("type", C.c_int32),
        ("optional", C.c_int32),
        ("null_frac", C.c_double),
        ("dict_size", C.c_int32),
        ("len_min", C.c_int32),
        ("len_max", C.c_int32),
        ("max_run", C.c_int32),
        ("force_plain", C.c_int32),
    ]


class _Opts(C.Structure):
    _fields_ = [
        ("layout", C.c_int32),
        ("rows_per_page", C.c_int32),
        ("footer_pad", C.c_int32),
        ("first_rg", C.c_int32),
    ]


@dataclass
class Col:
    name: str
    kind: int
    type: int
    optional: bool = False
    null_frac: float = 0.0
    dict_size: int = 0
    len_min: int = 0
    len_max: int = 0
    max_run: int = 0
    force_plain: bool = False

    def c(self) -> _Col:
        return _Col(self.name.encode(), self.kind, self.type, int(self.optional), self.null_frac,
                    self.dict_size, self.len_min, self.len_max, self.max_run, int(self.force_plain))


_lib = None


def lib():
    global _lib
    if _lib is None:
        L = C.CDLL(_paths.lib_path("libpqgen.so"))
        L.pqgen_build.argtypes = [C.POINTER(_Col), C.c_int, C.c_int64, C.c_int, C.c_uint64,
                                  C.POINTER(_Opts), C.POINTER(C.POINTER(C.c_uint8)),
                                  C.POINTER(C.c_size_t)]
        L.pqgen_values_dump.argtypes = [C.POINTER(_Col), C.c_int, C.c_int64, C.c_int, C.c_uint64,
                                        C.POINTER(C.POINTER(C.c_uint8)), C.POINTER(C.c_size_t)]
        L.pqgen_free.argtypes = [C.c_void_p]
        _lib = L
    return _lib


def build(cols: list[Col], rows_per_rg: int, nrg: int = 1, seed: int = 1,
          layout: int = REF_LAYOUT, rows_per_page: int = 0, footer_pad: bool = True,
          first_rg: int = 0) -> bytes:
    L = lib()
    arr = (_Col * len(cols))(*[c.c() for c in cols])
    opts = _Opts(layout, rows_per_page, int(footer_pad), first_rg)
    p = C.POINTER(C.c_uint8)()
    n = C.c_size_t()
    rc = L.pqgen_build(arr, len(cols), rows_per_rg, nrg, seed, C.byref(opts), C.byref(p),
                       C.byref(n))
    if rc != 0:
        raise RuntimeError(f"pqgen_build failed: {rc}")
    out = C.string_at(p, n.value)
    L.pqgen_free(p)
    return out


def values_dump(col: Col, col_idx: int, rows: int, rg: int = 0, seed: int = 1) -> bytes:
    L = lib()
    c = col.c()
    p = C.POINTER(C.c_uint8)()
    n = C.c_size_t()
    L.pqgen_values_dump(C.byref(c), col_idx, rows, rg, seed, C.byref(p), C.byref(n))
    out = C.string_at(p, n.value)
    L.pqgen_free(p)
    return out


# ── the five BASELINE.json configurations ──────────────────────
def c1_cols():
    return [Col("v", UNIFORM, INT32)]


def c2_cols():
    return [Col("s", DICT_STRINGS, BYTE_ARRAY, optional=True, null_frac=0.05, dict_size=1000,
                len_min=8, len_max=40, max_run=16)]


def c3_cols():
    return [Col("comment", COMMENT, BYTE_ARRAY, len_min=10, len_max=44)]


def c4_cols():
    return [
        Col("c0", UNIFORM, INT64), Col("c1", UNIFORM, INT64), Col("c2", UNIFORM, INT64),
        Col("c3", DOUBLE_RANGE, DOUBLE, optional=True, null_frac=0.01),
        Col("c4", DOUBLE_RANGE, DOUBLE, optional=True, null_frac=0.01),
        Col("c5", DOUBLE_RANGE, DOUBLE, optional=True, null_frac=0.01),
        Col("c6", DICT_STRINGS, BYTE_ARRAY, dict_size=4096, len_min=4, len_max=20, max_run=16),
        Col("c7", COMMENT, BYTE_ARRAY, len_min=10, len_max=44),
    ]


CONFIG_SEEDS = {"C1": 1, "C2": 2, "C3": 3, "C4": 4, "C5": 2}
