#!/usr/bin/env python3
"""Fixtures for the extended format scope: compressed
pages (SNAPPY, GZIP, LZ4_RAW, ZSTD) and DATA_PAGE_V2 pages, written by pyarrow 25
(the oracle for this row: the reference rejects every codec,
column_reader.cpp:13-15, and does not decode V2 pages, 56-67).

Writes ext_<codec>_v<1|2>.parquet (same table in every file) and
manifest.json: per file and column, the sha256 and length of the canonical
dump of the column as pyarrow reads it.
usage: python tests/golden/ext/make_ext.py"""
import hashlib
import json
import os
import struct
import sys

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq

HERE = os.path.dirname(os.path.abspath(__file__))
CODECS = ["none", "snappy", "gzip", "lz4", "zstd"]
VERSIONS = ["1.0", "2.0"]
ROWS = 3000
RG_ROWS = 1500


def table(rows: int, seed: int = 7) -> pa.Table:
    rng = np.random.default_rng(seed)
    words = ["".join(chr(97 + int(c)) for c in rng.integers(0, 26, int(k))) for k in rng.integers(3, 30, 120)]
    runs = np.repeat(rng.integers(0, len(words), rows), 1)  # dictionary column: uniform entries
    s_dict = [None if rng.random() < 0.05 else words[int(i)] for i in runs]
    s_plain = [" ".join(words[int(j)] for j in rng.integers(0, len(words), int(k)))[: int(t)]
               for k, t in zip(rng.integers(1, 6, rows), rng.integers(1, 60, rows))]
    i64 = rng.integers(-(1 << 62), 1 << 62, rows, dtype=np.int64)
    f64 = rng.random(rows) * 2000.0 - 1000.0
    f64_mask = rng.random(rows) < 0.03
    i32d = rng.integers(0, 50, rows).astype(np.int32)
    i32_mask = rng.random(rows) < 0.1
    b = rng.random(rows) < 0.4
    b_mask = rng.random(rows) < 0.2
    schema = pa.schema([
        pa.field("s_dict", pa.string(), nullable=True),
        pa.field("s_plain", pa.string(), nullable=False),
        pa.field("i64", pa.int64(), nullable=False),
        pa.field("f64", pa.float64(), nullable=True),
        pa.field("i32d", pa.int32(), nullable=True),
        pa.field("b", pa.bool_(), nullable=True),
    ])
    return pa.table([
        pa.array(s_dict, pa.string()),
        pa.array(s_plain, pa.string()),
        pa.array(i64),
        pa.array(f64, mask=f64_mask),
        pa.array(i32d, mask=i32_mask),
        pa.array(b, mask=b_mask),
    ], schema=schema)


def write(t: pa.Table, path, codec: str, version: str, page: int = 1024, rg: int = RG_ROWS):
    pq.write_table(t, path, compression=codec.upper() if codec != "lz4" else "LZ4", data_page_version=version,
                   data_page_size=page, row_group_size=rg, use_dictionary=["s_dict", "i32d"],
                   write_statistics=True, write_batch_size=64)


def canonical_dump(col: pa.ChunkedArray) -> bytes:
    """u8 is_null, then the value: BYTE_ARRAY u32 len + bytes, INT32/FLOAT 4 B,
    INT64/DOUBLE 8 B, BOOLEAN 1 B (little endian, bit patterns)."""
    t = col.type
    out = bytearray()
    fmt = {pa.int32(): "<i", pa.int64(): "<q", pa.float64(): "<d", pa.float32(): "<f"}.get(t)
    for v in col.to_pylist():
        if v is None:
            out += b"\x01"
            continue
        out += b"\x00"
        if pa.types.is_string(t) or pa.types.is_binary(t):
            bb = v.encode() if isinstance(v, str) else v
            out += struct.pack("<I", len(bb)) + bb
        elif pa.types.is_boolean(t):
            out += b"\x01" if v else b"\x00"
        else:
            out += struct.pack(fmt, v)
    return bytes(out)


def main():
    # --new: write only the files the manifest does not list yet (the others
    # stay byte for byte as committed)
    only_new = "--new" in sys.argv
    t = table(ROWS)
    man = {"rows": ROWS, "rg_rows": RG_ROWS, "pyarrow": pa.__version__, "files": {}}
    mpath = os.path.join(HERE, "manifest.json")
    if only_new and os.path.exists(mpath):
        with open(mpath) as fh:
            man = json.load(fh)
    for codec in CODECS:
        for v in VERSIONS:
            name = f"ext_{codec}_v{v[0]}.parquet"
            path = os.path.join(HERE, name)
            if only_new and name in man["files"]:
                continue
            write(t, path, codec, v)
            back = pq.read_table(path)
            cols = {}
            for c in back.column_names:
                d = canonical_dump(back.column(c))
                cols[c] = {"sha256": hashlib.sha256(d).hexdigest(), "len": len(d)}
            man["files"][name] = {"codec": codec, "version": v, "columns": cols}
    with open(os.path.join(HERE, "manifest.json"), "w") as fh:
        json.dump(man, fh, indent=1, sort_keys=True)
    print("wrote", len(man["files"]), "files", file=sys.stderr)


if __name__ == "__main__":
    main()
