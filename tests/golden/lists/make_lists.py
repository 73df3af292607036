#!/usr/bin/env python3
"""Repeated columns (max_rep > 0, SURVEY §8a R-LEVELS) as pyarrow 25 writes
them, within the reference's format scope (V1 data pages, no codec).

The Parquet spec lays a V1 page out as [rep levels][def levels][values];
the reference reads the first section as definition levels and the second as
repetition levels, which it decodes and drops (column_reader.cpp:146-164).
So on these files it reports the repetition levels, decoded at the
definition levels' bit width, as the null pattern, and then reads as many
values as that pattern has non-null rows.  Parity is with that behaviour,
not with pyarrow's reading of the lists.

  list_int64_req.parquet     list<int64> not null, elements not null
                             (max_def 1, max_rep 1: equal level bit widths),
                             PLAIN; empty lists
  list_str_req_dict.parquet  list<string>, same levels, dictionary pages
  list_str_opt_plain.parquet list<string> nullable, elements nullable
                             (max_def 3, bit width 2 over a 1-bit stream),
                             PLAIN
  list_int64_opt_plain.parquet  list<int64>, same levels as above, PLAIN
  list_double_opt_plain.parquet list<double>, same levels, PLAIN

(Dictionary pages with max_def 3 are left out: a level read above max_def
makes the reference index past its num_non_null indices, undefined
behaviour, column_reader.cpp:181-189.)

manifest.json: per file / row group / column the reference's result (rc,
message, sha256 + length of the canonical dump) from oracle/_ref, and the
oracle's, which must agree.
usage: python tests/golden/lists/make_lists.py (needs oracle/_ref)"""
import hashlib
import json
import os
import sys

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(HERE)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "duckdb-parquet-parser_amd"), os.path.join(ROOT, "tests")]


def words(rng, n, lo, hi):
    return ["".join(chr(97 + int(c)) for c in rng.integers(0, 26, int(rng.integers(lo, hi)))) for _ in range(n)]


def lists(rng, rows, maxlen, make, null_list=0.0, null_elem=0.0):
    out = []
    for _ in range(rows):
        if null_list and rng.random() < null_list:
            out.append(None)
            continue
        k = int(rng.integers(0, maxlen + 1))
        vals = make(k)
        if null_elem:
            vals = [None if rng.random() < null_elem else v for v in vals]
        out.append(vals)
    return out


def table(kind, rows, seed):
    rng = np.random.default_rng(seed)
    vocab = words(rng, 300, 3, 18)
    if kind == "int64_req":
        t = pa.list_(pa.field("element", pa.int64(), nullable=False))
        data = lists(rng, rows, 6, lambda k: [int(x) for x in rng.integers(-1 << 40, 1 << 40, k)])
        return pa.table({"a": pa.array(data, t)}, schema=pa.schema([pa.field("a", t, nullable=False)]))
    if kind == "str_req":
        t = pa.list_(pa.field("element", pa.string(), nullable=False))
        data = lists(rng, rows, 5, lambda k: [vocab[int(x)] for x in rng.integers(0, len(vocab), k)])
        return pa.table({"a": pa.array(data, t)}, schema=pa.schema([pa.field("a", t, nullable=False)]))
    if kind == "str_opt":
        t = pa.list_(pa.field("element", pa.string(), nullable=True))
        data = lists(rng, rows, 5, lambda k: [vocab[int(x)] for x in rng.integers(0, len(vocab), k)], 0.1, 0.15)
        return pa.table({"a": pa.array(data, t)})
    if kind == "int64_opt":
        t = pa.list_(pa.field("element", pa.int64(), nullable=True))
        data = lists(rng, rows, 4, lambda k: [int(x) for x in rng.integers(-1000, 1000, k)], 0.1, 0.1)
        return pa.table({"a": pa.array(data, t)})
    if kind == "double_opt":
        t = pa.list_(pa.field("element", pa.float64(), nullable=True))
        data = lists(rng, rows, 4, lambda k: [float(x) for x in rng.standard_normal(k)], 0.05, 0.2)
        return pa.table({"a": pa.array(data, t)})
    raise ValueError(kind)


FILES = {
    "list_int64_req.parquet": (lambda: table("int64_req", 6000, 41), False),
    "list_str_req_dict.parquet": (lambda: table("str_req", 6000, 42), True),
    "list_str_opt_plain.parquet": (lambda: table("str_opt", 5000, 43), False),
    "list_int64_opt_plain.parquet": (lambda: table("int64_opt", 5000, 44), False),
    "list_double_opt_plain.parquet": (lambda: table("double_opt", 5000, 45), False),
}
NAMES = list(FILES)


def write(name):
    make, use_dict = FILES[name]
    path = os.path.join(HERE, name)
    pq.write_table(make(), path, compression="NONE", data_page_version="1.0", use_dictionary=use_dict,
                   write_statistics=False, row_group_size=2500, data_page_size=2048, write_batch_size=256)
    return path


def main():
    from oracle import oracle as O
    from util import file_chunks, to_oracle_chunk
    if not O.have_ref():
        sys.exit("oracle/_ref/libpqref.so missing: run `make -C oracle ref` first")
    man = {"files": {}}
    for name in FILES:
        f = open(write(name), "rb").read()
        entry = {"bytes": len(f), "row_groups": []}
        for ch in file_chunks(f, 0):
            c = to_oracle_chunk(ch)
            rr, rmsg, rdump = O.ref_read_all(f, c)
            for _ in range(3):
                assert O.ref_read_all(f, c) == (rr, rmsg, rdump), ("reference not deterministic", name)
            rc, msg, col = O.read_all(f, c)
            assert (rc != 0) == (rr != 0) and msg == rmsg, (name, rc, msg, rr, rmsg)
            rec = {"max_def": c.max_def, "max_rep": c.max_rep, "num_values": c.num_values, "rc": rr, "msg": rmsg}
            if rr == 0:
                d = O.dump_column(col)
                assert d == rdump, name
                rec.update(len=len(d), sha256=hashlib.sha256(d).hexdigest(),
                           non_null=int(np.asarray(col.valid, dtype=np.int64).sum()))
            entry["row_groups"].append(rec)
        man["files"][name] = entry
        print(name, len(f), [(r["max_def"], r["rc"], r.get("non_null")) for r in entry["row_groups"]])
    with open(os.path.join(HERE, "manifest.json"), "w") as fp:
        json.dump(man, fp, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
