#!/usr/bin/env python3
"""Real-world dictionary shapes (VERDICT r2 "what's missing" 2-3), written by
pyarrow 25 within the reference's format scope (V1 data pages, no codec):

  fallback_opt.parquet / fallback_req.parquet
      a small dictionary_pagesize_limit makes the writer give up on the
      dictionary part-way through each row group: one chunk holds the
      dictionary page, RLE_DICTIONARY data pages, then PLAIN data pages
      (column_reader.cpp:174-177 vs 213-222 decide per page);
  big_dict.parquet
      a 3,000-entry dictionary page of ~120 KiB (over the 64 KiB the LDS
      dictionary kernels take);
  wide_dict.parquet
      a 100,000-entry dictionary page of ~1 MiB (over 65,535 entries: bit
      width 17, no u16 codes).

manifest.json holds, per file / row group / column, the sha256 and length of
the canonical dump that the oracle (oracle/pq_oracle.c) produces;
tests/test_dict_shapes.py pins that oracle to the compiled reference
(oracle/_ref) and to pyarrow's own reading, and the GPU tests compare every
kernel path with it.
usage: python tests/golden/dict_shapes/make_dict_shapes.py"""
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
    out = set()
    while len(out) < n:
        k = int(rng.integers(lo, hi))
        out.add("".join(chr(97 + int(c)) for c in rng.integers(0, 26, k)))
    return sorted(out)


def fallback_table(rows, optional, seed):
    rng = np.random.default_rng(seed)
    vocab = words(rng, 4000, 6, 30)
    # first rows draw from a small set, later rows from the whole vocabulary:
    # the dictionary grows past the limit part-way through the row group
    idx = np.where(np.arange(rows) % 3000 < 1200, rng.integers(0, 40, rows), rng.integers(0, len(vocab), rows))
    vals = [vocab[int(i)] for i in idx]
    mask = (rng.random(rows) < 0.07) if optional else None
    return pa.table({"s": pa.array(vals, pa.string(), mask=mask)},
                    schema=pa.schema([pa.field("s", pa.string(), nullable=optional)]))


def dict_table(rows, entries, lo, hi, seed, null_frac):
    rng = np.random.default_rng(seed)
    vocab = words(rng, entries, lo, hi)
    run = rng.integers(1, 6, rows)
    idx = np.repeat(rng.integers(0, entries, rows), run)[:rows]
    idx[: entries] = np.arange(entries)  # every entry used: the whole dictionary stays
    mask = rng.random(rows) < null_frac
    return pa.table({"s": pa.array([vocab[int(i)] for i in idx], pa.string(), mask=mask)})


FILES = {
    "fallback_opt.parquet": (lambda: fallback_table(6000, True, 31),
                             dict(row_group_size=3000, dictionary_pagesize_limit=4096, data_page_size=1024, write_batch_size=128)),
    "fallback_req.parquet": (lambda: fallback_table(6000, False, 32),
                             dict(row_group_size=3000, dictionary_pagesize_limit=4096, data_page_size=1024, write_batch_size=128)),
    "big_dict.parquet": (lambda: dict_table(40000, 3000, 30, 50, 33, 0.05),
                         dict(row_group_size=40000, dictionary_pagesize_limit=1 << 20, data_page_size=16384, write_batch_size=1024)),
    "wide_dict.parquet": (lambda: dict_table(150000, 100000, 6, 14, 34, 0.05),
                          dict(row_group_size=150000, dictionary_pagesize_limit=4 << 20, data_page_size=65536)),
}


def write(name):
    make, kw = FILES[name]
    path = os.path.join(HERE, name)
    pq.write_table(make(), path, compression="NONE", data_page_version="1.0", use_dictionary=True,
                   write_statistics=False, **kw)
    return path


def main():
    from oracle import oracle as O
    from util import file_chunks, oracle_read_column
    man = {"files": {}}
    for name in FILES:
        path = write(name)
        f = open(path, "rb").read()
        md = pq.ParquetFile(path).metadata
        entry = {"bytes": len(f), "row_groups": []}
        for rg in range(md.num_row_groups):
            cm = md.row_group(rg).column(0)
            encs = sorted(cm.encodings)
            chunks = file_chunks(f, 0)[rg:rg + 1]
            rc, msg, d = oracle_read_column(f, chunks)
            assert rc == 0, (name, rc, msg)
            entry["row_groups"].append({"encodings": list(encs), "len": len(d),
                                        "sha256": hashlib.sha256(d).hexdigest()})
        man["files"][name] = entry
        print(name, len(f), [r["encodings"] for r in entry["row_groups"]])
    with open(os.path.join(HERE, "manifest.json"), "w") as fp:
        json.dump(man, fp, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
