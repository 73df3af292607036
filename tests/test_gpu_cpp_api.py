"""GPU: the C++ mirror of the reference API (include/pqgpu/reader.hpp) and the
README CLI (pqgpu_parser), driven as separate processes like a user would."""
import os
import re
import struct
import subprocess

import numpy as np
import pytest

import pqbuild as B
from oracle import oracle as O
from pqgpu import capi, gen
from util import file_chunks, oracle_read_column, to_oracle_chunk

pytestmark = pytest.mark.gpu
BIN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "duckdb-parquet-parser_amd", "pqgpu")


def run(*args):
    return subprocess.run([os.path.join(BIN, args[0])] + list(args[1:]), capture_output=True, timeout=120)


@pytest.fixture(scope="module")
def mixed(tmp_path_factory):
    cols = gen.c4_cols()
    f = gen.build(cols, 3000, 2, seed=21, layout=gen.ARROW_LAYOUT, rows_per_page=700)
    path = str(tmp_path_factory.mktemp("api") / "mixed.parquet")
    with open(path, "wb") as fh:
        fh.write(f)
    return f, path, cols


def test_read_column_all_columns(mixed):
    f, path, cols = mixed
    for ci, c in enumerate(cols):
        r = run("api_check", path, "read_column", c.name)
        assert r.returncode == 0, r.stderr
        assert r.stdout == oracle_read_column(f, file_chunks(f, ci))[2]


def test_column_reader_and_read_pages(mixed):
    f, path, cols = mixed
    F = capi.File(f)
    for ci in (0, 3, 6, 7):
        r = run("api_check", path, "column_reader", "1", str(ci))
        assert r.returncode == 0, r.stderr
        rc, msg, col = O.read_all(f, to_oracle_chunk(F.chunk(1, ci)))
        assert r.stdout == O.dump_column(col)
        r = run("api_check", path, "read_pages", "1", str(ci))
        assert r.returncode == 0, r.stderr
        recs = [tuple(map(int, ln.split())) for ln in r.stderr.decode().splitlines()]
        assert recs == [(p[0], p[1], p[2], p[4]) for p in col.pages]
        assert r.stdout == O.dump_column(col)


def test_string_column_iterator(mixed):
    f, path, cols = mixed
    r = run("api_check", path, "iterator", "c6")
    assert r.returncode == 0, r.stderr
    rc, msg, d = oracle_read_column(f, file_chunks(f, 6))
    # rebuild (pos, len, bytes) of the non-null rows from the oracle dump
    exp = bytearray()
    i = row = 0
    while i < len(d):
        null = d[i]
        i += 1
        if not null:
            n = struct.unpack_from("<I", d, i)[0]
            exp += struct.pack("<QI", row, n) + d[i + 4:i + 4 + n]
            i += 4 + n
        row += 1
    assert r.stdout == bytes(exp)


def test_error_text_crosses_the_cpp_api(tmp_path):
    f, ch = B.build_file([B.data_header(9, 2, 0) + struct.pack("<I", 2) + b"ab" + b"\x09\x00\x00"],
                         gen.BYTE_ARRAY, False, 2)
    path = str(tmp_path / "bad.parquet")
    with open(path, "wb") as fh:
        fh.write(f)
    rc, msg, _ = oracle_read_column(f, [ch])
    r = run("api_check", path, "read_column", "c")
    assert r.returncode == 1
    assert r.stderr.decode().strip() == msg


def test_cli_regex_matches_golden(tmp_path):
    f = gen.build(gen.c3_cols(), 6000, 2, seed=31)
    path = str(tmp_path / "c3.parquet")
    with open(path, "wb") as fh:
        fh.write(f)
    F = capi.File(f)
    pidx = F.page_index()
    for pat, neg in [("special.*requests", False), ("e", True), ("^quickly ", False)]:
        args = ["pqgpu_parser", path, "--regex-column", "comment", "--regex", pat] + (["--neg-regex"] if neg else [])
        r = run(*args)
        assert r.returncode == 0, r.stderr
        got = [int(x) for x in r.stdout.decode().split("\n")[1:] if x.strip()]
        rx = re.compile(pat, re.ASCII)
        exp = []
        gid = 0
        for rg in range(F.num_row_groups):
            rc, msg, col = O.read_all(f, to_oracle_chunk(F.chunk(rg, 0)))
            for (_, pt, _, first, nrows) in col.pages:
                if pt != 0:
                    continue
                sat = any((rx.search(bytes(col.data[col.offsets[k]:col.offsets[k + 1]]).decode()) is not None) != neg
                          for k in range(first, first + nrows) if col.valid[k])
                if not sat:
                    exp.append(gid)
                gid += 1
        assert got == exp
    r = run("pqgpu_parser", path)
    assert r.returncode == 0 and b"comment (BYTE_ARRAY" in r.stdout
    assert r.stdout.count(b"\npage ") == len(pidx)


@pytest.mark.parametrize("k", [2, 3])
def test_read_column_sharded_over_devices(mixed, k):
    """ParquetReader::read_column(name, devices): every row group's chunk cut
    into k byte-balanced page ranges, one host thread per Device (here k
    contexts on the box's GPU(s)); == the oracle's read_column."""
    f, path, cols = mixed
    for ci, c in enumerate(cols):
        r = run("api_check", path, "sharded", c.name, str(k))
        assert r.returncode == 0, r.stderr
        assert r.stdout == oracle_read_column(f, file_chunks(f, ci))[2], c.name


def test_read_column_sharded_error_matches(tmp_path):
    f, ch = B.build_file([B.data_header(9, 2, 0) + struct.pack("<I", 2) + b"ab" + b"\x09\x00\x00"],
                         gen.BYTE_ARRAY, False, 2)
    path = str(tmp_path / "bad.parquet")
    with open(path, "wb") as fh:
        fh.write(f)
    rc, msg, _ = oracle_read_column(f, [ch])
    r = run("api_check", path, "sharded", "c", "2")
    assert r.returncode == 1
    assert r.stderr.decode().strip() == msg


def test_read_column_sharded_c2(tmp_path):
    cols = gen.c2_cols()
    n = 1_000_000
    f = gen.build(cols, n, 1, seed=gen.CONFIG_SEEDS["C2"], layout=gen.ARROW_LAYOUT)
    path = str(tmp_path / "c2.parquet")
    with open(path, "wb") as fh:
        fh.write(f)
    r = run("api_check", path, "sharded", cols[0].name, "4")
    assert r.returncode == 0, r.stderr
    assert r.stdout == gen.values_dump(cols[0], 0, n, 0, gen.CONFIG_SEEDS["C2"])


def _oracle_page_ids(f, col, pat, neg):
    """Global page ids (page index order) of column `col`'s data pages with no
    satisfying non-null value (README.md:54-64), from the oracle's decode."""
    F = capi.File(f)
    pidx = F.page_index()
    rx = re.compile(pat, re.ASCII)
    ids = [i for i in range(len(pidx)) if pidx[i][3] == col]
    out, k = [], 0
    for rg in range(F.num_row_groups):
        rc, msg, c = O.read_all(f, to_oracle_chunk(F.chunk(rg, col)))
        assert rc == 0, msg
        for (_, pt, _, first, nrows) in c.pages:
            if pt != 0:
                continue
            sat = any((rx.search(bytes(c.data[c.offsets[r]:c.offsets[r + 1]]).decode()) is not None) != neg
                      for r in range(first, first + nrows) if c.valid[r])
            if not sat:
                out.append(ids[k])
            k += 1
    return out


@pytest.mark.parametrize("k", [1, 2, 3])
@pytest.mark.parametrize("case", ["c2_ref", "c2_arrow", "c3_ref", "c4_dict", "c4_plain"])
def test_regex_pages_sharded_over_devices(tmp_path, case, k):
    """ParquetReader::regex_pages(name, pattern, neg, devices) and
    read_column_regex (decode + page filter per shard in one call): the page
    ids of the one-device filter / the oracle, the column of read_column, with
    every row group's chunk cut into k page ranges, one host thread per
    Device (k contexts on the box's GPU(s))."""
    if case.startswith("c2"):
        cols, n, rgs = gen.c2_cols(), 40000, 2
        f = gen.build(cols, n, rgs, seed=41, layout=gen.ARROW_LAYOUT if case == "c2_arrow" else gen.REF_LAYOUT,
                      rows_per_page=3000 if case == "c2_arrow" else 0)
        col, pats = 0, ["^qx", "e", "^[a-m]"]
    elif case == "c3_ref":
        cols = gen.c3_cols()
        f = gen.build(cols, 9000, 3, seed=42)
        col, pats = 0, ["special.*requests", "^(carefully|quickly) ", "e"]
    else:
        cols = gen.c4_cols()
        f = gen.build(cols, 4000, 2, seed=43, layout=gen.ARROW_LAYOUT, rows_per_page=700)
        col, pats = (6 if case == "c4_dict" else 7), ["^[a-d]", "e", "ly"]
    path = str(tmp_path / f"{case}.parquet")
    with open(path, "wb") as fh:
        fh.write(f)
    name = cols[col].name
    d_o = oracle_read_column(f, file_chunks(f, col))[2]
    for pat in pats:
        for neg in (False, True):
            exp = _oracle_page_ids(f, col, pat, neg)
            r = run("api_check", path, "regex_sharded", name, str(k), pat, str(int(neg)))
            assert r.returncode == 0, r.stderr
            assert [int(x) for x in r.stdout.split()] == exp, (pat, neg)
            r = run("api_check", path, "decode_regex_sharded", name, str(k), pat, str(int(neg)))
            assert r.returncode == 0, r.stderr
            assert r.stdout == d_o, (pat, neg)
            assert [int(x) for x in r.stderr.split()] == exp, (pat, neg)


@pytest.mark.parametrize("mode", ["regex_sharded", "decode_regex_sharded"])
def test_regex_sharded_error_matches(tmp_path, mode):
    """A page that cannot be decoded: the sharded filter reports the
    reference's first error, as the one-device call does."""
    good = B.plain_ba([b"special requests", b"quick"] * 20)
    bad = struct.pack("<I", 7) + b"special" + struct.pack("<I", 50) + b"xy"
    pages = [B.data_header(len(good), 40, 0) + good] * 3 + [B.data_header(len(bad), 2, 0) + bad] + \
            [B.data_header(len(good), 40, 0) + good] * 2
    f, ch = B.build_file(pages, gen.BYTE_ARRAY, False, 202)
    path = str(tmp_path / "bad.parquet")
    with open(path, "wb") as fh:
        fh.write(f)
    rc, msg, _ = oracle_read_column(f, [ch])
    assert rc != 0
    for k in (1, 2, 3):
        r = run("api_check", path, mode, "c", str(k), "special", "0")
        assert r.returncode == 1, (k, r.stderr)
        assert r.stderr.decode().strip().splitlines()[-1] == msg, k
