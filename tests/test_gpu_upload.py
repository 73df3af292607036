"""GPU: the upload paths give the same device image and
so the same decode.  raw_upload=1 sends a chunk's raw byte extent to HBM
during the host walk and builds the slot image with k_relayout; 0 builds it
on the host.  Extents that are too short (payloads outside them) fall back to
the host image; too long ones are cut at EOF.  Decodes are checked against
the oracle (the reference's ColumnReader::read_all restated,
/root/reference/src/reader/column_reader.cpp:18-71)."""
import ctypes as C

import numpy as np
import pytest

from pqgpu import capi, gen
from pqgpu.shard import data_page_ranges
from util import oracle_read_column

pytestmark = pytest.mark.gpu


def _desc(ch, total):
    d = capi.ChunkDesc()
    C.memmove(C.byref(d), C.byref(ch), C.sizeof(ch))
    d.total_compressed_size = total
    return d


def _decode(ctx, f, chunks, raw, stage=None):
    ctx.set_option("raw_upload", raw)
    if stage:
        ctx.set_option("stage_bufs", stage[0])
        ctx.set_option("stage_piece_kb", stage[1])
    try:
        dc = ctx.upload(f, chunks)
        dc.decode()
        out = capi.canonical_dump(dc.to_host())
        flags = dc.regex_pages("e.*a") if chunks[0].type == capi.BYTE_ARRAY else None
        dc.free()
        return out, flags
    finally:
        ctx.set_option("raw_upload", 1)
        ctx.set_option("stage_bufs", 6)
        ctx.set_option("stage_piece_kb", 8192)


CASES = {
    "c2_ref": lambda: gen.build(gen.c2_cols(), 200_000, 1, seed=2),
    "c2_arrow_2rg": lambda: gen.build(gen.c2_cols(), 100_000, 2, seed=2, layout=gen.ARROW_LAYOUT, rows_per_page=7000),
    "c3_ref": lambda: gen.build(gen.c3_cols(), 100_000, 1, seed=3),
    "c4_3rg": lambda: gen.build(gen.c4_cols(), 30_000, 3, seed=4, layout=gen.ARROW_LAYOUT, rows_per_page=4000),
}


@pytest.mark.parametrize("name", list(CASES))
def test_raw_and_host_images_decode_alike(ctx, name):
    f = CASES[name]()
    F = capi.File(f)
    for col in range(F.num_columns):
        chunks = [F.chunk(rg, col) for rg in range(F.num_row_groups)]
        assert all(c.total_compressed_size > 0 for c in chunks)
        rc, msg, exp = oracle_read_column(f, chunks)
        assert rc == 0, msg
        a, fa = _decode(ctx, f, chunks, 1)
        b, fb = _decode(ctx, f, chunks, 0)
        c, fc = _decode(ctx, f, chunks, 1, stage=(2, 64))  # many tiny pieces through a 2-buffer ring
        assert a == exp and b == exp and c == exp
        if fa is not None:
            assert np.array_equal(fa, fb) and np.array_equal(fa, fc)


def test_extent_hints_wrong(ctx):
    f = CASES["c3_ref"]()
    ch = capi.File(f).chunk(0, 0)
    rc, msg, exp = oracle_read_column(f, [ch])
    for total in (ch.total_compressed_size // 2, 17, ch.total_compressed_size * 3, len(f) * 2):
        a, _ = _decode(ctx, f, [_desc(ch, total)], 1)
        assert a == exp, total


def test_truncated_file_raw_upload(ctx):
    """Payloads past EOF read as zeros (the reference's zero-padding
    ReadRangeFunc): the same on both image paths."""
    f = CASES["c2_ref"]()
    ch = capi.File(f).chunk(0, 0)
    cut = f[: len(f) * 2 // 3]
    res = []
    for raw in (1, 0):
        ctx.set_option("raw_upload", raw)
        try:
            dc = ctx.upload(cut, [ch])
            try:
                dc.decode()
                res.append(("ok", capi.canonical_dump(dc.to_host())))
            except capi.PqError as e:
                res.append(("err", e.code, e.msg))
            dc.free()
        except capi.PqError as e:
            res.append(("upload_err", e.code, e.msg))
        finally:
            ctx.set_option("raw_upload", 1)
    assert res[0] == res[1]
    rc, msg, exp = oracle_read_column(cut, [ch])
    if rc == 0:
        assert res[0] == ("ok", exp)
    else:
        assert res[0][0] != "ok" and res[0][2] == msg


def test_page_range_raw_upload(ctx):
    f = CASES["c2_ref"]()
    ch = capi.File(f).chunk(0, 0)
    rc, msg, table = capi.build_page_table(f, ch)
    rc, msg, exp = oracle_read_column(f, [ch])
    for raw in (1, 0):
        ctx.set_option("raw_upload", raw)
        parts = []
        for a, b in data_page_ranges(table, 3):
            dc = ctx.upload_range(f, ch, table, a, b)
            dc.decode()
            parts.append(capi.canonical_dump(dc.to_host()))
            dc.free()
        ctx.set_option("raw_upload", 1)
        assert b"".join(parts) == exp
