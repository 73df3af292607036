"""GPU parity on repeated columns (SURVEY §8a R-LEVELS, max_rep > 0): the
pyarrow LIST fixtures (tests/golden/lists) on every decode path, every regex
page kernel and page-range shards, against the oracle (pinned to the
compiled reference by test_lists.py).  The crafted max_rep pages run through
test_gpu_decode.py's CRAFTED / ERRORS on every path."""
import numpy as np
import pytest

from lists_util import NAMES, STRING_NAMES, load, manifest, sha
from pqgpu import capi, shard
from test_gpu_regex import golden_pages
from util import file_chunks, gpu_read_column, oracle_read_column

pytestmark = pytest.mark.gpu
MAN = manifest()


@pytest.mark.parametrize("name", NAMES)
def test_decode_every_path(ctx, path, name):
    f = load(name)
    chunks = file_chunks(f, 0)
    for rg, ch in enumerate(chunks):
        rc, msg, d = gpu_read_column(ctx, f, [ch])
        exp = MAN["files"][name]["row_groups"][rg]
        assert (rc != 0, msg) == (exp["rc"] != 0, exp["msg"]), (name, rg, path)
        if rc == 0:
            assert len(d) == exp["len"] and sha(d) == exp["sha256"], (name, rg, path)
    rc_o, msg_o, d_o = oracle_read_column(f, chunks)
    rc_g, msg_g, d_g = gpu_read_column(ctx, f, chunks)
    assert (rc_g, msg_g, d_g) == (rc_o, msg_o, d_o)


@pytest.mark.parametrize("neg", [False, True], ids=["like", "notlike"])
@pytest.mark.parametrize("name", STRING_NAMES)
def test_regex_every_kernel(ctx, kernel, name, neg):
    f = load(name)
    chunks = file_chunks(f, 0)
    dc = ctx.upload(f, chunks)
    try:
        for p in ("^[a-f]", "qz", "e", "^[a-z]{8,12}$", "x*", "(ab|cd).*e$"):
            exp = golden_pages(f, chunks, p, neg)
            got = dc.regex_pages(p, neg)
            assert len(got) == len(exp)
            bad = np.nonzero(got != exp)[0]
            assert len(bad) == 0, (p, neg, bad[:10])
    finally:
        dc.free()


@pytest.mark.parametrize("neg", [False, True], ids=["like", "notlike"])
@pytest.mark.parametrize("name", STRING_NAMES)
def test_decode_regex_one_call(ctx, name, neg):
    f = load(name)
    chunks = file_chunks(f, 0)
    _, _, d_o = oracle_read_column(f, chunks)
    dc = ctx.upload(f, chunks)
    try:
        for p in ("^[a-f]", "e"):
            dc.decode_regex_async(p, neg)
            got = dc.regex_pages_result()
            dc.decode_check()
            assert np.array_equal(got, golden_pages(f, chunks, p, neg)), (p, neg)
            assert capi.canonical_dump(dc.to_host()) == d_o
    finally:
        dc.free()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("name", NAMES)
def test_page_range_shards(ctx, name, world):
    f = load(name)
    ch = capi.File(f).chunk(0, 0)
    rc, msg, table = capi.build_page_table(f, ch)
    assert rc == 0, msg
    _, _, d_o = oracle_read_column(f, [ch])
    parts = []
    for b, e in shard.data_page_ranges(table, world):
        dc = ctx.upload_range(f, ch, table, b, e)
        try:
            dc.decode()
            parts.append(capi.canonical_dump(dc.to_host()))
        finally:
            dc.free()
    assert b"".join(parts) == d_o
