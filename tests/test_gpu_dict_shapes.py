"""GPU parity on the real-world dictionary fixtures (tests/golden/dict_shapes):
chunks whose dictionary-encoded pages are followed by PLAIN pages, and
dictionaries over 64 KiB / 65,535 entries.  Every decode path and every regex
page kernel against the oracle (pinned to the compiled reference and pyarrow
by test_dict_shapes.py); page-range shards of the mixed chunks too."""
import numpy as np
import pytest

from dict_shapes_util import NAMES, load, manifest, sha
from pqgpu import capi, shard
from test_gpu_regex import PATTERNS, golden_pages
from util import file_chunks, gpu_read_column, oracle_read_column

pytestmark = pytest.mark.gpu
MAN = manifest()


@pytest.mark.parametrize("name", NAMES)
def test_decode_every_path(ctx, path, name):
    f = load(name)
    chunks = file_chunks(f, 0)
    for rg, ch in enumerate(chunks):
        rc, msg, d = gpu_read_column(ctx, f, [ch])
        assert (rc, msg) == (0, ""), (name, rg, msg)
        exp = MAN["files"][name]["row_groups"][rg]
        assert len(d) == exp["len"] and sha(d) == exp["sha256"], (name, rg, path)
    # the whole column in one upload (row groups concatenated)
    rc_o, _, d_o = oracle_read_column(f, chunks)
    assert gpu_read_column(ctx, f, chunks) == (rc_o, "", d_o)


@pytest.mark.parametrize("neg", [False, True], ids=["like", "notlike"])
@pytest.mark.parametrize("name", NAMES)
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


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("name", ["fallback_opt.parquet", "fallback_req.parquet", "wide_dict.parquet"])
def test_page_range_shards(ctx, name, world):
    """Shards of a chunk cut across its dictionary and PLAIN pages decode to
    the rows of the unsharded oracle dump."""
    f = load(name)
    F = capi.File(f)
    ch = F.chunk(0, 0)
    rc, msg, table = capi.build_page_table(f, ch)
    assert rc == 0
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
