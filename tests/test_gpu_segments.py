"""GPU parity: the segmented pipe decode (capi.hip pipe_segmented, options
pipe_segs / pipe_seg_min_tiles) against the oracle.

A segmented decode cuts the writer grid into K ranges of workgroups: segment
k's run-table and code passes run on the context's stream while segment
k - 1's write pass runs on a second stream.  Whatever K, the column must be
the oracle's byte for byte: pages the exact decoder takes in any segment,
pages of several tiles that straddle a segment boundary, out-of-range
indices, the dictionary decoded on the side stream, the armed page filter
(decode + regex in one pass), and repeated decodes (the per-decode zero
block the last writer clears for the next decode).  The full-size C2 decode
with the default four segments is test_gpu_decode.py's
test_c2_full_size_properties."""
import numpy as np
import pytest

import pqbuild as B
from pqgpu import capi, gen
from test_gpu_decode import _hybrid
from test_gpu_regex import golden_pages
from util import file_chunks, oracle_read_column, to_desc

pytestmark = pytest.mark.gpu

SEGS = [1, 2, 3, 5, 16]


@pytest.fixture
def segs(request, ctx):
    ctx.set_option("pipe_seg_min_tiles", 1)
    yield
    ctx.set_option("pipe_segs", 1)
    ctx.set_option("pipe_seg_min_tiles", 1024)
    ctx.set_option("pipe_run_dict", 1)


def _decode_n(ctx, f, chunks, times=3):
    dc = ctx.upload(f, [to_desc(c) for c in chunks])
    try:
        out = []
        for _ in range(times):
            dc.decode()
            out.append(capi.canonical_dump(dc.to_host()))
        return out
    finally:
        dc.free()


def _mixed_pages_file(npages: int, seed: int, optional: bool):
    """`npages` dictionary-encoded pages of 200-512 rows: runs of repeated
    indices, some past the 300-entry dictionary (NULL rows), every 37th page
    with a zero-count run after its first literal run (the exact decoder), every 41st with a 17-bit index
    width (the exact decoder), 10 % NULL when optional."""
    rng = np.random.default_rng(seed)
    dv = [b"e%d-" % i * (1 + i % 4) for i in range(300)]
    dpay = B.plain_ba(dv)
    pages = [B.dict_header(len(dpay), len(dv)) + dpay]
    total = 0
    for k in range(npages):
        n = int(rng.integers(200, 513)) if k % 5 else 512
        idx = []
        while len(idx) < n:
            idx += [int(rng.integers(0, 310))] * int(rng.integers(1, 12))
        idx = idx[:n]
        defs = None
        if optional:
            defs = [int(x) for x in rng.random(n) > 0.1]
            idx = [v for v, d in zip(idx, defs) if d]
        bw = 17 if k % 41 == 7 else 9
        if k % 37 == 5:  # a zero-count run after a literal run
            stream = bytes([bw]) + B.bitpack(idx[:8], bw) + B.rle(0, 1, bw) + _hybrid(idx[8:], bw, rng, 20)
        else:
            stream = bytes([bw]) + _hybrid(idx, bw, rng, 20)
        pay = (B.levels_section(_hybrid(defs, 1, rng)) if optional else b"") + stream
        pages.append(B.data_header(len(pay), n, 8) + pay)
        total += n
    return B.build_file(pages, gen.BYTE_ARRAY, optional, total, dict_at_start=True)


@pytest.mark.parametrize("k", SEGS)
def test_c2_shape_segments(ctx, segs, k):
    """The C2 shape (ref layout, 512-row OPTIONAL pages): every segment count
    equals the oracle on three decodes of one upload."""
    ctx.set_option("pipe_segs", k)
    f = gen.build(gen.c2_cols(), 300_000, 1, seed=21)
    chunks = file_chunks(f, 0)
    rc, msg, want = oracle_read_column(f, chunks)
    assert rc == 0, msg
    for got in _decode_n(ctx, f, chunks):
        assert got == want, k


@pytest.mark.parametrize("k", SEGS)
@pytest.mark.parametrize("optional", [False, True], ids=["required", "optional"])
def test_exact_pages_in_segments(ctx, segs, k, optional):
    """Pages the exact decoder takes, spread over every segment: each is
    decoded by its own segment's code pass before that segment's writer."""
    ctx.set_option("pipe_segs", k)
    f, chunk = _mixed_pages_file(420, seed=5 + k, optional=optional)
    rc, msg, want = oracle_read_column(f, [chunk])
    assert rc == 0, msg
    for got in _decode_n(ctx, f, [chunk], 2):
        assert got == want, (k, optional)


@pytest.mark.parametrize("k", [3, 16])
def test_multi_tile_pages_straddle(ctx, segs, k):
    """REQUIRED pages of 2,000 rows (four tiles): segment boundaries fall
    inside pages; a page's run table comes from the segment holding its first
    tile, its later tiles decode in the next segment."""
    ctx.set_option("pipe_segs", k)
    cols = [gen.Col("s", gen.DICT_STRINGS, gen.BYTE_ARRAY, dict_size=500, len_min=1, len_max=30, max_run=9)]
    f = gen.build(cols, 400_000, 1, seed=8, layout=gen.ARROW_LAYOUT, rows_per_page=2000)
    chunks = file_chunks(f, 0)
    rc, msg, want = oracle_read_column(f, chunks)
    assert rc == 0, msg
    for got in _decode_n(ctx, f, chunks, 2):
        assert got == want


@pytest.mark.parametrize("run_dict", [0, 1], ids=["side_stream", "in_runs"])
def test_dictionary_placement(ctx, segs, run_dict):
    ctx.set_option("pipe_segs", 5)
    ctx.set_option("pipe_run_dict", run_dict)
    f = gen.build(gen.c2_cols(), 200_000, 2, seed=23)
    chunks = file_chunks(f, 0)
    rc, msg, want = oracle_read_column(f, chunks)
    assert rc == 0, msg
    for got in _decode_n(ctx, f, chunks):
        assert got == want


@pytest.mark.parametrize("neg", [False, True])
def test_armed_filter_segments(ctx, segs, neg):
    """Decode + page filter in one pass over a segmented decode: the flags
    equal the oracle's, the column the plain decode's; a regex scan over the
    codes afterwards agrees too."""
    ctx.set_option("pipe_segs", 3)
    f = gen.build(gen.c2_cols(), 250_000, 1, seed=29)
    chunks = file_chunks(f, 0)
    rc, msg, want = oracle_read_column(f, chunks)
    assert rc == 0, msg
    dc = ctx.upload(f, [to_desc(c) for c in chunks])
    try:
        for p in ("^qx", "e", "a.{3}e"):
            exp = golden_pages(f, chunks, p, neg)
            dc.decode_regex_async(p, neg)
            got = dc.regex_pages_result()
            dc.decode_check()
            assert np.array_equal(got, exp), (p, neg)
            assert capi.canonical_dump(dc.to_host()) == want
            assert np.array_equal(dc.regex_pages(p, neg), exp)
    finally:
        dc.free()

