"""GPU: page-range shards (pq_chunk_upload_range) decoded one
after another on one GPU; the concatenation of the shards' canonical dumps
must equal the unsharded result byte for byte (the oracle's dump at small
sizes, the generator's oracle-pinned value dump at C2's full 10M rows), and
the shards' regex page flags concatenated must equal the whole chunk's.
Reference: pages decode independently given their chunk's dictionary
(/root/reference/src/reader/column_reader.cpp:140-225); the shard unit is the
global data-page id (/root/reference/src/reader/parquet_reader.cpp:559-605)."""
import hashlib

import numpy as np
import pytest

from pqgpu import capi, gen
from pqgpu.shard import column_page_shards, data_page_ranges, range_rows
from util import file_chunks, oracle_read_column

pytestmark = pytest.mark.gpu


def _decode_shards(ctx, f, ch, table, ranges, pattern=None):
    dumps, flags = [], []
    for a, b in ranges:
        dc = ctx.upload_range(f, ch, table, a, b)
        first, cnt = range_rows(table, a, b)
        assert dc.num_rows == cnt and dc.first_row == first
        dc.decode()
        dumps.append(capi.canonical_dump(dc.to_host()))
        if pattern is not None:
            flags.append(dc.regex_pages(pattern))
        dc.free()
    return dumps, flags


@pytest.mark.parametrize("layout", [gen.REF_LAYOUT, gen.ARROW_LAYOUT])
@pytest.mark.parametrize("world", [2, 4, 8])
def test_c2_full_size_page_shards(ctx, layout, world):
    cols = gen.c2_cols()
    n = 10_000_000
    f = gen.build(cols, n, 1, seed=gen.CONFIG_SEEDS["C2"], layout=layout)
    ch = capi.File(f).chunk(0, 0)
    rc, msg, table = capi.build_page_table(f, ch)
    assert rc == 0, msg
    ranges = data_page_ranges(table, world)
    dumps, _ = _decode_shards(ctx, f, ch, table, ranges)
    h = hashlib.sha256()
    for d in dumps:
        h.update(d)
    exp = hashlib.sha256(gen.values_dump(cols[0], 0, n, 0, gen.CONFIG_SEEDS["C2"])).hexdigest()
    assert h.hexdigest() == exp


@pytest.mark.parametrize("world", [2, 4, 8])
def test_c4_page_shards_vs_oracle(ctx, world):
    cols = gen.c4_cols()
    f = gen.build(cols, 200_000, 2, seed=gen.CONFIG_SEEDS["C4"], layout=gen.ARROW_LAYOUT, rows_per_page=6000)
    F = capi.File(f)
    pidx = F.page_index()
    for ci in range(len(cols)):
        rc, msg, exp = oracle_read_column(f, file_chunks(f, ci))
        assert rc == 0, msg
        got = []
        for pieces in column_page_shards(pidx, ci, world):
            for rg, a, b in pieces:
                ch = F.chunk(rg, ci)
                rc, msg, table = capi.build_page_table(f, ch)
                assert rc == 0, msg
                d, _ = _decode_shards(ctx, f, ch, table, [(a, b)])
                got += d
        assert b"".join(got) == exp, cols[ci].name


@pytest.mark.parametrize("layout", [gen.REF_LAYOUT, gen.ARROW_LAYOUT])
@pytest.mark.parametrize("cfg", ["c2", "c3"])
def test_shard_regex_flags_equal_whole(ctx, layout, cfg):
    cols = gen.c2_cols() if cfg == "c2" else gen.c3_cols()
    f = gen.build(cols, 300_000, 1, seed=7, layout=layout, rows_per_page=0 if layout == gen.REF_LAYOUT else 4000)
    ch = capi.File(f).chunk(0, 0)
    rc, msg, table = capi.build_page_table(f, ch)
    assert rc == 0, msg
    pat = "ab" if cfg == "c2" else "special.*requests"
    whole = ctx.upload(f, [ch])
    whole.decode()
    wdump = capi.canonical_dump(whole.to_host())
    wflags = whole.regex_pages(pat)
    whole.free()
    for world in (2, 5):
        dumps, flags = _decode_shards(ctx, f, ch, table, data_page_ranges(table, world), pattern=pat)
        assert b"".join(dumps) == wdump
        assert np.array_equal(np.concatenate(flags), wflags)


def test_empty_and_single_page_ranges(ctx):
    f = gen.build(gen.c2_cols(), 5000, 1, seed=3)
    ch = capi.File(f).chunk(0, 0)
    rc, msg, table = capi.build_page_table(f, ch)
    ndata = sum(1 for p in table if p.page_type == 0)
    rc, msg, exp = oracle_read_column(f, [ch])
    dumps, _ = _decode_shards(ctx, f, ch, table, [(0, 0), (0, 1)] + [(i, i + 1) for i in range(1, ndata)] + [(ndata, ndata)])
    assert b"".join(dumps) == exp
    with pytest.raises(capi.PqError):
        ctx.upload_range(f, ch, table, 0, ndata + 1)


@pytest.mark.parametrize("layout", [gen.REF_LAYOUT, gen.ARROW_LAYOUT])
def test_two_threads_two_contexts(layout):
    """Two host threads, each driving its own context (one per device in a
    multi-GPU run; both on this box's GPU here), decode alternate page ranges
    of one chunk concurrently, several rounds; the joined shards == the whole
    chunk (generator's oracle-pinned dump)."""
    import threading
    cols = gen.c2_cols()
    n = 2_000_000
    f = gen.build(cols, n, 1, seed=gen.CONFIG_SEEDS["C2"], layout=layout)
    ch = capi.File(f).chunk(0, 0)
    rc, msg, table = capi.build_page_table(f, ch)
    assert rc == 0, msg
    ranges = data_page_ranges(table, 8)
    ctxs = [capi.Context(0), capi.Context(0)]
    out = [None] * len(ranges)
    errs = []

    def work(t):
        try:
            for rnd in range(3):
                for i in range(t, len(ranges), 2):
                    dc = ctxs[t].upload_range(f, ch, table, *ranges[i])
                    dc.decode()
                    d = capi.canonical_dump(dc.to_host())
                    assert out[i] is None or out[i] == d
                    out[i] = d
                    dc.free()
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    th = [threading.Thread(target=work, args=(t,)) for t in range(2)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    for c in ctxs:
        c.close()
    assert not errs, errs
    exp = hashlib.sha256(gen.values_dump(cols[0], 0, n, 0, gen.CONFIG_SEEDS["C2"])).hexdigest()
    assert hashlib.sha256(b"".join(out)).hexdigest() == exp
