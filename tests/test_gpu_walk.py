"""GPU: the device page walk (pq_build_page_table_device, walk.hip) against
the host walk (pq_build_page_table, itself pinned to the reference's
ColumnReader walk by test_oracle_golden.py).

Whenever the device walk settles a chunk it must list exactly the host
walk's pages (every pq_page_desc field); where it refuses (status -8) the
caller walks on the host.  It must refuse every chunk whose host walk fails
(the host reports the reference's error), so the mutated fixtures of
test_fuzz_host.py check that no corrupt chain is ever listed."""
import glob
import os

import pytest

from pqgpu import capi, gen
from test_fuzz_host import _mutants
from util import to_desc
from oracle import oracle as O

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIELDS = [f for f, _ in capi.PageDesc._fields_]


def rows(table):
    return [tuple(getattr(p, f) for f in FIELDS) for p in table]


_CTX = []


def on_device(data: bytes):
    return _CTX[0].device_buffer(data)


def check(ctx, f: bytes, ch, segs=(512, 2048, 8192), base=0, dev=None):
    """Device vs host walk of one chunk; returns how many seg sizes settled it."""
    _CTX[:] = [ctx]
    rc_h, _, host = capi.build_page_table(f, ch)
    if dev is None:
        dev = on_device(f[base:])
    settled = 0
    for seg in segs:
        rc_d, pages = ctx.build_page_table_device(dev.data_ptr(), len(f) - base, base, ch, seg_bytes=seg)
        assert rc_d in (0, -8), rc_d
        if rc_d == 0:
            assert rc_h == 0, ("device listed a chunk the host walk fails", seg, rc_h)
            assert rows(pages) == rows(host), seg
            settled += 1
    return settled


def test_golden_fixtures(ctx):
    n_settled = n_chunks = 0
    for path in sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "**", "*.parquet"), recursive=True)):
        with open(path, "rb") as fh:
            f = fh.read()
        try:
            F = capi.File(f)
        except capi.PqError:
            continue
        _CTX[:] = [ctx]
        dev = on_device(f)
        for rg in range(F.num_row_groups):
            for col in range(F.num_columns):
                try:
                    ch = F.chunk(rg, col)
                except capi.PqError:
                    continue
                n_chunks += 1
                n_settled += check(ctx, f, ch, dev=dev) > 0
    assert n_chunks > 50 and n_settled > n_chunks // 3, (n_settled, n_chunks)


@pytest.mark.parametrize("cfg,layout,rows_", [("c2", gen.REF_LAYOUT, 200_000), ("c3", gen.REF_LAYOUT, 100_000),
                                              ("c2", gen.ARROW_LAYOUT, 200_000), ("c4", gen.ARROW_LAYOUT, 60_000)])
def test_generated_extent_only(ctx, cfg, layout, rows_):
    """The raw-upload shape: only the chunk's extent in device memory (base =
    the chunk's first byte, zeros past its end); ref-layout chunks settle at
    every segment size, arrow-layout pages longer than a segment refuse at
    small sizes and settle at large ones."""
    cols = {"c2": gen.c2_cols, "c3": gen.c3_cols, "c4": gen.c4_cols}[cfg]()
    seed = gen.CONFIG_SEEDS[cfg.upper()]
    f = gen.build(cols, rows_, 2, seed=seed, layout=layout)
    F = capi.File(f)
    settled = 0
    for rg in range(F.num_row_groups):
        for col in range(F.num_columns):
            ch = F.chunk(rg, col)
            start = min(ch.data_page_offset, ch.dictionary_page_offset) if ch.has_dictionary_page_offset else ch.data_page_offset
            ext = f[:start + ch.total_compressed_size]
            settled += check(ctx, ext, ch, segs=(1024, 8192, 262144), base=start)
    assert settled > 0


def test_full_size_c2_c3(ctx):
    """BASELINE configs 2 and 3 at 10M rows: settled at the default segment
    size, same table as the host walk."""
    for cols, seed in ((gen.c2_cols(), gen.CONFIG_SEEDS["C2"]), (gen.c3_cols(), gen.CONFIG_SEEDS["C3"])):
        f = gen.build(cols, 10_000_000, 1, seed=seed)
        ch = capi.File(f).chunk(0, 0)
        assert check(ctx, f, ch, segs=(0,)) == 1


def test_mutants_never_listed_wrong(ctx):
    """Mutated headers and payloads: the device walk lists the host walk's
    pages or refuses; it never lists a chunk whose host walk fails."""
    settled = 0
    for name, f, c in _mutants(200, seed=29):
        ch = to_desc(O.Chunk(*c))  # _mutants yields the manifest's chunk list
        settled += check(ctx, bytes(f), ch, segs=(256, 4096)) > 0
    assert settled > 0


def _decode_all(ctx, f, opt):
    """Every chunk of `f` uploaded with device_walk = opt: (rc, canonical bytes)."""
    ctx.set_option("device_walk", opt)
    try:
        try:
            F = capi.File(f)
        except capi.PqError as e:
            return [("file", str(e))]
        out = []
        for rg in range(F.num_row_groups):
            for col in range(F.num_columns):
                try:
                    ch = F.chunk(rg, col)
                except capi.PqError as e:
                    out.append(("chunk", str(e)))
                    continue
                try:
                    dc = ctx.upload(f, [ch])
                    dc.decode()
                    h = dc.to_host()
                    out.append((h.validity.tobytes(), h.data.tobytes(),
                                None if h.offsets is None else h.offsets.tobytes()))
                    dc.free()
                except capi.PqError as e:
                    out.append(("err", e.code, str(e)))
        return out
    finally:
        ctx.set_option("device_walk", 0)


@pytest.mark.parametrize("kind", ["golden", "generated", "mutants"])
def test_upload_option_device_walk(ctx, kind):
    """pq_chunk_upload with the device_walk option: the same decode (or the
    same error) as the host-walked upload, on the golden fixtures, generated
    ref/arrow files and mutated fixtures (refused chunks walk on the host)."""
    files = []
    if kind == "golden":
        for path in sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "*.parquet")))[:40]:
            with open(path, "rb") as fh:
                files.append(fh.read())
    elif kind == "generated":
        for cols, seed, layout in ((gen.c2_cols(), 2, gen.REF_LAYOUT), (gen.c3_cols(), 3, gen.REF_LAYOUT),
                                   (gen.c2_cols(), 2, gen.ARROW_LAYOUT)):
            files.append(gen.build(cols, 150_000, 2, seed=seed, layout=layout))
    else:
        files = [f for _, f, _ in _mutants(40, seed=31)]
    for f in files:
        assert _decode_all(ctx, f, 1) == _decode_all(ctx, f, 0)


def test_walk_buffers_survive_raw_regrowth():
    """A device walk, then an upload whose raw extent is larger than any
    before (the raw buffer regrows), then device walks again and the context
    is destroyed: the walk's buffers stay the walk's own (round-5 advice: the
    raw regrowth used to free them behind the walk's back)."""
    ctx = capi.Context(0)
    try:
        ctx.set_option("device_walk", 1)
        small = gen.build(gen.c2_cols(), 20_000, 1, seed=2)
        big = gen.build(gen.c2_cols(), 600_000, 1, seed=2)
        want = {}
        for f in (small, big, small, big):
            ch = capi.File(f).chunk(0, 0)
            dc = ctx.upload(f, [ch])
            dc.decode()
            h = dc.to_host()
            got = (h.validity.tobytes(), h.data.tobytes(), h.offsets.tobytes())
            assert want.setdefault(len(f), got) == got
            dc.free()
            assert check(ctx, f, ch, segs=(0, 2048)) >= 1
    finally:
        ctx.set_option("device_walk", 0)
        ctx.close()
