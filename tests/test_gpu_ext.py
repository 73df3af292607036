"""GPU parity for the extended format scope: compressed
pages (SNAPPY, GZIP, LZ4_RAW, ZSTD; codec.hip) and DATA_PAGE_V2 pages, decoded
through the C ABI with PQ_EXT_* flags and compared bit for bit with pyarrow's
reading of the same file (the oracle for this row; the reference decodes
neither).  Expectations: tests/golden/ext/manifest.json (make_ext.py)."""
import os
import sys

import numpy as np
import pytest

from ext_util import EXT_ALL, ext_chunks, load, manifest, sha
from pqgpu import capi

pytestmark = pytest.mark.gpu
MAN = manifest()
FILES = sorted(MAN["files"])
COLS = ["s_dict", "s_plain", "i64", "f64", "i32d", "b"]


def decode(ctx, f, col, flags=EXT_ALL):
    dc = ctx.upload(f, ext_chunks(f, col, flags))
    try:
        dc.decode()
        return dc.to_host()
    finally:
        dc.free()


@pytest.mark.parametrize("name", FILES)
@pytest.mark.parametrize("ci", range(len(COLS)))
def test_ext_decode_matches_pyarrow(ctx, name, ci):
    f = load(name)
    got = capi.canonical_dump(decode(ctx, f, ci))
    exp = MAN["files"][name]["columns"][COLS[ci]]
    assert len(got) == exp["len"] and sha(got) == exp["sha256"], (name, COLS[ci])


@pytest.mark.parametrize("version", ["1", "2"])
def test_ext_regex_same_across_codecs(ctx, version):
    """The regex page filter on a compressed chunk equals the one on the
    uncompressed file (same table, same page boundaries)."""
    for pattern, neg in (("^[a-d][a-e]", False), ("q", True), ("x.*y", False)):
        base = None
        for codec in ("none", "snappy", "gzip", "lz4", "zstd"):
            f = load(f"ext_{codec}_v{version}.parquet")
            dc = ctx.upload(f, ext_chunks(f, 1))
            try:
                flags = dc.regex_pages(pattern, neg)
            finally:
                dc.free()
            if base is None:
                base = flags
                assert len(flags) > 8
            else:
                assert np.array_equal(flags, base), (pattern, codec)


def test_ext_repeat_uploads(ctx):
    """The codec pass reuses its context buffers across uploads of different sizes."""
    for name in ("ext_gzip_v1.parquet", "ext_snappy_v2.parquet", "ext_lz4_v1.parquet", "ext_gzip_v2.parquet",
                 "ext_zstd_v1.parquet", "ext_zstd_v2.parquet"):
        f = load(name)
        got = capi.canonical_dump(decode(ctx, f, 0))
        assert sha(got) == MAN["files"][name]["columns"]["s_dict"]["sha256"]


def test_ext_host_fill_path(ctx):
    """Without the raw-upload path (option raw_upload = 0) the compressed
    payloads are gathered and uploaded separately: same result."""
    ctx.set_option("raw_upload", 0)
    try:
        for name in ("ext_snappy_v1.parquet", "ext_gzip_v2.parquet"):
            f = load(name)
            for ci in (0, 1, 5):
                got = capi.canonical_dump(decode(ctx, f, ci))
                assert sha(got) == MAN["files"][name]["columns"][COLS[ci]]["sha256"]
    finally:
        ctx.set_option("raw_upload", 1)


@pytest.mark.parametrize("name", ["ext_snappy_v1.parquet", "ext_gzip_v1.parquet", "ext_lz4_v2.parquet",
                                  "ext_zstd_v1.parquet"])
def test_ext_corrupt_page_fails_cleanly(ctx, name):
    """Damaged compressed bytes end in an error (decompression or decode), never a fault."""
    f = bytearray(load(name))
    d = ext_chunks(bytes(f), 1)[0]
    rc, msg, table = capi.build_page_table(bytes(f), d)
    assert rc == 0
    p = [q for q in table if q.page_type == 0][1]
    rng = np.random.default_rng(5)
    for k in rng.integers(0, p.payload_size, 24):
        f[p.payload_offset + int(k)] ^= 0x5A
    try:
        dc = ctx.upload(bytes(f), ext_chunks(bytes(f), 1))
    except capi.PqError as e:
        assert e.code in (-9, -2, -8), e
        return
    try:
        dc.decode()
    except capi.PqError:
        pass
    finally:
        dc.free()


pa = None
try:
    import pyarrow as pa  # noqa: F811
    import pyarrow.parquet as pq
except ImportError:  # pragma: no cover
    pass


@pytest.mark.skipif(pa is None, reason="pyarrow not importable")
@pytest.mark.parametrize("codec", ["snappy", "gzip", "lz4", "zstd"])
@pytest.mark.parametrize("version", ["1.0", "2.0"])
def test_ext_large_pages_vs_pyarrow(ctx, tmp_path, codec, version):
    """1 MiB pages (pyarrow's default), 400k rows: dictionary and PLAIN
    strings plus INT64 through every codec, against pyarrow's reading."""
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden", "ext"))
    from make_ext import canonical_dump, table
    t = table(400_000, seed=11).select(["s_dict", "s_plain", "i64"])
    path = tmp_path / f"big_{codec}_{version}.parquet"
    pq.write_table(t, path, compression=codec.upper() if codec != "lz4" else "LZ4", data_page_version=version,
                   use_dictionary=["s_dict"], row_group_size=400_000)
    f = path.read_bytes()
    back = pq.read_table(path)
    for ci, c in enumerate(back.column_names):
        got = capi.canonical_dump(decode(ctx, f, ci))
        assert sha(got) == sha(canonical_dump(back.column(c))), c


@pytest.mark.skipif(pa is None, reason="pyarrow not importable")
@pytest.mark.parametrize("codec", ["snappy", "lz4", "zstd"])
@pytest.mark.parametrize("version", ["1.0", "2.0"])
@pytest.mark.parametrize("page", [5000, 8100])
def test_ext_pages_both_layouts(ctx, tmp_path, codec, version, page):
    """Pages on both sides of the small-page layout's 8 KiB history (codec.hip
    kSRing) in one chunk: the small-page and the full-layout launches each take
    their own pages of the same upload, equal to pyarrow."""
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden", "ext"))
    from make_ext import canonical_dump, table
    t = table(60_000, seed=13).select(["s_dict", "s_plain", "i64", "f64"])
    path = tmp_path / f"mix_{codec}_{version}_{page}.parquet"
    pq.write_table(t, path, compression=codec.upper() if codec != "lz4" else "LZ4", data_page_version=version,
                   use_dictionary=["s_dict"], row_group_size=60_000, data_page_size=page)
    f = path.read_bytes()
    back = pq.read_table(path)
    sizes = set()
    for ci, c in enumerate(back.column_names):
        rc, _, tab = capi.build_page_table(f, ext_chunks(f, ci)[0])
        assert rc == 0
        sizes |= {p.uncompressed_size >= 8192 for p in tab if p.page_type in (0, 3)}
        got = capi.canonical_dump(decode(ctx, f, ci))
        assert sha(got) == sha(canonical_dump(back.column(c))), c
    assert sizes == {False, True}  # both layouts ran


@pytest.mark.skipif(pa is None, reason="pyarrow not importable")
@pytest.mark.parametrize("codec", ["snappy", "lz4"])
@pytest.mark.parametrize("page", [3000, 1 << 20])
def test_ext_lz_command_shapes(ctx, tmp_path, codec, page):
    """Streams of every LZ command shape (codec.hip snappy / lz4_block):
    distance-1 and distance-3 runs (overlapping copies), incompressible bytes
    (long literals), text (short commands), runs of exactly 64 and 65 bytes
    (one wave step and one past it); equal to pyarrow.  A batched executor
    (a command per lane, pointer jumping inside a batch) measured slower
    than this one-command-per-step form (r6i: SNAPPY 7.2 vs 7.8 GB/s, LZ4
    5.7 vs 8.0) and was removed (kept in history at fb5192f)."""
    rng = np.random.default_rng(17)
    vals = []
    for i in range(6000):
        k = i % 6
        if k == 0:
            vals.append("a" * int(rng.integers(1, 300)))
        elif k == 1:
            vals.append("xyz" * int(rng.integers(1, 100)))
        elif k == 2:
            vals.append(bytes(rng.integers(32, 127, int(rng.integers(1, 500)), dtype=np.uint8)).decode())
        elif k == 3:
            vals.append("the quick brown fox " * int(rng.integers(1, 6)))
        elif k == 4:
            vals.append("b" * (64 if i % 12 == 4 else 65))
        else:
            vals.append(str(int(rng.integers(0, 10**9))))
    t = pa.table({"s": pa.array(vals, pa.string())})
    path = tmp_path / f"lz_{codec}_{page}.parquet"
    pq.write_table(t, path, compression=codec.upper() if codec != "lz4" else "LZ4", use_dictionary=False,
                   data_page_size=page, write_statistics=False)  # (long min/max strings overrun the 256-byte header window)
    f = path.read_bytes()
    got = capi.canonical_dump(decode(ctx, f, 0))
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden", "ext"))
    from make_ext import canonical_dump
    assert sha(got) == sha(canonical_dump(pq.read_table(path).column("s")))


@pytest.mark.skipif(pa is None, reason="pyarrow not importable")
@pytest.mark.parametrize("codec", ["snappy", "lz4"])
@pytest.mark.parametrize("page", [3000, 1 << 20])
def test_ext_lz_mutants_vs_pyarrow(ctx, tmp_path, codec, page):
    """Seeded damage to SNAPPY / LZ4 page payloads (byte flips, bursts of
    one value, and a few bytes set to the 255 that extends LZ4 lengths),
    through the two-wave parse/execute pass (codec.hip QSink / lz_execute):
    every mutant ends in a clean error or a decode, never a fault or a hang;
    where pyarrow also decodes the mutant, the values are equal (the formats
    carry no checksum, so a damaged stream can be a valid one)."""
    rng = np.random.default_rng(29)
    words = ["special", "requests", "carefully", "quickly", "pending", "deposits", "the", "of", " "]
    vals = [" ".join(rng.choice(words, int(rng.integers(1, 12)))) for _ in range(20000)]
    path = tmp_path / f"mut_{codec}_{page}.parquet"
    pq.write_table(pa.table({"s": pa.array(vals, pa.string())}), path, compression=codec.upper(),
                   use_dictionary=False, data_page_size=page, write_statistics=False)
    base = path.read_bytes()
    rc, _, table = capi.build_page_table(base, ext_chunks(base, 0)[0])
    assert rc == 0
    pages = [q for q in table if q.page_type == 0 and q.payload_size > 64]
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden", "ext"))
    from make_ext import canonical_dump
    import io
    both = errors = 0
    for m in range(30):
        f = bytearray(base)
        p = pages[m % len(pages)]
        kind = m % 3
        for _ in range(1 + m % 4):
            o = p.payload_offset + int(rng.integers(0, p.payload_size))
            if kind == 0:
                f[o] ^= int(rng.integers(1, 256))
            elif kind == 1:
                n = int(rng.integers(2, 40))
                f[o:o + n] = bytes([int(rng.integers(0, 256))]) * len(f[o:o + n])
            else:
                f[o] = 0xFF
        f = bytes(f)
        try:
            got = capi.canonical_dump(decode(ctx, f, 0))
        except capi.PqError as e:
            assert e.code in (-9, -2, -8), e
            errors += 1
            continue
        try:
            exp = canonical_dump(pq.read_table(io.BytesIO(f)).column("s"))
        except Exception:  # pyarrow refuses it; ours decoded (no checksum to tell)
            continue
        both += 1
        assert sha(got) == sha(exp), (codec, page, m)
    assert errors > 0  # the damage reached the parsers
