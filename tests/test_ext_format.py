"""Extended format scope on the host: the page walk of
compressed and DATA_PAGE_V2 chunks, and the pyarrow fixtures' manifest.
The reference rejects every codec (column_reader.cpp:13-15) and skips V2
pages uncounted (56-67); without PQ_EXT_* flags the walk keeps that
behaviour, with them it lists what the GPU codec pass rebuilds."""
import pytest

from ext_util import EXT_ALL, ext_chunks, load, manifest, sha
from pqgpu import capi

MAN = manifest()
FILES = sorted(MAN["files"])
CODEC_ID = {"none": 0, "snappy": 1, "gzip": 2, "lz4": 7, "zstd": 6}


def test_manifest_matches_pyarrow():
    """The committed expectations are pyarrow's reading of the committed files."""
    pa = pytest.importorskip("pyarrow")
    import pyarrow.parquet as pq
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden", "ext"))
    from make_ext import canonical_dump
    for name in FILES:
        t = pq.read_table(os.path.join(os.path.dirname(__file__), "golden", "ext", name))
        for c, e in MAN["files"][name]["columns"].items():
            assert sha(canonical_dump(t.column(c))) == e["sha256"], (name, c)
    assert pa.__version__


@pytest.mark.parametrize("name", FILES)
def test_ext_walk(name):
    f = load(name)
    info = MAN["files"][name]
    F = capi.File(f)
    codec = CODEC_ID[info["codec"]]
    v2 = info["version"] == "2.0"
    for col in range(F.num_columns):
        for d in ext_chunks(f, col):
            assert d.codec == codec
            rc, msg, table = capi.build_page_table(f, d)
            assert rc == 0, msg
            data = [p for p in table if p.page_type == 0]
            assert sum(p.num_values for p in data) == d.num_values
            rows = 0
            for p in data:
                assert p.first_row == rows
                rows += p.num_values
                assert bool(p.flags & capi.PAGE_V2) == v2
                if codec:
                    # V2 pages may store their values uncompressed (is_compressed = false)
                    assert bool(p.flags & capi.PAGE_COMPRESSED) or v2
                if p.flags & capi.PAGE_COMPRESSED:
                    assert (p.flags >> 8) & 0xFF == codec
                if v2:
                    assert p.v2_def_len >= 0 and p.v2_rep_len == 0
                    assert p.v2_def_len + p.v2_rep_len <= p.payload_size
                if not codec and not v2:
                    assert p.uncompressed_size == p.payload_size


@pytest.mark.parametrize("name", [n for n in FILES if MAN["files"][n]["codec"] != "none"])
def test_reference_scope_rejects_codecs(name):
    """Without PQ_EXT_CODECS: the reference's error (column_reader.cpp:13-15)."""
    f = load(name)
    d = ext_chunks(f, 0, flags=0)[0]
    rc, msg, _ = capi.build_page_table(f, d)
    assert rc == -1 and msg == "Only uncompressed parquet files are supported"


def test_unknown_codec_rejected():
    f = load("ext_snappy_v1.parquet")
    d = ext_chunks(f, 0)[0]
    d.codec = 4  # BROTLI: not decoded
    rc, msg, _ = capi.build_page_table(f, d)
    assert rc == -1 and "Unsupported compression codec 4" in msg


def test_v2_without_flag_is_not_counted():
    """Without PQ_EXT_PAGE_V2 a V2 page is skipped uncounted, as the reference
    does (column_reader.cpp:56-67): the walk never reaches num_values inside
    the chunk and runs on past it."""
    f = load("ext_none_v2.parquet")
    d = ext_chunks(f, 2, flags=capi.EXT_CODECS)[0]
    rc, msg, table = capi.build_page_table(f, d)
    data = [p for p in table if p.page_type == 0]
    assert sum(p.num_values for p in data) < d.num_values or rc != 0
