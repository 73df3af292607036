"""CPU: pin the oracle (and the host format layer) to the reference's outputs.

tests/golden/manifest.json holds what the compiled reference returned for
every fixture (tests/golden/make_golden.py).  The oracle must reproduce the
dump bytes, the read_pages page records and the error text; the product's
host layer must reproduce ParquetReader's page index and chunk metadata.
"""
import hashlib
import json
import os

import pytest

from oracle import oracle as O
from pqgpu import capi

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
with open(os.path.join(HERE, "manifest.json")) as fh:
    MANIFEST = json.load(fh)


def _load(name):
    with open(os.path.join(HERE, name + ".parquet"), "rb") as fh:
        return fh.read()


@pytest.mark.parametrize("name", sorted(MANIFEST))
def test_oracle_matches_reference_outputs(name):
    data = _load(name)
    for col in MANIFEST[name]["columns"]:
        for rec in col:
            ch = O.Chunk(*rec["chunk"])
            rc, msg, out = O.read_all(data, ch)
            if rec["rc"] != 0:
                assert rc != 0, "reference failed, oracle did not"
                if rec["msg"].startswith("ByteBuffer") or "FIXED_LEN" in rec["msg"]:
                    assert msg == rec["msg"]
                continue
            assert rc == 0, msg
            dump = O.dump_column(out)
            assert len(dump) == rec["len"]
            assert hashlib.sha256(dump).hexdigest() == rec["sha256"]
            if "dump" in rec:
                with open(os.path.join(HERE, rec["dump"]), "rb") as fh:
                    assert dump == fh.read()
            got_pages = [[p[0], p[1], p[2], p[4]] for p in out.pages]
            assert got_pages == rec["pages"]


@pytest.mark.parametrize("name", sorted(n for n in MANIFEST if MANIFEST[n]["page_index"] is not None))
def test_host_page_index_and_metadata(name):
    data = _load(name)
    F = capi.File(data)
    assert F.page_index().tolist() == MANIFEST[name]["page_index"]
    cols = MANIFEST[name]["columns"]
    assert F.num_columns == len(cols)
    for ci, col in enumerate(cols):
        for rg, rec in enumerate(col):
            d = F.chunk(rg, ci)
            dict_off = d.dictionary_page_offset if d.has_dictionary_page_offset else None
            assert [d.num_values, d.data_page_offset, dict_off, d.codec, d.type, d.max_def_level,
                    d.max_rep_level] == rec["chunk"]


@pytest.mark.parametrize("name", sorted(MANIFEST))
def test_host_page_walk_matches_read_pages(name):
    """pq_build_page_table (R-WALK) yields the reference's read_pages records."""
    data = _load(name)
    for col in MANIFEST[name]["columns"]:
        for rec in col:
            if rec["rc"] != 0:
                continue
            ch = O.Chunk(*rec["chunk"])
            from util import to_desc
            rc, msg, pages = capi.build_page_table(data, to_desc(ch))
            assert rc == 0, msg
            got = [[p.page_num, p.page_type, p.num_values] for p in pages if p.page_type in (0, 2)]
            assert got == [r[:3] for r in rec["pages"]]


@pytest.mark.skipif(not O.have_ref(), reason="reference harness not built")
@pytest.mark.parametrize("name", sorted(MANIFEST))
def test_reference_harness_reproduces_manifest(name):
    """The live reference (oracle/_ref) still gives the recorded outputs."""
    data = _load(name)
    for col in MANIFEST[name]["columns"]:
        for rec in col:
            rc, msg, dump = O.ref_read_all(data, O.Chunk(*rec["chunk"]))
            assert (rc, msg) == (rec["rc"], rec["msg"])
            if rc == 0:
                assert hashlib.sha256(dump).hexdigest() == rec["sha256"]


@pytest.mark.skipif(not O.have_ref(), reason="reference harness not built")
@pytest.mark.parametrize("neg", [False, True])
def test_native_regex_baseline_matches_python_re(neg):
    """bench.py's native regex CPU baseline (reference ColumnReader + the
    build's host DFA, page-parallel) reports the same pages as the oracle
    decode + Python `re` (make_bench_expect.page_flags) for the four C3
    patterns."""
    import sys
    import numpy as np
    from pqgpu import gen
    from pqgpu.shard import data_page_ranges, extract_range
    from util import to_oracle_chunk
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts"))
    from make_bench_expect import page_flags
    f = gen.build(gen.c3_cols(), 60000, 1, seed=3)
    ch = capi.File(f).chunk(0, 0)
    rc, msg, table = capi.build_page_table(f, ch)
    assert rc == 0, msg
    data = [p for p in table if p.page_type == 0]
    shards, counts = [], []
    for a, b in data_page_ranges(table, 7):
        sub, d = extract_range(f, ch, table, a, b)
        shards.append((sub, to_oracle_chunk(d)))
        counts.append([p.num_values for p in data[a:b]])
    for pat in ("special.*requests", "^(carefully|quickly) ", "[0-9]", "e"):
        s, fl = O.ref_time_regex_pages_multi(shards, ch.type, ch.max_def_level, ch.max_rep_level, counts, pat,
                                             neg, reps=2, threads=3)
        assert np.array_equal(fl, page_flags(f, ch, pat, neg)), pat
