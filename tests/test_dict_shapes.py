"""Pins the oracle on the real-world dictionary fixtures (CPU): chunks whose
dictionary-encoded pages are followed by PLAIN pages (the writer's dictionary
fallback; the reference decides per page, column_reader.cpp:174-177 vs
213-222) and dictionaries over 64 KiB / 65,535 entries (no size limit in the
reference, column_reader.cpp:128-138, 184-196).  The oracle's canonical dumps
must equal the manifest, the compiled reference (oracle/_ref) and pyarrow's
own reading of the same files."""
import numpy as np
import pyarrow.parquet as pq
import pytest

from dict_shapes_util import DIR, NAMES, load, manifest, sha
from oracle import oracle as O
from pqgpu import capi
from util import file_chunks, oracle_read_column, to_oracle_chunk

MAN = manifest()


@pytest.mark.parametrize("name", NAMES)
def test_fixture_shape(name):
    """The files hold the shapes they are named for."""
    f = load(name)
    F = capi.File(f)
    for rg in range(F.num_row_groups):
        rc, msg, t = capi.build_page_table(f, F.chunk(rg, 0))
        assert rc == 0, msg
        data = [p for p in t if p.page_type == 0]
        dicts = [p for p in t if p.page_type == 2]
        assert len(dicts) == 1
        encs = [p.encoding for p in data]
        if name.startswith("fallback"):
            k = encs.index(0)
            assert k > 0 and all(e == 8 for e in encs[:k]) and all(e == 0 for e in encs[k:])
        elif name == "big_dict.parquet":
            assert dicts[0].payload_size > 65536 and all(e == 8 for e in encs)
        else:
            assert dicts[0].num_values > 65535 and all(e == 8 for e in encs)


@pytest.mark.parametrize("name", NAMES)
def test_oracle_matches_manifest_and_pyarrow(name):
    f = load(name)
    chunks = file_chunks(f, 0)
    t = pq.read_table(f"{DIR}/{name}")
    col = t.column(0).combine_chunks()
    row0 = 0
    for rg, ch in enumerate(chunks):
        rc, msg, d = oracle_read_column(f, [ch])
        assert rc == 0, msg
        exp = MAN["files"][name]["row_groups"][rg]
        assert len(d) == exp["len"] and sha(d) == exp["sha256"]
        n = ch.num_values
        part = col.slice(row0, n)
        valid = np.array([v is not None for v in part.to_pylist()], dtype=np.uint8)
        strs = [(s or "").encode() for s in part.to_pylist()]
        offs = np.concatenate([[0], np.cumsum([len(s) if valid[i] else 0 for i, s in enumerate(strs)])]).astype(np.int64)
        data = np.frombuffer(b"".join(s for i, s in enumerate(strs) if valid[i]) or b"\0", dtype=np.uint8)
        assert O.canonical_dump(valid, offs, data, capi.BYTE_ARRAY) == d, (name, rg)
        row0 += n


@pytest.mark.skipif(not O.have_ref(), reason="oracle/_ref not built")
@pytest.mark.parametrize("name", NAMES)
def test_oracle_matches_compiled_reference(name):
    f = load(name)
    for ch in file_chunks(f, 0):
        rc, msg, col = O.read_all(f, to_oracle_chunk(ch))
        rr, rmsg, rcol = O.ref_read_all(f, to_oracle_chunk(ch))
        assert (rc, msg) == (rr, rmsg)
        assert O.dump_column(col) == rcol  # the reference harness returns the canonical dump
