"""Pins the oracle on repeated columns (CPU, SURVEY §8a R-LEVELS, max_rep > 0).

tests/golden/lists holds pyarrow-written LIST columns (spec page order: the
reference reads the repetition section as definition levels); the crafted
max_rep pages of tests/test_gpu_decode.py (reference read order, spec order,
errors) are pinned by test_oracle_golden.py through tests/golden/manifest.json.
Here: the oracle's dumps equal the manifest and the compiled reference, and
the host layer gives the reference's max_def / max_rep for the leaf
(ParquetReader::build_columns_recursive, parquet_reader.cpp:495-543)."""
import json
import os

import pytest

from lists_util import NAMES, DIR, load, manifest, sha
from oracle import oracle as O
from pqgpu import capi
from util import file_chunks, to_oracle_chunk

MAN = manifest()
GOLDEN = os.path.join(os.path.dirname(DIR), "manifest.json")


@pytest.mark.parametrize("name", NAMES)
def test_oracle_matches_manifest(name):
    f = load(name)
    chunks = file_chunks(f, 0)
    recs = MAN["files"][name]["row_groups"]
    assert len(chunks) == len(recs)
    for ch, rec in zip(chunks, recs):
        assert (ch.max_def_level, ch.max_rep_level, ch.num_values) == (rec["max_def"], rec["max_rep"], rec["num_values"])
        assert rec["max_rep"] == 1
        rc, msg, col = O.read_all(f, to_oracle_chunk(ch))
        assert (rc != 0, msg) == (rec["rc"] != 0, rec["msg"])
        if rc == 0:
            d = O.dump_column(col)
            assert len(d) == rec["len"] and sha(d) == rec["sha256"]


@pytest.mark.skipif(not O.have_ref(), reason="oracle/_ref not built")
@pytest.mark.parametrize("name", NAMES)
def test_oracle_matches_compiled_reference(name):
    f = load(name)
    chunks, _, pidx = O.ref_open(os.path.join(DIR, name))
    F = capi.File(f)
    assert F.page_index().tolist() == pidx.tolist()
    for rg, row in enumerate(chunks):
        ref = row[0]
        ch = F.chunk(rg, 0)
        assert (ch.max_def_level, ch.max_rep_level) == (ref.max_def, ref.max_rep)
        rc, msg, col = O.read_all(f, to_oracle_chunk(ch))
        rr, rmsg, rdump = O.ref_read_all(f, ref)
        assert (rc != 0, msg) == (rr != 0, rmsg)
        if rc == 0:
            assert O.dump_column(col) == rdump


def test_crafted_repeated_pages_are_pinned():
    """Every crafted max_rep > 0 case of test_gpu_decode.py is in the golden
    manifest (pinned to the compiled reference), errors included."""
    import test_gpu_decode as D
    with open(GOLDEN) as fh:
        man = json.load(fh)
    names = [k for k in list(D.CRAFTED) + list(D.ERRORS) if k.startswith("rep_")]
    assert len(names) >= 10
    for k in names:
        e = man["crafted_" + k]
        rec = e["columns"][0][0]
        assert rec["chunk"][6] == 1, k  # max_rep
        assert (rec["rc"] == 0) == (k in D.CRAFTED), k
