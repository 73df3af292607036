"""GPU parity for the --regex-column page filter (SURVEY §8a R-REGEX).

Golden: for every data page (global page order of the column), decode its
values with the oracle and ask Python `re.search(p, value, re.ASCII)`; the
page is reported iff no non-null value satisfies the predicate (match, or
non-match with --neg-regex).  NULLs never satisfy either.
"""
import re

import numpy as np
import pytest

from oracle import oracle as O
from pqgpu import capi, gen
from util import file_chunks, to_desc, to_oracle_chunk

pytestmark = pytest.mark.gpu

PATTERNS = ["special.*requests", "^(carefully|quickly) ", "[0-9]", "e", "^$", "s$",
            "(ironic|bold) (foxes|ideas)", "a.{3}e", "[^a-z ]", r"\bx" if False else "ly\\s",
            "qu?i(ck|et)ly", "^[a-z]{1,4} ", "^[a-m]",
            "x*",            # every string matches (the scan kernels skip the automaton)
            # prefilter literals ("pend" also occurs in "dependencies", "ly f"
            # after both branches, "slyl" with a $ anchor)
            "pending (foxes|ideas)", "(quick|slow)ly fur", "slyly.*deposits$", "ironic",
            "a.{5}b.{5}c"]   # over a thousand DFA states: the byte-indexed window DFA does not fit


def golden_pages(f: bytes, chunks, pattern: str, neg: bool) -> np.ndarray:
    rx = re.compile(pattern, re.ASCII)
    flags = []
    for ch in chunks:
        rc, msg, col = O.read_all(f, to_oracle_chunk(ch))
        assert rc == 0, msg
        for (_, ptype, _, first, nrows) in col.pages:
            if ptype != 0:
                continue
            sat = False
            for r in range(first, first + nrows):
                if not col.valid[r]:
                    continue
                s = bytes(col.data[col.offsets[r]:col.offsets[r + 1]]).decode("utf-8")
                m = rx.search(s) is not None
                if m != neg:
                    sat = True
                    break
            flags.append(0 if sat else 1)
    return np.array(flags, dtype=np.uint8)


CASES = [
    ("c3_ref", gen.c3_cols(), 4000, gen.REF_LAYOUT),
    ("c3_arrow", gen.c3_cols(), 9000, gen.ARROW_LAYOUT),
    ("c2_dict", gen.c2_cols(), 20000, gen.REF_LAYOUT),
    ("c2_dict_arrow", gen.c2_cols(), 20000, gen.ARROW_LAYOUT),
    ("c3_optional", [gen.Col("c", gen.COMMENT, gen.BYTE_ARRAY, optional=True, null_frac=0.3,
                             len_min=3, len_max=20)], 5000, gen.REF_LAYOUT),
    # 20,000-row arrow pages (k_pipe_big on the codes path)
    ("c2_dict_arrow_big", gen.c2_cols(), 50000, gen.ARROW_LAYOUT),
    # short dictionary entries: "e", "s$", "a.{3}e" split the pages
    ("dict_short", [gen.Col("w", gen.DICT_STRINGS, gen.BYTE_ARRAY, optional=True, null_frac=0.2, dict_size=300,
                            len_min=1, len_max=5, max_run=3)], 30000, gen.ARROW_LAYOUT),
    # eight entries in runs of up to 3000 rows: "^[a-m]" splits the pages
    ("dict_runs_big", [gen.Col("w", gen.DICT_STRINGS, gen.BYTE_ARRAY, optional=True, null_frac=0.05, dict_size=8,
                               len_min=1, len_max=3, max_run=3000)], 60000, gen.ARROW_LAYOUT),
]


@pytest.mark.parametrize("neg", [False, True], ids=["like", "notlike"])
@pytest.mark.parametrize("name,cols,n,layout", CASES, ids=[c[0] for c in CASES])
def test_regex_pages(ctx, kernel, name, cols, n, layout, neg):
    f = gen.build(cols, n, 2, seed=7, layout=layout, rows_per_page=0 if name.endswith("_big") else 700)
    chunks = file_chunks(f, 0)
    dc = ctx.upload(f, chunks)
    for p in PATTERNS:
        exp = golden_pages(f, chunks, p, neg)
        got = dc.regex_pages(p, neg)
        assert len(got) == len(exp)
        bad = np.nonzero(got != exp)[0]
        assert len(bad) == 0, (p, neg, bad[:10])
    dc.free()


def test_regex_reports_decode_errors(ctx, kernel):
    """A page whose values cannot be decoded fails the scan with the decode's
    own error text, even when an earlier value already matched."""
    import struct
    import pqbuild as B
    pay = struct.pack("<I", 7) + b"special" + struct.pack("<I", 50) + b"xy"
    f, ch = B.build_file([B.data_header(len(pay), 2, 0) + pay], gen.BYTE_ARRAY, False, 2)
    rc_o, msg_o, _ = O.read_all(f, to_oracle_chunk(ch))
    assert rc_o != 0
    dc = ctx.upload(f, [to_desc(ch)])
    with pytest.raises(capi.PqError) as ei:
        dc.regex_pages("special", False)
    assert ei.value.code == rc_o and ei.value.msg == msg_o
    dc.free()


@pytest.mark.parametrize("nrg", [1, 2])
@pytest.mark.parametrize("layout", [gen.REF_LAYOUT, gen.ARROW_LAYOUT])
def test_regex_reuses_checked_decode_codes(ctx, layout, nrg):
    """regex_reuse: after a checked decode the scan reads that decode's codes
    (no dict/run/codes passes); page sets equal the oracle's, interleaved
    with further decodes, and the decode's output stays correct."""
    cols = gen.c2_cols()
    f = gen.build(cols, 40000, nrg, seed=9, layout=layout, rows_per_page=0 if layout == gen.REF_LAYOUT else 3000)
    chunks = file_chunks(f, 0)
    dc = ctx.upload(f, chunks)
    pats = ["^qx", "e", "^[a-m]", "a.{3}e"]
    exp = {(p, n): golden_pages(f, chunks, p, n) for p in pats for n in (False, True)}
    dc.decode()
    ref = capi.canonical_dump(dc.to_host())
    fronts = ("dict_index", "pipe_runs", "pipe_codes", "pipe_big", "pipe_count")
    ctx.timing(True)
    ctx.timing_reset()
    dc.decode()
    base = {k: ctx.timing_get(k)[1] for k in fronts}
    ctx.timing_reset()
    for p in pats:
        for n in (False, True):
            assert np.array_equal(dc.regex_pages(p, n), exp[(p, n)]), (p, n)
        dc.decode_async()
        dc.regex_pages_async(p, True)
        assert np.array_equal(dc.regex_pages_result(), exp[(p, True)])
    ctx.timing(False)
    for k in fronts:  # only the decodes ran the front passes
        assert ctx.timing_get(k)[1] == len(pats) * base[k], (k, base)
    assert capi.canonical_dump(dc.to_host()) == ref
    dc.free()


@pytest.mark.parametrize("case", ["zero_count", "dict_truncated", "missing_bw"])
def test_regex_reuse_not_taken_after_failed_decode(ctx, case):
    """A decode that failed leaves no reusable codes or entries: the scan
    reports the decode's error itself, every time."""
    import struct
    import pqbuild as B
    dvals = [b"alpha", b"", b"gamma-gamma", b"d"]
    dpay = B.plain_ba(dvals)
    if case == "zero_count":  # a zero-count RLE run before any literal run
        idx, nv, opt = bytes([2]) + B.rle(0, 1, 2) + B.rle(3, 1, 2), 3, False
    elif case == "dict_truncated":
        dpay, idx, nv, opt = struct.pack("<I", 1) + b"a" + b"\x05", bytes([1]) + B.rle(2, 0, 1), 2, False
    else:  # the index stream has no bit-width byte
        idx, nv, opt = B.levels_section(B.rle(4, 0, 1)), 4, True
    ndict = 2 if case == "dict_truncated" else len(dvals)
    f, ch = B.build_file([B.dict_header(len(dpay), ndict) + dpay, B.data_header(len(idx), nv, 8) + idx],
                         gen.BYTE_ARRAY, opt, nv, dict_at_start=True)
    rc_o, msg_o, _ = O.read_all(f, to_oracle_chunk(ch))
    assert rc_o != 0
    dc = ctx.upload(f, [to_desc(ch)])
    for _ in range(2):
        with pytest.raises(capi.PqError) as e1:
            dc.decode()
        assert e1.value.code == rc_o
        with pytest.raises(capi.PqError) as e2:
            dc.regex_pages("a", False)
        assert (e2.value.code, e2.value.msg) == (e1.value.code, e1.value.msg)
    dc.free()


@pytest.mark.parametrize("neg", [False, True])
@pytest.mark.parametrize("name,cols,n,layout", [c for c in CASES if c[0] != "c3_optional"],
                         ids=[c[0] for c in CASES if c[0] != "c3_optional"])
def test_decode_regex_one_pass(ctx, name, cols, n, layout, neg):
    """pq_decode_regex_async: the page flags equal the separate scan's and the
    oracle's, and the column equals the plain decode's, on every case (the
    writer's armed filter on pipe chunks, decode + scan elsewhere); repeated
    passes and plain decodes in between keep both right."""
    f = gen.build(cols, n, 1, seed=11, layout=layout, rows_per_page=0 if name.endswith("_big") else 700)
    chunks = file_chunks(f, 0)
    dc = ctx.upload(f, chunks)
    dc.decode()
    ref = capi.canonical_dump(dc.to_host())
    for p in ("^qx", "e", "^[a-m]", "a.{3}e", "special.*requests"):
        exp = golden_pages(f, chunks, p, neg)
        for _ in range(2):
            dc.decode_regex_async(p, neg)
            got = dc.regex_pages_result()
            dc.decode_check()
            assert np.array_equal(got, exp), (p, neg)
            assert capi.canonical_dump(dc.to_host()) == ref
        dc.decode_async()
        dc.decode_check()
    dc.free()


FRESH_REDO = ["opt_plain_extra", "opt_plain_spec_extra", "plain_spec_extra", "plain_spec_long",
              "opt_plain_page", "plain_pages"]


@pytest.mark.parametrize("neg", [False, True], ids=["like", "notlike"])
@pytest.mark.parametrize("case", FRESH_REDO)
def test_decode_regex_fresh_chunk_redo(ctx, case, neg):
    """pq_decode_regex_async on a freshly uploaded chunk (no checked decode
    before it) whose pages do not fit the one-pass PLAIN form (bytes after
    the strings, fewer values declared than the page holds, OPTIONAL value
    sections, chains that need the generic path): the decode's redo runs
    before the scan clears the status words, so both the column and the page
    flags equal the oracle's on the first call."""
    import test_gpu_decode as D
    f, ch = D.CRAFTED[case]()
    rc_o, msg_o, d_o = O.read_all(f, to_oracle_chunk(ch))
    assert rc_o == 0, msg_o
    exp_dump = O.dump_column(d_o)
    for p in ("a", "^[a-m]", "zz", "q.*x"):
        exp = golden_pages(f, [ch], p, neg)
        dc = ctx.upload(f, [to_desc(ch)])
        try:
            dc.decode_regex_async(p, neg)
            got = dc.regex_pages_result()
            dc.decode_check()
            assert np.array_equal(got, exp), (case, p, neg)
            assert capi.canonical_dump(dc.to_host()) == exp_dump, (case, p)
        finally:
            dc.free()


@pytest.mark.parametrize("layout,rpp", [(gen.REF_LAYOUT, 0), (gen.ARROW_LAYOUT, 700), (gen.ARROW_LAYOUT, 1300),
                                        (gen.ARROW_LAYOUT, 2500)], ids=["ref", "arrow_21k", "arrow_40k", "arrow_77k"])
def test_string_index_reuse(ctx, layout, rpp):
    """REQUIRED PLAIN chunks: the first error-free windowed scan files the
    string index, later scans read it; a window-size change rebuilds it; the
    page sets stay the oracle's throughout, with the index on and off.  Pages
    of ~21, ~40 and ~77 KB: windows up to the u16 offset limit, and pages
    past it (k_regex_lanes)."""
    cols = gen.c3_cols()
    f = gen.build(cols, 30000, 1, seed=13, layout=layout, rows_per_page=rpp)
    chunks = file_chunks(f, 0)
    pats = ["special.*requests", "e", "^(carefully|quickly) ", "[0-9]", "ly\\s"]
    exp = {(p, n): golden_pages(f, chunks, p, n) for p in pats for n in (False, True)}
    dc = ctx.upload(f, chunks)
    try:
        for win in (8192, 4096, 8192):
            ctx.set_option("regex_win", win)
            for idx in (1, 0, 2, 1):  # 2: every scan files the index again (cold)
                ctx.set_option("regex_index", idx)
                for p in pats:
                    for n in (False, True):
                        assert np.array_equal(dc.regex_pages(p, n), exp[(p, n)]), (win, idx, p, n)
    finally:
        ctx.set_option("regex_win", 8192)
        ctx.set_option("regex_index", 1)
        dc.free()


def test_string_index_not_filed_on_error(ctx):
    """A chunk whose scan fails files no index: every later scan reports the
    same error."""
    import struct
    import pqbuild as B
    pay = struct.pack("<I", 7) + b"special" + struct.pack("<I", 50) + b"xy"
    f, ch = B.build_file([B.data_header(len(pay), 2, 0) + pay], gen.BYTE_ARRAY, False, 2)
    rc_o, msg_o, _ = O.read_all(f, to_oracle_chunk(ch))
    dc = ctx.upload(f, [to_desc(ch)])
    for _ in range(3):
        with pytest.raises(capi.PqError) as ei:
            dc.regex_pages("special", False)
        assert ei.value.code == rc_o and ei.value.msg == msg_o
    dc.free()


REP_BA = ["rep_list_dict", "rep_list_dict_big", "rep_list_plain_ba", "rep_list_plain_ba_big", "rep_repeated_plain_ba",
          "rep_repeated_dict", "rep_spec_order_repeated_dict", "rep_spec_order_list_plain_ba"]


@pytest.mark.parametrize("neg", [False, True], ids=["like", "notlike"])
@pytest.mark.parametrize("case", REP_BA)
def test_regex_repeated_columns(ctx, kernel, case, neg):
    """Repeated BYTE_ARRAY columns (max_rep 1): every page kernel skips the
    repetition section as the reference does (column_reader.cpp:156-164) and
    reports the oracle's page set."""
    import test_gpu_decode as D
    f, ch = D.CRAFTED[case]()
    dc = ctx.upload(f, [to_desc(ch)])
    try:
        for p in ("e", "^[a-g]", "re.*n", "zz", "x*"):
            exp = golden_pages(f, [ch], p, neg)
            got = dc.regex_pages(p, neg)
            assert np.array_equal(got, exp), (case, p, neg, np.nonzero(got != exp)[0][:10])
    finally:
        dc.free()


@pytest.mark.parametrize("case", ["rep_len_overrun", "rep_len_missing"])
def test_regex_repeated_column_errors(ctx, kernel, case):
    import test_gpu_decode as D
    f, ch = D.ERRORS[case]()
    rc_o, msg_o, _ = O.read_all(f, to_oracle_chunk(ch))
    assert rc_o != 0
    if ch["type"] != gen.BYTE_ARRAY:
        pytest.skip("not a string column")
    dc = ctx.upload(f, [to_desc(ch)])
    try:
        with pytest.raises(capi.PqError) as ei:
            dc.regex_pages("e", False)
        assert ei.value.code == rc_o and ei.value.msg == msg_o
    finally:
        dc.free()


@pytest.mark.parametrize("case", ["huge_dict_wide_mixed", "huge_dict_wide_small_pages", "huge_dict_wide_oob",
                                  "huge_dict_wide_bw26"])
def test_regex_wide_dictionary(ctx, kernel, case):
    """Dictionaries of more than 65,535 entries (the wide pipe's 32-bit codes:
    k_pipe_match_w on the codes path), also after a checked decode (codes
    reused) and through the decode + filter call."""
    from test_gpu_decode import CRAFTED
    f, ch = CRAFTED[case]()
    chunks = [to_desc(ch)]
    dc = ctx.upload(f, chunks)
    for p in ("^qx", "e", "a.{3}e", "^[a-m]+$"):
        for neg in (False, True):
            exp = golden_pages(f, chunks, p, neg)
            assert np.array_equal(dc.regex_pages(p, neg), exp), (p, neg)
    dc.decode()
    ref = capi.canonical_dump(dc.to_host())
    rc_o, msg_o, col = O.read_all(f, to_oracle_chunk(ch))
    assert rc_o == 0 and ref == O.dump_column(col)
    for neg in (False, True):
        assert np.array_equal(dc.regex_pages("e", neg), golden_pages(f, chunks, "e", neg))
    dc.free()
