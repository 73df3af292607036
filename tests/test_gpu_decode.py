"""GPU parity: the HIP decode path (through the C ABI) against the oracle.

Bit-exact comparison of the canonical dump: u8 is_null, then the
value bytes (FLOAT/DOUBLE compared as bit patterns; the north star's 1-ulp
float tolerance is never needed because decode is a byte copy).  Error cases
must fail with the same error class and message text as the oracle.
"""
import hashlib
import struct

import numpy as np
import pytest

import pqbuild as B
from pqgpu import capi, gen
from util import file_chunks, gpu_read_column, oracle_read_column, to_desc

pytestmark = pytest.mark.gpu

SMALL = [
    ("c1_int32", gen.c1_cols(), 10000),
    ("c2_dict", gen.c2_cols(), 30000),
    ("c3_plain", gen.c3_cols(), 6000),
    ("c4_mixed", gen.c4_cols(), 5000),
    ("bool", [gen.Col("b", gen.UNIFORM, gen.BOOLEAN, optional=True, null_frac=0.3)], 3000),
    ("bool_plain", [gen.Col("b", gen.UNIFORM, gen.BOOLEAN, optional=True, null_frac=0.3, force_plain=True)], 3000),
    ("float", [gen.Col("f", gen.DOUBLE_RANGE, gen.FLOAT, optional=True, null_frac=0.1)], 4000),
    ("small_int_dict", [gen.Col("i", gen.SMALL_INT, gen.INT64, optional=True, null_frac=0.2, dict_size=7)], 9000),
    ("small_int32_dict", [gen.Col("i", gen.SMALL_INT, gen.INT32, dict_size=300)], 9000),
    ("all_null", [gen.Col("s", gen.DICT_STRINGS, gen.BYTE_ARRAY, optional=True, null_frac=1.0)], 2000),
    # dictionary entries longer than k_dict_index's 64-byte candidate window:
    # the fine slices cannot link and the coarse walk decides
    ("long_dict", [gen.Col("s", gen.DICT_STRINGS, gen.BYTE_ARRAY, dict_size=600, len_min=40, len_max=300)], 4000),
    ("mixed_dict", [gen.Col("s", gen.DICT_STRINGS, gen.BYTE_ARRAY, optional=True, null_frac=0.1, dict_size=3000,
                            len_min=1, len_max=70)], 6000),
    ("long_strings", [gen.Col("s", gen.DICT_STRINGS, gen.BYTE_ARRAY, optional=True, null_frac=0.1,
                              dict_size=40, len_min=100, len_max=3000)], 4000),
    ("wide_dict", [gen.Col("s", gen.DICT_STRINGS, gen.BYTE_ARRAY, dict_size=70000, len_min=1, len_max=6,
                           max_run=2)], 400000),
    # pipe-sized dictionary (< 64 KiB) with more entries than k_pipe_big's LDS
    # length table (kBigLens = 8192): the lengths of later entries come from HBM
    ("lens_past_lds", [gen.Col("s", gen.DICT_STRINGS, gen.BYTE_ARRAY, optional=True, null_frac=0.1,
                               dict_size=9000, len_min=3, len_max=4, max_run=2)], 60000),
    # OPTIONAL PLAIN BYTE_ARRAY (levels, then value sections on the PLAIN
    # kernels): 1 KiB pages (windows) and 3000-row arrow pages (chunk chains),
    # sparse, all-NULL, strings over the chunk chains' 60-byte reach
    ("opt_plain", [gen.Col("s", gen.COMMENT, gen.BYTE_ARRAY, optional=True, null_frac=0.2, len_min=0,
                           len_max=40)], 6000),
    ("opt_plain_sparse", [gen.Col("s", gen.COMMENT, gen.BYTE_ARRAY, optional=True, null_frac=0.9, len_min=5,
                                  len_max=30)], 7000),
    ("opt_plain_all_null", [gen.Col("s", gen.COMMENT, gen.BYTE_ARRAY, optional=True, null_frac=1.0)], 3000),
    ("opt_plain_long", [gen.Col("s", gen.COMMENT, gen.BYTE_ARRAY, optional=True, null_frac=0.1, len_min=50,
                                len_max=200)], 4000),
]


@pytest.mark.parametrize("layout", [gen.REF_LAYOUT, gen.ARROW_LAYOUT], ids=["ref", "arrow"])
@pytest.mark.parametrize("name,cols,n", SMALL, ids=[s[0] for s in SMALL])
def test_generated_columns(ctx, path, name, cols, n, layout):
    f = gen.build(cols, n, 2, seed=11, layout=layout, rows_per_page=3000)
    for ci in range(len(cols)):
        chunks = file_chunks(f, ci)
        rc_o, msg_o, d_o = oracle_read_column(f, chunks)
        rc_g, msg_g, d_g = gpu_read_column(ctx, f, chunks)
        assert (rc_g, msg_g) == (rc_o, msg_o), (name, ci)
        assert d_g == d_o, (name, ci, len(d_g or b""), len(d_o or b""))


@pytest.mark.parametrize("run_dict", [0, 1], ids=["side_stream", "in_runs"])
@pytest.mark.parametrize("layout", [gen.REF_LAYOUT, gen.ARROW_LAYOUT], ids=["ref", "arrow"])
@pytest.mark.parametrize("name,cols,n", [s for s in SMALL if s[0] in ("c2_dict", "c4_mixed", "long_dict", "mixed_dict")],
                         ids=lambda v: v if isinstance(v, str) else "")
def test_dict_decode_placement(ctx, run_dict, layout, name, cols, n):
    """The pipe's dictionary page decoded by k_pipe_runs' leading workgroups
    (pipe_run_dict=1, default) and by its own k_dict_index launch on the side
    stream (0); three decodes per upload, each equal to the oracle."""
    ctx.set_option("pipe_run_dict", run_dict)
    try:
        f = gen.build(cols, n, 2, seed=13, layout=layout, rows_per_page=3000)
        for ci in range(len(cols)):
            chunks = file_chunks(f, ci)
            rc_o, _, d_o = oracle_read_column(f, chunks)
            assert rc_o == 0
            dc = ctx.upload(f, [to_desc(c) for c in chunks])
            try:
                for _ in range(3):
                    dc.decode()
                    assert capi.canonical_dump(dc.to_host()) == d_o, (name, ci)
            finally:
                dc.free()
    finally:
        ctx.set_option("pipe_run_dict", 1)


@pytest.mark.parametrize("name,cols,n", [s for s in SMALL if s[0] in
                                         ("c2_dict", "c4_mixed", "all_null", "long_strings", "wide_dict")],
                         ids=lambda v: v if isinstance(v, str) else "")
def test_small_arrow_pages(ctx, path, name, cols, n):
    """Arrow-style pages of 700 rows: bit-packed def-level runs, RLE runs
    >= 8, several tiles per page."""
    f = gen.build(cols, n, 2, seed=12, layout=gen.ARROW_LAYOUT, rows_per_page=700)
    for ci in range(len(cols)):
        chunks = file_chunks(f, ci)
        rc_o, msg_o, d_o = oracle_read_column(f, chunks)
        rc_g, msg_g, d_g = gpu_read_column(ctx, f, chunks)
        assert (rc_g, msg_g) == (rc_o, msg_o), (name, ci)
        assert d_g == d_o, (name, ci)


def test_repeat_decode_reuses_buffers(ctx):
    """Decoding twice into the same output gives identical bytes (no stale state)."""
    f = gen.build(gen.c2_cols(), 50000, 1, seed=3)
    chunks = file_chunks(f, 0)
    dc = ctx.upload(f, chunks)
    dc.decode()
    a = capi.canonical_dump(dc.to_host())
    dc.decode()
    b = capi.canonical_dump(dc.to_host())
    dc.free()
    assert a == b
    assert a == oracle_read_column(f, chunks)[2]


# ── crafted pages: reference quirks and error behaviour ────────────────────
def _dict_ba_file(idx_stream: bytes, nvals: int, dict_vals, def_stream: bytes | None = None,
                  enc: int = 8, extra_pages=()):
    dpay = B.plain_ba(dict_vals)
    pages = [B.dict_header(len(dpay), len(dict_vals)) + dpay]
    pay = (B.levels_section(def_stream) if def_stream is not None else b"") + idx_stream
    pages.append(B.data_header(len(pay), nvals, enc) + pay)
    pages += list(extra_pages)
    return B.build_file(pages, gen.BYTE_ARRAY, def_stream is not None, nvals + sum(
        0 for _ in extra_pages), dict_at_start=True)


def _hybrid(values, bw, rng, max_groups=63):
    """A hybrid RLE/bit-packed stream of `values`: RLE runs for repeats of 8
    or more, bit-packed groups (1..max_groups per run) otherwise."""
    out, i, n = [], 0, len(values)
    while i < n:
        j = i
        while j < n and values[j] == values[i]:
            j += 1
        if j - i >= 8:
            out.append(B.rle(j - i, values[i], bw))
            i = j
            continue
        g = int(rng.integers(1, max_groups + 1))
        chunk = values[i:i + 8 * g]
        out.append(B.bitpack(chunk, bw))
        i += len(chunk)
    return b"".join(out)


def _big_dict_file(nvals, seed, optional=True, bw=3, dict_vals=None, tail=b"", cut=0, max_groups=63, run=12):
    """One dictionary page and one data page of `nvals` > kPipeSmallRows rows
    (the k_pipe_big path): runs of repeated indices, some out of range, 10%
    NULL; `tail` is appended to the index stream, `cut` bytes removed."""
    rng = np.random.default_rng(seed)
    dv = dict_vals if dict_vals is not None else [b"v%d-" % i * (1 + i % 3) for i in range((1 << bw) - 2)]
    idx = []
    while len(idx) < nvals:
        idx += [int(rng.integers(0, 1 << bw))] * int(rng.integers(1, run))
    idx = idx[:nvals]
    defs = None
    if optional:
        defs = [int(x) for x in rng.random(nvals) > 0.1]
        for k in range(0, nvals, 997):  # long valid stretches: RLE level runs
            defs[k:k + 40] = [1] * len(defs[k:k + 40])
        idx = [v for v, d in zip(idx, defs) if d]
    stream = bytes([bw]) + _hybrid(idx, bw, rng, max_groups) + tail
    if cut:
        stream = stream[:-cut]
    dstream = _hybrid(defs, 1, rng) if optional else None
    return _dict_ba_file(stream, nvals, dv, def_stream=dstream)


DICT = [b"alpha", b"", b"gamma-gamma", b"d"]


def _big_plain_file(seed, cut=None):
    """REQUIRED PLAIN BYTE_ARRAY pages of 40-110 KB; `cut` truncates the second
    page's payload at that many bytes (the chain runs past the page)."""
    rng = np.random.default_rng(seed)
    pages, total = [], 0
    for k in range(3):
        vals = [bytes(rng.integers(97, 123, int(rng.choice([rng.integers(0, 30), rng.integers(60, 200)]))).astype(np.uint8))
                for _ in range(int(rng.integers(900, 1800)))]
        if k == 1:
            vals.insert(7, b"y" * 50000)
        pay = B.plain_ba(vals)
        if cut is not None and k == 1:
            pay = pay[:cut]
        pages.append(B.data_header(len(pay), len(vals), 0) + pay)
        total += len(vals)
    return B.build_file(pages, gen.BYTE_ARRAY, False, total)


def _spec_plain_file(seed, n=3000, cut=None, nvals=None, binary=False, pages=2, lmax=44):
    """REQUIRED PLAIN BYTE_ARRAY pages of `n` short strings (16-100 KB: the
    speculative chunk path); `cut` drops bytes from the end of the last page,
    `nvals` overrides the header value count, `binary` draws string bytes from
    0..255 (more plausible false chain starts)."""
    rng = np.random.default_rng(seed)
    out, total = [], 0
    for k in range(pages):
        lo, hi = (0, 256) if binary else (97, 123)
        vals = [bytes(rng.integers(lo, hi, int(rng.integers(0, lmax + 1))).astype(np.uint8)) for _ in range(n)]
        pay = B.plain_ba(vals)
        nv = n
        if k == pages - 1:
            if cut:
                pay = pay[:-cut]
            if nvals is not None:
                nv = nvals
        out.append(B.data_header(len(pay), nv, 0) + pay)
        total += nv
    return B.build_file(out, gen.BYTE_ARRAY, False, total)


def _opt_levels_file(stream: bytes, nvals: int, nn: int, seed: int):
    """One OPTIONAL INT64 page with the given def-level stream and nn values."""
    rng = np.random.default_rng(seed)
    vals = struct.pack(f"<{nn}q", *[int(x) for x in rng.integers(-1 << 40, 1 << 40, nn)])
    pay = B.levels_section(stream) + vals
    return B.build_file([B.data_header(len(pay), nvals, 0) + pay], gen.INT64, True, nvals)


def _opt_fixed_file(ptype, fmt, nvals, seed, rle_levels=False, drop=0):
    """One OPTIONAL PLAIN fixed-width page; `drop` trailing values removed
    from the payload (the read overruns on the last non-null rows)."""
    rng = np.random.default_rng(seed)
    if rle_levels:
        k = nvals * 2 // 3
        defs = [1] * k + [0] * (nvals - k)
        stream = B.rle(k, 1, 1) + B.rle(nvals - k, 0, 1)
    else:
        defs = [int(x) for x in rng.random(nvals) < 0.7]
        head = (nvals // 2) // 8 * 8
        stream = B.bitpack(defs[:head], 1) + B.rle(nvals - head, 1, 1)
        defs = defs[:head] + [1] * (nvals - head)
    nn = sum(defs) - drop
    vals = b"".join(struct.pack(fmt, *([int(rng.integers(-1 << 40, 1 << 40))] if fmt in ("<q",) else
                                       [float(rng.standard_normal())] if fmt in ("<d", "<f") else
                                       [int(rng.integers(-1 << 60, 1 << 60)), int(rng.integers(-1 << 30, 1 << 30))]))
                    for _ in range(nn))
    pay = B.levels_section(stream) + vals
    return B.build_file([B.data_header(len(pay), nvals, 0) + pay], ptype, True, nvals)

def _opt_plain_file(nvals, seed, null_frac=0.3, lmax=30, extra=b"", drop=0, all_bitpacked=False):
    """One OPTIONAL PLAIN BYTE_ARRAY page: bit-packed and RLE def levels,
    then the non-null strings; `extra` bytes after them, `drop` trailing
    strings removed (the read overruns)."""
    rng = np.random.default_rng(seed)
    defs = [int(x) for x in rng.random(nvals) >= null_frac]
    head = nvals // 8 * 8 if all_bitpacked else (nvals // 2) // 8 * 8
    stream = B.bitpack(defs[:head], 1) + (B.rle(nvals - head, 1, 1) if nvals > head else b"")
    defs = defs[:head] + [1] * (nvals - head)
    nn = sum(defs) - drop
    strs = [bytes(rng.integers(97, 123, int(rng.integers(0, lmax + 1))).astype(np.uint8)) for _ in range(nn)]
    pay = B.levels_section(stream) + B.plain_ba(strs) + extra
    return B.build_file([B.data_header(len(pay), nvals, 0) + pay], gen.BYTE_ARRAY, True, nvals)


def _huge_dict_file(n: int, seed: int, lmin: int = 1, lmax: int = 14, decl: int | None = None, tail: bytes = b"",
                    cut: int = 0, nrows: int = 5000, pages: int = 1, mixed: bool = False, bw_add: int = 0):
    """A dictionary page beyond k_dict_index's LDS (> 128 KiB: the
    multi-workgroup index, launch_dict_big) and data pages of indices spread
    over the whole dictionary (17-bit codes when n > 65,536; the wide pipe,
    k_pipe_big<true> -> k_pipe_wwide): one RLE run per value, or (mixed)
    bit-packed groups between RLE runs; bw_add widens the indices past what
    the pipe's run parse takes (> 24 bits: the exact decoder's 32-bit codes)."""
    rng = np.random.default_rng(seed)
    vals = [bytes(rng.integers(97, 123, size=int(rng.integers(lmin, lmax + 1)), dtype=np.uint8)) for _ in range(n)]
    dpay = B.plain_ba(vals) + tail
    if cut:
        dpay = dpay[:-cut]
    bw = max(1, int(n - 1).bit_length()) + bw_add
    out = [B.dict_header(len(dpay), n if decl is None else decl) + dpay]
    per = nrows // pages
    for k in range(pages):
        m = per if k < pages - 1 else nrows - per * (pages - 1)
        idx = [int(x) for x in rng.integers(0, n, size=m)]
        if mixed:
            body, i = b"", 0
            while i < m:
                if rng.random() < 0.5 and m - i >= 8:
                    g = int(min((m - i) // 8, rng.integers(1, 9)))
                    body += B.bitpack(idx[i:i + 8 * g], bw)
                    i += 8 * g
                else:
                    r = int(min(m - i, rng.integers(1, 20)))
                    body += B.rle(r, idx[i], bw)
                    i += r
        else:
            body = b"".join(B.rle(1, v, bw) for v in idx)
        stream = bytes([bw]) + body
        out.append(B.data_header(len(stream), m, 8) + stream)
    return B.build_file(out, gen.BYTE_ARRAY, False, nrows, dict_at_start=True)


def _rep_pages(ptype, nested, optional, rows_per_page, npages, seed, enc=0, dict_vals=None, spec_order=False,
               rep_len_delta=0, cut_after_def=False):
    """Pages of a repeated column (max_rep 1) in the order the reference reads
    them, [u32 def_len][def][u32 rep_len][rep][values] (column_reader.cpp:
    146-170: definition levels first, repetition levels decoded and dropped);
    spec_order writes [rep][def] as the Parquet spec (and pyarrow) lay V1
    pages out, which the reference then reads with the sections swapped.
    Levels mix RLE and bit-packed runs; values are PLAIN (INT64 / DOUBLE /
    BOOLEAN / BYTE_ARRAY) or dictionary indices (enc 8, dict_vals)."""
    rng = np.random.default_rng(seed)
    max_def = (2 + (1 if optional else 0)) if nested == "list" else 1
    dbw, rbw = max(1, int(max_def).bit_length()), 1
    pages = []
    if dict_vals is not None:
        dpay = B.plain_ba(dict_vals)
        pages.append(B.dict_header(len(dpay), len(dict_vals)) + dpay)
    total = 0
    for k in range(npages):
        n = rows_per_page
        defs, reps, i = [], [], 0
        while i < n:  # runs of one level (RLE) and stretches of random levels (bit-packed)
            if rng.random() < 0.4:
                m = int(min(n - i, rng.integers(8, 60)))
                defs += [max_def] * m if rng.random() < 0.7 else [int(rng.integers(0, max_def + 1))] * m
            else:
                m = int(min(n - i, 8 * rng.integers(1, 6)))
                defs += [int(x) for x in np.where(rng.random(m) < 0.75, max_def, rng.integers(0, max_def + 1, m))]
            i += m
        defs = defs[:n]
        reps = [0 if (j == 0 or rng.random() < 0.3) else 1 for j in range(n)]
        dstream = _hybrid(defs, dbw, rng, max_groups=4)
        rstream = _hybrid(reps, rbw, rng, max_groups=3)
        nn = sum(1 for d in defs if d == max_def)
        if dict_vals is not None:
            bw = max(1, (len(dict_vals) - 1).bit_length())
            vals = bytes([bw]) + _hybrid([int(x) for x in rng.integers(0, len(dict_vals), nn)], bw, rng)
        elif ptype == gen.INT64:
            vals = struct.pack(f"<{nn}q", *[int(x) for x in rng.integers(-1 << 50, 1 << 50, nn)])
        elif ptype == gen.DOUBLE:
            vals = struct.pack(f"<{nn}d", *[float(x) for x in rng.standard_normal(nn)])
        elif ptype == gen.BOOLEAN:
            vals = bytes(int(x) for x in rng.integers(0, 256, (nn + 7) // 8))
        else:
            vals = B.plain_ba([bytes(rng.integers(97, 123, int(rng.integers(0, 25))).astype(np.uint8))
                               for _ in range(nn)])
        first, second = (rstream, dstream) if spec_order else (dstream, rstream)
        if cut_after_def and k == npages - 1:
            pay = B.levels_section(first) + b"\x01\x00"
        else:
            pay = (B.levels_section(first) + struct.pack("<I", len(second) + rep_len_delta) + second + vals)
        pages.append(B.data_header(len(pay), n, enc) + pay)
        total += n
    return B.build_file(pages, ptype, optional, total, dict_at_start=dict_vals is not None, nested=nested)


REP_DICT = [b"red", b"", b"green-green", b"blue", b"violet and more", b"k"]

CRAFTED = {
    # repeated columns (max_rep 1), R-LEVELS: definition levels then
    # repetition levels in the reference's read order, over every value kind;
    # LIST shape (max_def 3, bit width 2) and a REPEATED leaf (max_def 1);
    # 20,000-row pages for the large-page kernels; spec-order pages (the
    # reference reads the repetition section as definition levels)
    "rep_list_dict": lambda: _rep_pages(gen.BYTE_ARRAY, "list", True, 700, 3, seed=91, enc=8, dict_vals=REP_DICT),
    "rep_list_dict_big": lambda: _rep_pages(gen.BYTE_ARRAY, "list", True, 20000, 2, seed=92, enc=8,
                                            dict_vals=REP_DICT),
    "rep_list_int64": lambda: _rep_pages(gen.INT64, "list", True, 900, 3, seed=93),
    "rep_list_int64_required": lambda: _rep_pages(gen.INT64, "list", False, 600, 2, seed=94),
    "rep_list_double_big": lambda: _rep_pages(gen.DOUBLE, "list", True, 5000, 2, seed=95),
    "rep_list_plain_ba": lambda: _rep_pages(gen.BYTE_ARRAY, "list", True, 800, 3, seed=96),
    "rep_list_plain_ba_big": lambda: _rep_pages(gen.BYTE_ARRAY, "list", True, 6000, 2, seed=97),
    "rep_repeated_plain_ba": lambda: _rep_pages(gen.BYTE_ARRAY, "repeated", False, 500, 3, seed=98),
    "rep_repeated_dict": lambda: _rep_pages(gen.BYTE_ARRAY, "repeated", False, 1500, 2, seed=99, enc=8,
                                            dict_vals=REP_DICT),
    "rep_repeated_bool": lambda: _rep_pages(gen.BOOLEAN, "repeated", False, 700, 2, seed=100),
    # (spec order with a dictionary needs equal level bit widths: a level above
    # max_def on a dictionary page is undefined behaviour in the reference,
    # indices[] read past num_non_null, column_reader.cpp:181-189)
    "rep_spec_order_repeated_dict": lambda: _rep_pages(gen.BYTE_ARRAY, "repeated", False, 700, 2, seed=101, enc=8,
                                                       dict_vals=REP_DICT, spec_order=True),
    "rep_spec_order_list_plain_ba": lambda: _rep_pages(gen.BYTE_ARRAY, "list", True, 640, 3, seed=105,
                                                       spec_order=True),

    # dictionary pages beyond LDS: short entries (the parallel slices link),
    # entries over 64 bytes (uncovered slice entries: the serial walk), bytes
    # after the declared entries, 17-bit indices
    "huge_dict_short": lambda: _huge_dict_file(40000, seed=81),
    "huge_dict_wide": lambda: _huge_dict_file(100000, seed=82, lmin=4, lmax=9),
    "huge_dict_long": lambda: _huge_dict_file(3000, seed=83, lmin=60, lmax=140),
    "huge_dict_tail": lambda: _huge_dict_file(30000, seed=84, tail=b"\x07\x00\x00\x00garbage!" * 5),
    "huge_dict_fewer_used": lambda: _huge_dict_file(30000, seed=85, decl=20000),
    # the wide pipe: bit-packed 17-bit indices between RLE runs over pages of
    # 2,500 and of 400 rows (small pages take k_pipe_big there too); indices
    # past a shorter declared count; 26-bit indices (the exact decoder)
    "huge_dict_wide_mixed": lambda: _huge_dict_file(100000, seed=88, lmin=4, lmax=9, nrows=10000, pages=4, mixed=True),
    "huge_dict_wide_small_pages": lambda: _huge_dict_file(90000, seed=89, lmin=2, lmax=30, nrows=4000, pages=10,
                                                          mixed=True),
    "huge_dict_wide_oob": lambda: _huge_dict_file(100000, seed=90, lmin=4, lmax=9, decl=70000, nrows=6000, pages=2,
                                                  mixed=True),
    "huge_dict_wide_bw26": lambda: _huge_dict_file(100000, seed=91, lmin=4, lmax=9, nrows=3000, pages=2, mixed=True,
                                                   bw_add=9),
    # pages of 24-48 KiB: k_pipe_big's jump table in two segments (a wide
    # dictionary's 17-bit indices, and a 3,000-entry dictionary's 12-bit ones)
    "huge_dict_wide_bigpage": lambda: _huge_dict_file(100000, seed=92, lmin=4, lmax=9, nrows=20000, pages=1, mixed=True),
    "dict_bigpage_two_segments": lambda: _huge_dict_file(3000, seed=93, lmin=2, lmax=12, nrows=40000, pages=2,
                                                         mixed=True),
    # OPTIONAL PLAIN BYTE_ARRAY: a window page; a chunk-chain page whose values
    # start inside chunk 0 past its candidate range, one whose levels fill
    # several chunks; bytes after the last value (the one-pass form does not
    # hold: the general path decodes it)
    "opt_plain_page": lambda: _opt_plain_file(900, seed=61),
    "opt_plain_spec": lambda: _opt_plain_file(6000, seed=62, lmax=40),
    "opt_plain_spec_levels": lambda: _opt_plain_file(20000, seed=63, lmax=12, null_frac=0.5, all_bitpacked=True),
    "opt_plain_extra": lambda: _opt_plain_file(700, seed=64, extra=b"trailing bytes"),
    "opt_plain_spec_extra": lambda: _opt_plain_file(5000, seed=65, extra=b"\x03\x00\x00\x00abc"),
    # RLE level runs that start exactly on 512-row tile edges
    "opt_plain_tile_edges": lambda: B.build_file(
        [B.data_header(len(pay), 1800, 0) + pay for pay in
         [B.levels_section(B.rle(512, 1, 1) + B.rle(512, 0, 1) + B.rle(776, 1, 1)) +
          B.plain_ba([b"v%d" % i for i in range(1288)])]], gen.BYTE_ARRAY, True, 1800),
    # bit width 0: every index is 0
    "bw0_rle": lambda: _dict_ba_file(bytes([0]) + B.rle(10, 0, 0), 10, DICT),
    # literal run then exhaustion -> zero fill
    "exhausted": lambda: _dict_ba_file(bytes([2]) + B.bitpack([3, 2, 1], 2, 1), 20, DICT),
    # out-of-range indices -> NULL
    "oob_index": lambda: _dict_ba_file(bytes([3]) + B.bitpack([0, 7, 4, 3, 5, 1, 6, 2], 3), 8, DICT),
    # zero-group bit-packed run: literal counter wraps, rest read from cursor
    "zero_group_bp": lambda: _dict_ba_file(bytes([2]) + B.rle(2, 1, 2) + B.varint(1) + bytes([0b11100100, 0x1b, 0xff]), 12, DICT),
    # zero-count RLE after a literal run: stale literal cursor
    "zero_count_rle_after_lit": lambda: _dict_ba_file(bytes([2]) + B.bitpack([1, 2, 3, 0, 1, 2, 3, 0], 2) + B.rle(0, 3, 2) + bytes([0x1b, 0xe4]), 16, DICT),
    # more runs than the batched path's run list holds for this page size
    "many_tiny_runs": lambda: _dict_ba_file(bytes([2]) + b"".join(B.rle(1, i % 4, 2) for i in range(40)), 40, DICT),
    # more runs per stream than the three-pass path's run table holds
    "runs_200": lambda: _dict_ba_file(bytes([2]) + b"".join(B.rle(1 + i % 3, i % 4, 2) for i in range(200)), 400, DICT),
    # index stream ends inside a run header (truncated varint)
    "trunc_varint": lambda: _dict_ba_file(bytes([2]) + B.rle(3, 1, 2) + bytes([0x85]), 10, DICT),
    # literal def-level run reading past the level section into the page
    "def_lit_overrun": lambda: _dict_ba_file(bytes([2]) + B.rle(16, 3, 2), 16, DICT,
                                             def_stream=bytes([(2 << 1) | 1, 0xFF])),
    # PLAIN BYTE_ARRAY over several pages, empty strings, a 5000-byte string
    "plain_pages": lambda: B.build_file([B.data_header(len(B.plain_ba(v)), len(v), 0) + B.plain_ba(v) for v in
                                         ([b"a", b"", b"bcd"], [b"x" * 5000], [b"", b""], [b"tail-%d" % i for i in range(300)])],
                                        gen.BYTE_ARRAY, False, 306),
    # PLAIN BYTE_ARRAY pages larger than every LDS window: speculative chain
    # walk, strings longer than a slice's candidate range, a 50 KB string
    "plain_big": lambda: _big_plain_file(seed=21),
    # PLAIN pages over a window: speculative chunk chains linked per page
    "plain_spec": lambda: _spec_plain_file(seed=41),
    "plain_spec_binary": lambda: _spec_plain_file(seed=42, binary=True),
    "plain_spec_empty_strings": lambda: _spec_plain_file(seed=43, lmax=3, n=9000),
    # fewer values declared than the page holds: later bytes are never read
    "plain_spec_extra": lambda: _spec_plain_file(seed=44, nvals=2100),
    "plain_spec_extra_trunc": lambda: _spec_plain_file(seed=45, nvals=1000, cut=500),
    # 60-byte strings: chains entering chunks past the candidate range (fallback)
    "plain_spec_long": lambda: _spec_plain_file(seed=46, lmax=120),
    # multi-byte varint run header (count 300)
    "long_rle_run": lambda: _dict_ba_file(bytes([2]) + B.rle(300, 2, 2), 300, DICT),
    # def levels + nulls, RLE and bit-packed level runs
    "levels_mixed": lambda: _dict_ba_file(bytes([2]) + B.rle(5, 3, 2) + B.bitpack([0, 1, 2, 3, 0, 1, 2, 3], 2), 20, DICT,
                                          def_stream=B.bitpack([1, 0, 1, 1, 0, 1, 1, 1], 1) + B.rle(12, 1, 1)),
    # wide bit width (40 bits): low 32 bits taken, as static_cast<int32_t>
    "bw40": lambda: _dict_ba_file(bytes([40]) + B.bitpack([0, 1, 2, 3, 1 << 33, (1 << 32) + 2, 3, 1], 40), 8, DICT),
    # dictionary encoding without a dictionary page: PLAIN path (column_reader.cpp:177 vs 213)
    "dict_enc_no_dict": lambda: B.build_file([B.data_header(len(B.plain_ba([b"x", b"yz"])), 2, 8) + B.plain_ba([b"x", b"yz"])],
                                             gen.BYTE_ARRAY, False, 2),
    # unknown page type (INDEX_PAGE) is skipped
    "index_page_skipped": lambda: B.build_file([B.data_header(3, 0, 0, ptype=1) + b"abc",
                                                B.data_header(len(B.plain_ba([b"q"])), 1, 0) + B.plain_ba([b"q"])],
                                               gen.BYTE_ARRAY, False, 1),
    # INT96 plain -> "INT96(hi:lo)" string
    "int96": lambda: B.build_file([B.data_header(24, 2, 0) + struct.pack("<qiqi", -5, 7, 1 << 40, -1)],
                                  gen.INT96, False, 2),
    # BOOLEAN plain bits over non-null values only
    "bool_bits": lambda: B.build_file([B.data_header(len(B.levels_section(B.bitpack([1, 0, 1, 1, 1, 0, 1, 1], 1))) + 1, 8, 0)
                                       + B.levels_section(B.bitpack([1, 0, 1, 1, 1, 0, 1, 1], 1)) + bytes([0b101101])],
                                      gen.BOOLEAN, True, 8),
    # OPTIONAL INT64 over several 512-row tiles: bit-packed and RLE level runs
    "opt_int64_tiles": lambda: _opt_fixed_file(gen.INT64, "<q", 1700, seed=5),
    # OPTIONAL DOUBLE, one long all-valid RLE level run then nulls
    "opt_double_rle_levels": lambda: _opt_fixed_file(gen.DOUBLE, "<d", 1300, seed=6, rle_levels=True),
    # OPTIONAL INT96
    "opt_int96": lambda: _opt_fixed_file(gen.INT96, "<qi", 600, seed=7),
    # OPTIONAL fixed width, def streams for the workgroup run builder (run_spec.hpp):
    # exhausted before the value count (zero levels), many one-group literal
    # runs, a zero-count run (exact serial path)
    "opt_levels_exhausted": lambda: _opt_levels_file(B.rle(2000, 1, 1), 3000, 2000, seed=51),
    "opt_levels_tiny_runs": lambda: _opt_levels_file(b"".join(B.bitpack([1, 0, 1, 1, 0, 1, 1, 1], 1) + B.rle(9, 1, 1)
                                                              for _ in range(300)), 5100, 300 * 15, seed=52),
    "opt_levels_zero_run": lambda: _opt_levels_file(B.bitpack([1] * 16, 1) + B.rle(0, 1, 1) + B.rle(100, 1, 1),
                                                    116, 116, seed=53),
    # REQUIRED INT32 over several tiles, pages of different sizes
    "req_int32_tiles": lambda: B.build_file([B.data_header(4 * n, n, 0) + struct.pack(f"<{n}i", *range(-n, 0))
                                             for n in (1500, 1, 513)], gen.INT32, False, 2014),
    # pages over kPipeSmallRows rows (k_pipe_big): speculative run headers,
    # pointer-doubled jumps, one tile per wave
    "big_opt": lambda: _big_dict_file(5000, seed=31),
    "big_opt_full": lambda: _big_dict_file(32768, seed=32, bw=5),
    "big_required": lambda: _big_dict_file(9000, seed=33, optional=False, bw=4),
    "big_short_literals": lambda: _big_dict_file(4000, seed=34, max_groups=1, run=3),
    "big_long_literals": lambda: _big_dict_file(6000, seed=35, max_groups=63, run=2),
    # index stream runs out: zero fill of the remaining ranks
    "big_exhausted": lambda: _big_dict_file(3000, seed=36, cut=40),
    # zero-count RLE run after a literal run (exact decoder)
    "big_zero_count": lambda: _big_dict_file(3000, seed=37, tail=B.rle(0, 3, 3) + bytes([0x1b, 0xe4]) * 8),
    # index bit width 0 with tiny runs: more runs than the record table holds
    "big_bw0_tiny_runs": lambda: _dict_ba_file(bytes([0]) + b"".join(B.rle(1, 0, 0) for _ in range(3000)), 3000,
                                               DICT),
    # pages past the k_pipe_big limits (rows, bytes) next to small pages
    "big_and_small_pages": lambda: B.build_file(
        [B.dict_header(len(B.plain_ba(DICT)), len(DICT)) + B.plain_ba(DICT)] +
        [B.data_header(len(pay), nv, 8) + pay for nv, pay in
         ((600, bytes([2]) + B.rle(600, 2, 2)), (3000, bytes([2]) + B.rle(2999, 1, 2) + B.rle(1, 3, 2)),
          (100, bytes([2]) + B.rle(100, 3, 2)))], gen.BYTE_ARRAY, False, 3700, dict_at_start=True),
    # empty chunk
    "empty": lambda: B.build_file([], gen.INT64, False, 0),
    # multiple dictionary pages: the latest one is in force
    "two_dicts": lambda: B.build_file([
        B.dict_header(len(B.plain_ba([b"a", b"b"])), 2) + B.plain_ba([b"a", b"b"]),
        B.data_header(3, 4, 8) + bytes([1]) + B.rle(4, 1, 1),
        B.dict_header(len(B.plain_ba([b"X", b"Y"])), 2) + B.plain_ba([b"X", b"Y"]),
        B.data_header(3, 3, 8) + bytes([1]) + B.rle(3, 0, 1)], gen.BYTE_ARRAY, False, 7, dict_at_start=True),
}

ERRORS = {
    # repeated columns: the repetition section's length runs past the page;
    # the page ends before the repetition length word
    "rep_len_overrun": lambda: _rep_pages(gen.INT64, "list", True, 300, 2, seed=103, rep_len_delta=100000),
    "rep_len_missing": lambda: _rep_pages(gen.BYTE_ARRAY, "list", True, 300, 2, seed=104, enc=8,
                                          dict_vals=REP_DICT, cut_after_def=True),
    # spec order, LIST shape: more rows read as non-null than the page holds values
    "rep_spec_order_int64_short": lambda: _rep_pages(gen.INT64, "list", True, 640, 2, seed=102, spec_order=True),
    # dictionary pages beyond LDS: a truncated last entry; more entries
    # declared than the page holds (the chain ends at the page end)
    "huge_dict_truncated": lambda: _huge_dict_file(30000, seed=86, cut=3),
    "huge_dict_short_count": lambda: _huge_dict_file(30000, seed=87, decl=30001),
    # truncated PLAIN BYTE_ARRAY value
    "truncated_plain": lambda: B.build_file([B.data_header(9, 2, 0) + struct.pack("<I", 2) + b"ab" + struct.pack("<I", 9)[:3]],
                                            gen.BYTE_ARRAY, False, 2),
    # PLAIN BYTE_ARRAY: the chain runs out in the second page
    "plain_short_page2": lambda: B.build_file([B.data_header(len(B.plain_ba([b"ok"])), 1, 0) + B.plain_ba([b"ok"]),
                                               B.data_header(len(B.plain_ba([b"abc", b"de"])), 3, 0) + B.plain_ba([b"abc", b"de"])],
                                              gen.BYTE_ARRAY, False, 4),
    # PLAIN BYTE_ARRAY page of 60 KB whose chain overruns in its second window
    "plain_big_overrun": lambda: _big_plain_file(seed=22, cut=40000),
    # speculative chunk path: the last page's chain runs past its end
    "plain_spec_trunc": lambda: _spec_plain_file(seed=47, cut=700),
    "plain_spec_trunc_len": lambda: _spec_plain_file(seed=48, cut=2),
    # more values declared than the page holds: the read at the page end fails
    "plain_spec_short": lambda: _spec_plain_file(seed=49, nvals=3100),
    # OPTIONAL PLAIN BYTE_ARRAY values run out (window page, chunk-chain page)
    "opt_plain_short": lambda: _opt_plain_file(800, seed=66, drop=2),
    "opt_plain_spec_short": lambda: _opt_plain_file(6000, seed=67, lmax=40, drop=5),
    # def_len beyond the page
    "def_len_overrun": lambda: B.build_file([B.data_header(6, 3, 0) + struct.pack("<I", 50) + b"xy"], gen.INT32, True, 3),
    # dictionary page index stream without the bit-width byte
    "missing_bw_byte": lambda: _dict_ba_file(b"", 4, DICT, def_stream=B.rle(4, 0, 1)),
    # data page header without DataPageHeader -> bad_optional_access
    "no_dph": lambda: B.build_file([B.data_header(4, 1, 0, with_dph=False) + b"abcd"], gen.INT32, False, 1),
    # PLAIN INT64 page too short
    "short_int64": lambda: B.build_file([B.data_header(12, 2, 0) + struct.pack("<q", 5) + b"abcd"], gen.INT64, False, 2),
    # REQUIRED INT32, three tiles, values run out inside the second tile
    "req_int32_short_tile2": lambda: B.build_file([B.data_header(4 * 700, 1500, 0) + bytes(4 * 700)],
                                                  gen.INT32, False, 1500),
    # OPTIONAL FLOAT, values run out after a later null-only stretch
    "opt_float_short": lambda: _opt_fixed_file(gen.FLOAT, "<f", 1200, seed=8, drop=3),
    # FLBA with a non-null value
    "flba": lambda: B.build_file([B.data_header(4, 1, 0) + b"abcd"], gen.FLBA, False, 1),
    # dictionary page truncated
    "dict_truncated": lambda: B.build_file([B.dict_header(6, 2) + struct.pack("<I", 1) + b"a" + b"\x05",
                                            B.data_header(3, 2, 8) + bytes([1]) + B.rle(2, 0, 1)],
                                           gen.BYTE_ARRAY, False, 2, dict_at_start=True),
    # zero-count RLE run before any literal run (reference: NULL literal pointer)
    "zero_count_no_literal": lambda: _dict_ba_file(bytes([2]) + B.rle(0, 1, 2) + B.rle(3, 1, 2), 3, DICT),
}


@pytest.mark.parametrize("case", sorted(CRAFTED), ids=sorted(CRAFTED))
def test_crafted_pages(ctx, path, case):
    f, chunk = CRAFTED[case]()
    rc_o, msg_o, d_o = oracle_read_column(f, [chunk])
    assert rc_o == 0, msg_o
    rc_g, msg_g, d_g = gpu_read_column(ctx, f, [chunk])
    assert (rc_g, msg_g) == (0, "")
    assert d_g == d_o


@pytest.mark.parametrize("case", sorted(ERRORS), ids=sorted(ERRORS))
def test_error_pages(ctx, path, case):
    f, chunk = ERRORS[case]()
    rc_o, msg_o, _ = oracle_read_column(f, [chunk])
    assert rc_o != 0
    rc_g, msg_g, _ = gpu_read_column(ctx, f, [chunk])
    assert rc_g == rc_o, (msg_g, msg_o)
    if rc_o in (-2, -4):  # ByteBuffer / FLBA: the reference's exact text
        assert msg_g == msg_o


@pytest.mark.slow
@pytest.mark.parametrize("layout", [gen.REF_LAYOUT, gen.ARROW_LAYOUT], ids=["ref", "arrow"])
def test_c2_full_size_properties(ctx, layout):
    """BASELINE config #2 at full size (10M rows), in both layouts (arrow =
    20,000-row pages, the k_pipe_big path): validity/length/content properties
    plus sha256 of the canonical dump against the generator's own values."""
    cols = gen.c2_cols()
    n = 10_000_000
    f = gen.build(cols, n, 1, seed=gen.CONFIG_SEEDS["C2"], layout=layout)
    chunks = file_chunks(f, 0)
    dc = ctx.upload(f, chunks)
    dc.decode()
    host = dc.to_host()
    dc.free()
    assert host.num_rows == n
    # offsets monotone, chars length consistent
    assert np.all(np.diff(host.offsets) >= 0)
    assert host.offsets[-1] == len(host.data)
    # nulls carry no bytes
    lens = np.diff(host.offsets)
    assert np.all(lens[host.validity == 0] == 0)
    got = hashlib.sha256(capi.canonical_dump(host)).hexdigest()
    exp = hashlib.sha256(gen.values_dump(cols[0], 0, n, 0, gen.CONFIG_SEEDS["C2"])).hexdigest()
    assert got == exp



@pytest.mark.parametrize("case", ["plain_spec", "plain_spec_binary", "plain_spec_empty_strings", "plain_spec_extra",
                                  "plain_spec_extra_trunc"])
def test_plain_spec_no_fallback(ctx, case):
    """Pages of short strings stay on the speculative chunk path (no generic
    re-run): the second decode launches k_plain_spec again."""
    f, chunk = CRAFTED[case]()
    dc = ctx.upload(f, [to_desc_(chunk)])
    dc.decode()
    ctx.timing(True)
    ctx.timing_reset()
    dc.decode_async()
    ctx.sync()
    ms, n = ctx.timing_get("plain_spec")
    gms, gn = ctx.timing_get("ba_rows")
    ctx.timing(False)
    dc.decode_check()
    dc.free()
    assert n == 1 and gn == 0


@pytest.mark.parametrize("key,value", [("write_waves", 0), ("write_waves", 17), ("pipe_run_pages", 33),
                                       ("regex_win", 1000), ("fused_claim", 0), ("regex_index", 3), ("no_such_option", 1)])
def test_set_option_rejects(ctx, key, value):
    """Out-of-range tuning values and unknown keys fail with PQ_ERR_ARG and
    leave the setting alone."""
    with pytest.raises(capi.PqError) as e:
        ctx.set_option(key, value)
    assert e.value.code == -20 and key in e.value.msg


def to_desc_(chunk):
    from util import to_desc
    return chunk if isinstance(chunk, capi.ChunkDesc) else to_desc(chunk)


@pytest.mark.gpu
@pytest.mark.parametrize("layout", [gen.REF_LAYOUT, gen.ARROW_LAYOUT], ids=["ref", "arrow"])
def test_row_groups_over_two_contexts(ctx, layout):
    """Row groups alternated over two contexts (two HIP streams, as bench.py's
    C5 leg runs them): after one sizing decode, rounds of decodes queued on
    both streams before any check; every row group then equals the oracle."""
    cols = gen.c2_cols()
    f = gen.build(cols, 30000, 4, seed=17, layout=layout, rows_per_page=20000)
    chunks = file_chunks(f, 0)
    ctx2 = capi.Context(0)
    try:
        dcs = [(ctx if i % 2 == 0 else ctx2).upload(f, [to_desc(c)]) for i, c in enumerate(chunks)]
        for dc in dcs:  # sizes the outputs (decode_check does not fill the column record)
            dc.decode()
        for _ in range(3):
            for dc in dcs:
                dc.decode_async()
            for dc in dcs:
                dc.decode_check()
        for c, dc in zip(chunks, dcs):
            rc_o, _, d_o = oracle_read_column(f, [c])
            assert rc_o == 0
            assert capi.canonical_dump(dc.to_host()) == d_o
        for dc in dcs:
            dc.free()
    finally:
        ctx2.close()


@pytest.mark.gpu
@pytest.mark.parametrize("wide", [1, 0], ids=["wide_rows", "serial"])
@pytest.mark.parametrize("name,col,rows", [
    ("dict100k_opt", gen.Col("s", gen.DICT_STRINGS, gen.BYTE_ARRAY, optional=True, null_frac=0.05, dict_size=100_000,
                             len_min=4, len_max=12, max_run=1), 120_000),
    ("dict100k_req", gen.Col("s", gen.DICT_STRINGS, gen.BYTE_ARRAY, dict_size=100_000, len_min=4, len_max=12,
                             max_run=3), 200_000),
    ("dict_bw19_sparse", gen.Col("s", gen.DICT_STRINGS, gen.BYTE_ARRAY, optional=True, null_frac=0.6,
                                 dict_size=3_000_000, len_min=5, len_max=8, max_run=1), 700_000),
], ids=lambda v: v if isinstance(v, str) else "")
def test_wide_dictionary_20k_pages(ctx, wide, name, col, rows):
    """Dictionaries beyond the pipe's LDS (17-20-bit indices) on pyarrow-sized
    20,000-row pages: the generic rows pass by a workgroup per page
    (k_wide_rows: speculative run records for both streams) and by the
    wave-per-page walk, both equal to the oracle."""
    ctx.set_option("wide_rows", wide)
    try:
        f = gen.build([col], rows, 1, seed=21, layout=gen.ARROW_LAYOUT)
        chunks = file_chunks(f, 0)
        rc_o, msg_o, d_o = oracle_read_column(f, chunks)
        rc_g, msg_g, d_g = gpu_read_column(ctx, f, chunks)
        assert (rc_g, msg_g) == (rc_o, msg_o)
        assert d_g == d_o
    finally:
        ctx.set_option("wide_rows", 1)
