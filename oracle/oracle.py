"""ctypes bindings for the parity checker — TEST INFRASTRUCTURE ONLY.

`liboracle.so` is the plain-C restatement of the reference decode path
(oracle/pq_oracle.c); `_ref/libpqref.so` is the reference itself, compiled
from its own sources by oracle/Makefile.  Only tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg import this module, and only as the checker.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_ORACLE = os.path.join(HERE, "liboracle.so")
_REF = os.path.join(HERE, "_ref", "libpqref.so")

u8p = C.POINTER(C.c_uint8)
i64p = C.POINTER(C.c_int64)


class PqoChunk(C.Structure):
    _fields_ = [
        ("num_values", C.c_int64),
        ("data_page_offset", C.c_int64),
        ("dictionary_page_offset", C.c_int64),
        ("has_dictionary_page_offset", C.c_int32),
        ("codec", C.c_int32),
        ("type", C.c_int32),
        ("max_def_level", C.c_int16),
        ("max_rep_level", C.c_int16),
    ]


class PqoPage(C.Structure):
    _fields_ = [
        ("page_num", C.c_int32),
        ("page_type", C.c_int32),
        ("num_values", C.c_int32),
        ("first_row", C.c_int64),
        ("nrows", C.c_int64),
    ]


class PqoColumn(C.Structure):
    _fields_ = [
        ("nrows", C.c_int64),
        ("type", C.c_int32),
        ("valid", u8p),
        ("offsets", i64p),
        ("data", u8p),
        ("data_len", C.c_int64),
        ("pages", C.POINTER(PqoPage)),
        ("npages", C.c_int32),
    ]


@dataclass
class Chunk:
    """ColumnMetaData + ColumnInfo fields the decode path reads."""

    num_values: int
    data_page_offset: int
    dictionary_page_offset: int | None
    codec: int
    type: int
    max_def: int
    max_rep: int

    def c(self) -> PqoChunk:
        d = self.dictionary_page_offset
        return PqoChunk(self.num_values, self.data_page_offset, d if d is not None else 0,
                        1 if d is not None else 0, self.codec, self.type, self.max_def, self.max_rep)


@dataclass
class Column:
    valid: np.ndarray   # uint8 [n]
    offsets: np.ndarray  # int64 [n+1]
    data: np.ndarray    # uint8
    pages: list          # (page_num, type, num_values, first_row, nrows)
    type: int


_lib = None
_ref = None


def lib():
    global _lib
    if _lib is None:
        L = C.CDLL(_ORACLE)
        L.pqo_read_all.argtypes = [u8p, C.c_size_t, C.POINTER(PqoChunk), C.POINTER(PqoColumn),
                                   C.c_char_p, C.c_size_t]
        L.pqo_free.argtypes = [C.POINTER(PqoColumn)]
        L.pqo_dump.argtypes = [C.POINTER(PqoColumn), C.POINTER(u8p), C.POINTER(C.c_size_t)]
        L.pqo_free_buf.argtypes = [C.c_void_p]
        L.pqo_rle_decode.argtypes = [u8p, C.c_uint32, C.c_uint32, C.POINTER(C.c_int32), C.c_uint32]
        L.pqo_chunk_assign.argtypes = [u8p, C.POINTER(C.c_int64), C.c_int64, C.c_int64, C.POINTER(C.c_int64),
                                       C.POINTER(C.c_int64)]
        L.pqo_chunk_assign.restype = None
        _lib = L
    return _lib


def have_ref() -> bool:
    return os.path.exists(_REF)


def ref():
    global _ref
    if _ref is None:
        L = C.CDLL(_REF)
        common = [u8p, C.c_size_t, C.c_int64, C.c_int64, C.c_int64, C.c_int, C.c_int32, C.c_int32,
                  C.c_int16, C.c_int16, C.POINTER(u8p), C.POINTER(C.c_size_t)]
        L.pqref_read_all.argtypes = common + [C.c_char_p, C.c_size_t]
        L.pqref_read_pages.argtypes = common + [i64p, C.c_int, C.POINTER(C.c_int), C.c_char_p,
                                                C.c_size_t]
        L.pqref_open.argtypes = [C.c_char_p, i64p, i64p, i64p, C.c_int, i64p, C.c_int64, i64p,
                                 C.c_char_p, C.c_size_t]
        L.pqref_read_column.argtypes = [C.c_char_p, C.c_char_p, C.POINTER(u8p),
                                        C.POINTER(C.c_size_t), C.c_char_p, C.c_size_t]
        L.pqref_write.argtypes = [C.c_char_p, C.c_int, C.POINTER(C.c_char_p), C.POINTER(C.c_int32),
                                  C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(u8p),
                                  C.c_int64, C.c_char_p, C.c_size_t]
        L.pqref_time_read_all.argtypes = [u8p, C.c_size_t, C.c_int64, C.c_int64, C.c_int64, C.c_int,
                                          C.c_int32, C.c_int16, C.c_int16, C.c_int, C.c_int, i64p]
        L.pqref_time_read_all.restype = C.c_double
        L.pqref_time_read_all_multi.argtypes = [C.c_int, C.POINTER(u8p), C.POINTER(C.c_size_t), i64p, i64p, i64p,
                                                C.POINTER(C.c_int32), C.c_int32, C.c_int16, C.c_int16, C.c_int,
                                                C.c_int, i64p]
        L.pqref_time_read_all_multi.restype = C.c_double
        L.pqref_free.argtypes = [C.c_void_p]
        _ref = L
    return _ref


def _buf(b: bytes):
    return C.cast(C.c_char_p(b), u8p)


def read_all(file: bytes, ch: Chunk):
    """Oracle decode -> (rc, message, Column | None)."""
    L = lib()
    col = PqoColumn()
    err = C.create_string_buffer(512)
    cc = ch.c()
    rc = L.pqo_read_all(_buf(file), len(file), C.byref(cc), C.byref(col), err, 512)
    if rc != 0:
        return rc, err.value.decode(errors="replace"), None
    n = col.nrows
    valid = np.ctypeslib.as_array(col.valid, shape=(max(n, 1),))[:n].copy()
    offsets = np.ctypeslib.as_array(col.offsets, shape=(n + 1,)).copy()
    data = (np.ctypeslib.as_array(col.data, shape=(max(col.data_len, 1),))[:col.data_len].copy())
    pages = [(col.pages[i].page_num, col.pages[i].page_type, col.pages[i].num_values,
              col.pages[i].first_row, col.pages[i].nrows) for i in range(col.npages)]
    out = Column(valid, offsets, data, pages, col.type)
    L.pqo_free(C.byref(col))
    return 0, "", out


def dump_column(col: Column) -> bytes:
    """Canonical dump built from a columnar result."""
    return canonical_dump(col.valid, col.offsets, col.data, col.type)


def canonical_dump(valid, offsets, data, ptype: int) -> bytes:
    var = ptype in (3, 6)
    n = len(valid)
    valid = np.asarray(valid, dtype=np.uint8)
    offsets = np.asarray(offsets, dtype=np.int64)
    lens = np.where(valid != 0, np.diff(offsets), 0).astype(np.int64)
    rec = 1 + lens + (4 * (valid != 0) if var else 0)
    total = int(rec.sum())
    out = np.zeros(total, dtype=np.uint8)
    starts = np.concatenate([[0], np.cumsum(rec)[:-1]]) if n else np.zeros(0, np.int64)
    out[starts] = (valid == 0).astype(np.uint8)
    nz = np.nonzero(valid)[0]
    if len(nz):
        pay = starts[nz] + 1
        if var:
            l32 = lens[nz].astype("<u4").view(np.uint8).reshape(-1, 4)
            for k in range(4):
                out[pay + k] = l32[:, k]
            pay = pay + 4
        # scatter payload bytes
        L = lens[nz]
        src_start = offsets[nz]
        tot = int(L.sum())
        if tot:
            rep_dst = np.repeat(pay - np.concatenate([[0], np.cumsum(L)[:-1]]), L)
            rep_src = np.repeat(src_start - np.concatenate([[0], np.cumsum(L)[:-1]]), L)
            ar = np.arange(tot, dtype=np.int64)
            out[rep_dst + ar] = np.asarray(data, dtype=np.uint8)[rep_src + ar]
    return out.tobytes()


def rle_decode(stream: bytes, bit_width: int, count: int):
    out = (C.c_int32 * max(count, 1))()
    rc = lib().pqo_rle_decode(_buf(stream), len(stream), bit_width, out, count)
    return rc, list(out)[:count]


# ── the reference itself ───────────────────────────────────────────────────

def _take(p, n) -> bytes:
    b = C.string_at(p, n) if n else b""
    ref().pqref_free(p)
    return b


def ref_read_all(file: bytes, ch: Chunk):
    R = ref()
    p = u8p()
    n = C.c_size_t()
    err = C.create_string_buffer(512)
    d = ch.dictionary_page_offset
    rc = R.pqref_read_all(_buf(file), len(file), ch.num_values, ch.data_page_offset,
                          d if d is not None else 0, 1 if d is not None else 0, ch.codec, ch.type,
                          ch.max_def, ch.max_rep, C.byref(p), C.byref(n), err, 512)
    if rc != 0:
        return rc, err.value.decode(errors="replace"), None
    return 0, "", _take(p, n.value)


def ref_read_pages(file: bytes, ch: Chunk, cap: int = 1 << 20, lib_=None):
    R = lib_ or ref()
    p = u8p()
    n = C.c_size_t()
    err = C.create_string_buffer(512)
    pages = (C.c_int64 * (4 * cap))()
    npages = C.c_int()
    d = ch.dictionary_page_offset
    rc = R.pqref_read_pages(_buf(file), len(file), ch.num_values, ch.data_page_offset,
                            d if d is not None else 0, 1 if d is not None else 0, ch.codec, ch.type,
                            ch.max_def, ch.max_rep, C.byref(p), C.byref(n), pages, cap,
                            C.byref(npages), err, 512)
    if rc != 0:
        return rc, err.value.decode(errors="replace"), None, None
    pl = [tuple(pages[4 * i:4 * i + 4]) for i in range(min(npages.value, cap))]
    return 0, "", _take(p, n.value), pl


def ref_open(path: str, meta_cap: int = 4096, pidx_cap: int = 1 << 22):
    """-> (chunks[rg][col] as Chunk, num_rows[rg], page_index[(off,size,rg,col)])."""
    R = ref()
    nrg, ncol, npg = C.c_int64(), C.c_int64(), C.c_int64()
    meta = (C.c_int64 * (8 * meta_cap))()
    pidx = np.zeros(4 * pidx_cap, dtype=np.int64)
    err = C.create_string_buffer(512)
    rc = R.pqref_open(path.encode(), C.byref(nrg), C.byref(ncol), meta, meta_cap,
                      pidx.ctypes.data_as(i64p), pidx_cap, C.byref(npg), err, 512)
    if rc != 0:
        raise RuntimeError(err.value.decode())
    chunks, rows = [], []
    k = 0
    for rg in range(nrg.value):
        row = []
        for c in range(ncol.value):
            m = meta[8 * k:8 * k + 8]
            k += 1
            row.append(Chunk(m[0], m[1], m[2] if m[2] >= 0 else None, m[3], m[4], m[5], m[6]))
            if c == 0:
                rows.append(m[7])
        chunks.append(row)
    npages = min(npg.value, pidx_cap)
    return chunks, rows, pidx[:4 * npages].reshape(-1, 4)


def ref_read_column(path: str, name: str, lib_=None):
    R = lib_ or ref()
    p = u8p()
    n = C.c_size_t()
    err = C.create_string_buffer(512)
    rc = R.pqref_read_column(path.encode(), name.encode(), C.byref(p), C.byref(n), err, 512)
    if rc != 0:
        return rc, err.value.decode(errors="replace"), None
    b = C.string_at(p, n.value) if n.value else b""
    R.pqref_free(p)
    return 0, "", b


_REF_GPU = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_ref", "librefgpu.so")
_ref_gpu = None


def have_ref_gpu() -> bool:
    return os.path.exists(_REF_GPU)


def ref_gpu():
    """The reference's own ParquetReader / ColumnReader with the bodies of
    read_all and read_pages replaced by INTEGRATION.md path B (integration/column_reader_gpu.cpp over
    libpqgpu.so): the maintainer-side binding, built by `make refgpu`."""
    global _ref_gpu
    if _ref_gpu is None:
        L = C.CDLL(_REF_GPU)
        L.pqref_read_column.argtypes = [C.c_char_p, C.c_char_p, C.POINTER(u8p), C.POINTER(C.c_size_t), C.c_char_p,
                                        C.c_size_t]
        common = [u8p, C.c_size_t, C.c_int64, C.c_int64, C.c_int64, C.c_int, C.c_int32, C.c_int32,
                  C.c_int16, C.c_int16, C.POINTER(u8p), C.POINTER(C.c_size_t)]
        L.pqref_read_all.argtypes = common + [C.c_char_p, C.c_size_t]
        L.pqref_read_pages.argtypes = common + [i64p, C.c_int, C.POINTER(C.c_int), C.c_char_p, C.c_size_t]
        L.pqref_free.argtypes = [C.c_void_p]
        _ref_gpu = L
    return _ref_gpu


def ref_write(path: str, cols: list, nrows: int):
    """cols: list of (name, type, repetition, converted or -1, canonical_dump bytes)."""
    R = ref()
    n = len(cols)
    names = (C.c_char_p * n)(*[c[0].encode() for c in cols])
    types = (C.c_int32 * n)(*[c[1] for c in cols])
    reps = (C.c_int32 * n)(*[c[2] for c in cols])
    conv = (C.c_int32 * n)(*[c[3] for c in cols])
    keep = [C.create_string_buffer(c[4], len(c[4]) or 1) for c in cols]
    dumps = (u8p * n)(*[C.cast(k, u8p) for k in keep])
    err = C.create_string_buffer(512)
    rc = R.pqref_write(path.encode(), n, names, types, reps, conv, dumps, nrows, err, 512)
    if rc != 0:
        raise RuntimeError(err.value.decode())


def ref_time_read_all(file: bytes, ch: Chunk, reps: int = 1, threads: int = 1):
    """Wall seconds for reps x ColumnReader::read_all on `threads` readers."""
    R = ref()
    nv = C.c_int64()
    d = ch.dictionary_page_offset
    keep = C.create_string_buffer(file, len(file))
    s = R.pqref_time_read_all(C.cast(keep, u8p), len(file), ch.num_values, ch.data_page_offset,
                              d if d is not None else 0, 1 if d is not None else 0, ch.type,
                              ch.max_def, ch.max_rep, reps, threads, C.byref(nv))
    return s, nv.value


def ref_time_read_all_multi(shards, ptype: int, max_def: int, max_rep: int, reps: int = 1, threads: int = 1):
    """Wall seconds for `reps` rounds of ColumnReader::read_all over every
    (file bytes, Chunk) shard, on `threads` readers (page-parallel baseline)."""
    R = ref()
    n = len(shards)
    keep = [C.create_string_buffer(f, len(f) or 1) for f, _ in shards]
    files = (u8p * n)(*[C.cast(k, u8p) for k in keep])
    lens = (C.c_size_t * n)(*[len(f) for f, _ in shards])
    nv = (C.c_int64 * n)(*[c.num_values for _, c in shards])
    do = (C.c_int64 * n)(*[c.data_page_offset for _, c in shards])
    dd = (C.c_int64 * n)(*[c.dictionary_page_offset or 0 for _, c in shards])
    hd = (C.c_int32 * n)(*[1 if c.dictionary_page_offset is not None else 0 for _, c in shards])
    out = C.c_int64()
    s = R.pqref_time_read_all_multi(n, files, lens, nv, do, dd, hd, ptype, max_def, max_rep, reps, threads,
                                    C.byref(out))
    return s, out.value


def ref_time_regex_pages_multi(shards, ptype: int, max_def: int, max_rep: int, page_counts, pattern: str,
                               neg: bool = False, reps: int = 1, threads: int = 1):
    """Regex CPU baseline: `reps` rounds of ColumnReader::read_all over every
    shard on `threads` threads, each page's values tested with the build's
    host DFA (libpqgpu pq_regex_host_match) until one satisfies the
    predicate.  page_counts[i]: shard i's data-page row counts.  Returns
    (wall seconds, page flags)."""
    import numpy as np
    from pqgpu import capi
    R = ref()
    L = capi.lib()
    L.pq_regex_host_new.restype = C.c_void_p
    L.pq_regex_host_new.argtypes = [C.c_char_p]
    L.pq_regex_host_free.argtypes = [C.c_void_p]
    h = L.pq_regex_host_new(pattern.encode())
    if not h:
        raise ValueError(f"pattern {pattern!r}: no host DFA")
    n = len(shards)
    keep = [C.create_string_buffer(f, len(f) or 1) for f, _ in shards]
    files = (u8p * n)(*[C.cast(k, u8p) for k in keep])
    lens = (C.c_size_t * n)(*[len(f) for f, _ in shards])
    nv = (C.c_int64 * n)(*[c.num_values for _, c in shards])
    do = (C.c_int64 * n)(*[c.data_page_offset for _, c in shards])
    dd = (C.c_int64 * n)(*[c.dictionary_page_offset or 0 for _, c in shards])
    hd = (C.c_int32 * n)(*[1 if c.dictionary_page_offset is not None else 0 for _, c in shards])
    first = np.concatenate([[0], np.cumsum([len(c) for c in page_counts])]).astype(np.int64)
    cnt = np.ascontiguousarray(np.concatenate([np.asarray(c, np.int32) for c in page_counts]), dtype=np.int32)
    flags = np.zeros(max(int(first[-1]), 1), dtype=np.uint8)
    fn = C.cast(L.pq_regex_host_match, C.c_void_p)
    R.pqref_time_regex_pages_multi.restype = C.c_double
    R.pqref_time_regex_pages_multi.argtypes = [
        C.c_int, C.POINTER(u8p), C.POINTER(C.c_size_t), C.POINTER(C.c_int64), C.POINTER(C.c_int64),
        C.POINTER(C.c_int64), C.POINTER(C.c_int32), C.c_int32, C.c_int16, C.c_int16, C.c_void_p, C.c_void_p,
        C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p]
    try:
        s = R.pqref_time_regex_pages_multi(n, files, lens, nv, do, dd, hd, ptype, max_def, max_rep,
                                           first.ctypes.data, cnt.ctypes.data, fn, h, int(neg), reps, threads,
                                           flags.ctypes.data)
    finally:
        L.pq_regex_host_free(h)
    return s, flags[:int(first[-1])]


def chunk_assign(col: Column, chunk_size: int = 4096):
    """src/main.cpp:17-32 restated (pqo_chunk_assign) over an oracle column:
    (tuple_to_chunk int64[nrows], num_chunks)."""
    import numpy as np
    n = len(col.valid)
    valid = np.ascontiguousarray(np.asarray(col.valid, dtype=np.uint8))
    offs = np.ascontiguousarray(np.asarray(col.offsets, dtype=np.int64))
    out = np.zeros(max(n, 1), dtype=np.int64)
    k = C.c_int64()
    lib().pqo_chunk_assign(valid.ctypes.data_as(u8p), offs.ctypes.data_as(C.POINTER(C.c_int64)), n, chunk_size,
                           out.ctypes.data_as(C.POINTER(C.c_int64)), C.byref(k))
    return out[:n], k.value
