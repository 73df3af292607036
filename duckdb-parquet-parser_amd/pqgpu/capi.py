"""ctypes binding of the C ABI in include/pq_gpu.h (libpqgpu.so).

Python is plumbing here (tests, bench); the product is the C ABI and its HIP
kernels.  Every call goes through libpqgpu.so; there is no CPU fallback — a
missing library or GPU raises.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _paths

PQ_ERRORS = {
    -1: "CODEC", -2: "BUFFER", -3: "OPTIONAL", -4: "FLBA", -5: "TYPE", -6: "THRIFT",
    -7: "ALLOC", -8: "UNSUPPORTED", -9: "DECOMPRESS", -20: "ARG", -21: "HIP", -22: "REGEX",
}
EXT_CODECS, EXT_PAGE_V2 = 1, 2          # pq_chunk_desc.ext_flags
PAGE_COMPRESSED, PAGE_V2 = 1, 2         # pq_page_desc.flags (codec in bits 8..15)
BOOLEAN, INT32, INT64, INT96, FLOAT, DOUBLE, BYTE_ARRAY, FLBA = range(8)
WIDTH = {BOOLEAN: 1, INT32: 4, FLOAT: 4, INT64: 8, DOUBLE: 8, INT96: 12}


class PqError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"[{PQ_ERRORS.get(code, code)}] {msg}")
        self.code = code
        self.msg = msg


class ChunkDesc(C.Structure):
    _fields_ = [
        ("num_values", C.c_int64),
        ("data_page_offset", C.c_int64),
        ("dictionary_page_offset", C.c_int64),
        ("has_dictionary_page_offset", C.c_int32),
        ("codec", C.c_int32),
        ("type", C.c_int32),
        ("max_def_level", C.c_int16),
        ("max_rep_level", C.c_int16),
        ("total_compressed_size", C.c_int64),
        ("ext_flags", C.c_int32),
        ("ext_reserved", C.c_int32),
    ]


class PageDesc(C.Structure):
    _fields_ = [
        ("header_offset", C.c_int64),
        ("payload_offset", C.c_int64),
        ("payload_size", C.c_int32),
        ("page_type", C.c_int32),
        ("num_values", C.c_int32),
        ("encoding", C.c_int32),
        ("page_num", C.c_int32),
        ("dict_page", C.c_int32),
        ("first_row", C.c_int64),
        ("uncompressed_size", C.c_int32),
        ("flags", C.c_int32),
        ("v2_def_len", C.c_int32),
        ("v2_rep_len", C.c_int32),
    ]


class ColumnOut(C.Structure):
    _fields_ = [
        ("num_rows", C.c_int64),
        ("type", C.c_int32),
        ("value_width", C.c_int32),
        ("d_validity", C.c_void_p),
        ("d_values", C.c_void_p),
        ("d_offsets", C.c_void_p),
        ("num_bytes", C.c_int64),
        ("capacity_rows", C.c_int64),
        ("capacity_bytes", C.c_int64),
    ]


_lib = None
vp = C.c_void_p
u8p = C.POINTER(C.c_uint8)


def lib():
    global _lib
    if _lib is None:
        L = C.CDLL(_paths.lib_path("libpqgpu.so"))
        sig = {
            "pq_device_count": ([], C.c_int),
            "pq_plan_page_ranges": ([C.POINTER(PageDesc), C.c_int64, C.c_int, C.POINTER(C.c_int64)], C.c_int),
            "pq_ctx_create": ([C.c_int], vp),
            "pq_ctx_destroy": ([vp], None),
            "pq_last_error": ([vp], C.c_char_p),
            "pq_ctx_stream": ([vp], vp),
            "pq_ctx_sync": ([vp], C.c_int),
            "pq_ctx_set_option": ([vp, C.c_char_p, C.c_int64], C.c_int),
            "pq_device_buffer": ([vp, u8p, C.c_size_t, C.POINTER(vp)], C.c_int),
            "pq_device_buffer_free": ([vp, vp], None),
            "pq_build_page_table_device": ([vp, vp, C.c_size_t, C.c_int64, C.POINTER(ChunkDesc), C.c_int64,
                                            C.c_int64, C.POINTER(PageDesc), C.c_int64, C.POINTER(C.c_int64)],
                                           C.c_int),
            "pq_build_page_table": ([u8p, C.c_size_t, C.POINTER(ChunkDesc), C.POINTER(PageDesc),
                                     C.c_int64, C.POINTER(C.c_int64), C.c_char_p, C.c_size_t], C.c_int),
            "pq_chunk_upload": ([vp, u8p, C.c_size_t, C.POINTER(ChunkDesc), C.c_int,
                                 C.POINTER(vp)], C.c_int),
            "pq_chunk_upload_range": ([vp, u8p, C.c_size_t, C.POINTER(ChunkDesc), C.POINTER(PageDesc),
                                       C.c_int64, C.c_int64, C.c_int64, C.POINTER(vp)], C.c_int),
            "pq_chunk_free": ([vp, vp], None),
            "pq_chunk_first_row": ([vp], C.c_int64),
            "pq_chunk_num_rows": ([vp], C.c_int64),
            "pq_chunk_num_pages": ([vp], C.c_int64),
            "pq_chunk_payload_bytes": ([vp], C.c_int64),
            "pq_chunk_pages": ([vp, C.POINTER(PageDesc), C.c_int64, C.POINTER(C.c_int64)], C.c_int),
            "pq_decode": ([vp, vp, C.POINTER(ColumnOut)], C.c_int),
            "pq_decode_async": ([vp, vp, C.POINTER(ColumnOut)], C.c_int),
            "pq_decode_check": ([vp, vp], C.c_int),
            "pq_column_copy_out": ([vp, C.POINTER(ColumnOut), vp, vp, vp], C.c_int),
            "pq_column_free": ([vp, C.POINTER(ColumnOut)], None),
            "pq_chunk_assign": ([vp, C.POINTER(ColumnOut), C.c_int64, vp, vp, C.POINTER(C.c_int64)], C.c_int),
            "pq_regex_compile_check": ([C.c_char_p, C.c_char_p, C.c_size_t], C.c_int),
            "pq_regex_pages": ([vp, vp, C.c_char_p, C.c_int, vp], C.c_int),
            "pq_decode_regex_async": ([vp, vp, C.POINTER(ColumnOut), C.c_char_p, C.c_int], C.c_int),
            "pq_regex_pages_async": ([vp, vp, C.c_char_p, C.c_int], C.c_int),
            "pq_regex_pages_result": ([vp, vp, vp], C.c_int),
            "pq_regex_match_host": ([C.c_char_p, u8p, C.c_size_t], C.c_int),
            "pq_regex_match_host_dfa": ([C.c_char_p, u8p, C.c_size_t], C.c_int),
            "pq_regex_dfa_sinks": ([C.c_char_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)], C.c_int),
            "pq_timing_enable": ([vp, C.c_int], None),
            "pq_timing_reset": ([vp], None),
            "pq_timing_get": ([vp, C.c_char_p, C.POINTER(C.c_double), C.POINTER(C.c_int64)], C.c_int),
            "pq_fused_prof_read": ([vp, C.POINTER(C.c_uint64), C.c_int], C.c_int),
            "pq_file_open": ([u8p, C.c_size_t, C.POINTER(vp), C.c_char_p, C.c_size_t], C.c_int),
            "pq_file_close": ([vp], None),
            "pq_file_num_rows": ([vp], C.c_int64),
            "pq_file_num_row_groups": ([vp], C.c_int),
            "pq_file_num_columns": ([vp], C.c_int),
            "pq_file_column_name": ([vp, C.c_int, C.c_char_p, C.c_size_t], C.c_int),
            "pq_file_find_column": ([vp, C.c_char_p], C.c_int),
            "pq_file_chunk": ([vp, C.c_int, C.c_int, C.POINTER(ChunkDesc)], C.c_int),
            "pq_file_row_group_rows": ([vp, C.c_int], C.c_int64),
            "pq_file_num_pages": ([vp], C.c_int64),
            "pq_file_page_index": ([vp, C.POINTER(C.c_int64), C.c_int64], C.c_int),
        }
        for name, (args, res) in sig.items():
            f = getattr(L, name)
            f.argtypes = args
            f.restype = res
        _lib = L
    return _lib


def exported_symbols() -> list[str]:
    """Names the header declares (checked against the .so by the CPU tests)."""
    lib()
    return [n for n in dir(_lib) if n.startswith("pq_")]


def _buf(b: bytes):
    return C.cast(C.c_char_p(b), u8p)


# ── host page walk ─────────────────────────────────────────────────────────
def build_page_table(file: bytes, chunk: ChunkDesc, cap: int = 0):
    """(status, message, pages): the walk's pages as a ctypes PageDesc array
    (indexable, iterable; pass it back to Context.upload_range as is)."""
    if cap <= 0:  # a page is >= ~16 bytes of header + payload
        cap = max(64, min(len(file) // 16 + 64, 1 << 20))
    while True:
        pages = (PageDesc * cap)()
        n = C.c_int64()
        err = C.create_string_buffer(512)
        rc = lib().pq_build_page_table(_buf(file), len(file), C.byref(chunk), pages, cap, C.byref(n),
                                       err, 512)
        if n.value <= cap:
            break
        cap = n.value
    exact = (PageDesc * n.value)()
    C.memmove(exact, pages, C.sizeof(PageDesc) * n.value)
    return rc, err.value.decode(errors="replace"), exact


def plan_page_ranges(table, world: int) -> list[tuple[int, int]]:
    """pq_plan_page_ranges: byte-balanced contiguous data-page ranges of a
    chunk's page table (build_page_table) for `world` shards."""
    arr = table if isinstance(table, C.Array) else (PageDesc * max(len(table), 1))(*table)
    out = (C.c_int64 * (2 * world))()
    rc = lib().pq_plan_page_ranges(arr, len(table), world, out)
    if rc:
        raise PqError(rc, "pq_plan_page_ranges failed")
    return [(int(out[2 * k]), int(out[2 * k + 1])) for k in range(world)]


# ── file metadata (ParquetReader::open) ────────────────────────────────────
class File:
    def __init__(self, data: bytes):
        self.data = data
        h = vp()
        err = C.create_string_buffer(512)
        rc = lib().pq_file_open(_buf(data), len(data), C.byref(h), err, 512)
        if rc != 0:
            raise PqError(rc, err.value.decode(errors="replace"))
        self.h = h

    def __del__(self):
        if getattr(self, "h", None):
            lib().pq_file_close(self.h)
            self.h = None

    @property
    def num_rows(self) -> int:
        return lib().pq_file_num_rows(self.h)

    @property
    def num_row_groups(self) -> int:
        return lib().pq_file_num_row_groups(self.h)

    @property
    def num_columns(self) -> int:
        return lib().pq_file_num_columns(self.h)

    def column_names(self) -> list[str]:
        out = []
        b = C.create_string_buffer(1024)
        for i in range(self.num_columns):
            lib().pq_file_column_name(self.h, i, b, 1024)
            out.append(b.value.decode())
        return out

    def find_column(self, name: str) -> int:
        return lib().pq_file_find_column(self.h, name.encode())

    def chunk(self, rg: int, col: int) -> ChunkDesc:
        d = ChunkDesc()
        rc = lib().pq_file_chunk(self.h, rg, col, C.byref(d))
        if rc != 0:
            raise PqError(rc, "ColumnChunk has no metadata" if rc == -3 else "bad chunk index")
        return d

    def row_group_rows(self, rg: int) -> int:
        return lib().pq_file_row_group_rows(self.h, rg)

    def page_index(self) -> np.ndarray:
        n = lib().pq_file_num_pages(self.h)
        out = np.zeros(4 * max(n, 1), dtype=np.int64)
        lib().pq_file_page_index(self.h, out.ctypes.data_as(C.POINTER(C.c_int64)), n)
        return out[:4 * n].reshape(-1, 4)


# ── device context / chunks / columns ──────────────────────────────────────
@dataclass
class HostColumn:
    type: int
    validity: np.ndarray  # uint8 0/1 per row
    data: np.ndarray      # uint8: fixed-width values (n*width) or chars
    offsets: np.ndarray | None  # int64 n+1 (BYTE_ARRAY)

    @property
    def num_rows(self) -> int:
        return len(self.validity)


class DeviceBuffer:
    def __init__(self, ctx: "Context", h, n: int):
        self.ctx, self.h, self.n = ctx, h, n

    def data_ptr(self) -> int:
        return self.h.value or 0

    def free(self):
        if self.h and self.ctx.h:
            lib().pq_device_buffer_free(self.ctx.h, self.h)
        self.h = None

    def __del__(self):
        self.free()


class Context:
    def __init__(self, device: int = 0):
        self.h = lib().pq_ctx_create(device)
        if not self.h:
            raise PqError(-21, f"pq_ctx_create({device}) failed: no HIP device")

    def close(self):
        if self.h:
            lib().pq_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def set_option(self, key: str, value: int):
        self.check(lib().pq_ctx_set_option(self.h, key.encode(), int(value)))

    def error(self) -> str:
        return lib().pq_last_error(self.h).decode(errors="replace")

    def check(self, rc: int):
        if rc != 0:
            raise PqError(rc, self.error())

    def upload(self, file: bytes, chunks) -> "DeviceChunk":
        if isinstance(chunks, ChunkDesc):
            chunks = [chunks]
        arr = (ChunkDesc * len(chunks))(*chunks)
        h = vp()
        self.check(lib().pq_chunk_upload(self.h, _buf(file), len(file), arr, len(chunks), C.byref(h)))
        return DeviceChunk(self, h)

    def device_buffer(self, data: bytes) -> "DeviceBuffer":
        """A device copy of `data` (pq_device_buffer), freed with the object."""
        h = vp()
        self.check(lib().pq_device_buffer(self.h, _buf(data), len(data), C.byref(h)))
        return DeviceBuffer(self, h, len(data))

    def build_page_table_device(self, d_ptr: int, length: int, base: int, chunk: ChunkDesc, seg_bytes: int = 0,
                                rec_cap: int = 0, cap: int = 0):
        """pq_build_page_table_device over file bytes [base, base + length)
        already in device memory at d_ptr: (status, pages) with pages a
        PageDesc array (status PQ_ERR_UNSUPPORTED = -8: walk on the host)."""
        if cap <= 0:
            cap = max(64, min(length // 16 + 64, 1 << 22))
        pages = (PageDesc * cap)()
        n = C.c_int64()
        rc = lib().pq_build_page_table_device(self.h, C.c_void_p(d_ptr), length, base, C.byref(chunk), seg_bytes,
                                              rec_cap, pages, cap, C.byref(n))
        if rc == 0 and n.value > cap:
            raise PqError(-20, "page table over its capacity")
        exact = (PageDesc * n.value)()
        C.memmove(exact, pages, C.sizeof(PageDesc) * n.value)
        return rc, exact

    def upload_range(self, file: bytes, chunk: ChunkDesc, table, data_begin: int, data_end: int) -> "DeviceChunk":
        """Data pages [data_begin, data_end) of one chunk (+ their dictionary
        pages) from its page table (build_page_table): a page-range shard."""
        arr = table if isinstance(table, C.Array) else (PageDesc * max(len(table), 1))(*table)
        h = vp()
        self.check(lib().pq_chunk_upload_range(self.h, _buf(file), len(file), C.byref(chunk), arr, len(table),
                                               data_begin, data_end, C.byref(h)))
        return DeviceChunk(self, h)

    def timing(self, on: bool = True):
        lib().pq_timing_enable(self.h, int(on))

    def timing_reset(self):
        lib().pq_timing_reset(self.h)

    def timing_get(self, name: str):
        ms = C.c_double()
        n = C.c_int64()
        ok = lib().pq_timing_get(self.h, name.encode(), C.byref(ms), C.byref(n))
        return (ms.value, n.value) if ok else (0.0, 0)

    def sync(self):
        self.check(lib().pq_ctx_sync(self.h))

    PROF_PHASES = ("stage", "def", "levels", "values", "rows", "lookback", "slotwait", "pages",
                   "w_wait", "w_offsets", "w_gather", "w_pages", "hyb_A", "hyb_B", "hyb_C", "hyb_D")

    def fused_prof_read(self, raw: bool = False):
        """Per-phase shader-clock sums of k_ba_fused / k_ba_batch since the
        last read (option "fused_prof" must be 1)."""
        buf = (C.c_uint64 * 16)()
        k = lib().pq_fused_prof_read(self.h, buf, 16)
        if raw:
            return [int(buf[i]) for i in range(k)]
        return {self.PROF_PHASES[i] if i < len(self.PROF_PHASES) else str(i): int(buf[i]) for i in range(k)}


class DeviceChunk:
    def __init__(self, ctx: Context, h):
        self.ctx = ctx
        self.h = h
        self.out = ColumnOut()

    def free(self):
        if self.h:
            lib().pq_column_free(self.ctx.h, C.byref(self.out))
            lib().pq_chunk_free(self.ctx.h, self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass

    @property
    def num_rows(self) -> int:
        return lib().pq_chunk_num_rows(self.h)

    @property
    def num_pages(self) -> int:
        return lib().pq_chunk_num_pages(self.h)

    @property
    def first_row(self) -> int:
        return lib().pq_chunk_first_row(self.h)

    @property
    def payload_bytes(self) -> int:
        return lib().pq_chunk_payload_bytes(self.h)

    def pages(self):
        n = C.c_int64()
        lib().pq_chunk_pages(self.h, None, 0, C.byref(n))
        arr = (PageDesc * max(n.value, 1))()
        lib().pq_chunk_pages(self.h, arr, n.value, C.byref(n))
        return [arr[i] for i in range(n.value)]

    def decode(self):
        self.ctx.check(lib().pq_decode(self.ctx.h, self.h, C.byref(self.out)))
        return self.out

    def decode_async(self):
        self.ctx.check(lib().pq_decode_async(self.ctx.h, self.h, C.byref(self.out)))

    def decode_check(self):
        self.ctx.check(lib().pq_decode_check(self.ctx.h, self.h))

    def to_host(self) -> HostColumn:
        o = self.out
        n = o.num_rows
        words = np.zeros((n + 31) // 32 + 1, dtype=np.uint32)
        data = np.zeros(max(o.num_bytes, 1), dtype=np.uint8)
        offs = np.zeros(n + 1, dtype=np.int64) if o.type == BYTE_ARRAY else None
        self.ctx.check(lib().pq_column_copy_out(
            self.ctx.h, C.byref(o), words.ctypes.data_as(vp), data.ctypes.data_as(vp),
            offs.ctypes.data_as(vp) if offs is not None else None))
        valid = np.unpackbits(words.view(np.uint8), bitorder="little")[:n].astype(np.uint8)
        return HostColumn(o.type, valid, data[:o.num_bytes], offs)

    def chunk_assign(self, chunk_bytes: int = 4096):
        """(tuple_to_chunk int64[num_rows], num_chunks) of the decoded column
        (the example driver's 4 KiB chunker, src/main.cpp:17-32)."""
        n = self.out.num_rows
        out = np.zeros(max(n, 1), dtype=np.int64)
        k = C.c_int64()
        self.ctx.check(lib().pq_chunk_assign(self.ctx.h, C.byref(self.out), chunk_bytes, None,
                                             out.ctypes.data_as(vp), C.byref(k)))
        return out[:n], k.value

    def regex_pages(self, pattern: str, neg: bool = False) -> np.ndarray:
        flags = np.zeros(max(self.num_pages, 1), dtype=np.uint8)
        self.ctx.check(lib().pq_regex_pages(self.ctx.h, self.h, pattern.encode(), int(neg),
                                            flags.ctypes.data_as(vp)))
        return flags[:self.num_pages]

    def regex_pages_async(self, pattern: str, neg: bool = False):
        self.ctx.check(lib().pq_regex_pages_async(self.ctx.h, self.h, pattern.encode(), int(neg)))

    def decode_regex_async(self, pattern: str, neg: bool = False):
        """pq_decode_regex_async: decode + page filter in one pass (flags via
        regex_pages_result, the column via decode_check / to_host)."""
        self.ctx.check(lib().pq_decode_regex_async(self.ctx.h, self.h, C.byref(self.out), pattern.encode(),
                                                   int(neg)))

    def regex_pages_result(self) -> np.ndarray:
        flags = np.zeros(max(self.num_pages, 1), dtype=np.uint8)
        self.ctx.check(lib().pq_regex_pages_result(self.ctx.h, self.h, flags.ctypes.data_as(vp)))
        return flags[:self.num_pages]


def regex_check(pattern: str):
    err = C.create_string_buffer(256)
    rc = lib().pq_regex_compile_check(pattern.encode(), err, 256)
    return rc, err.value.decode(errors="replace")


def regex_match_host(pattern: str, s: bytes) -> int:
    return lib().pq_regex_match_host(pattern.encode(), _buf(s), len(s))


def regex_dfa_sinks(pattern: str):
    """(rc, absorbing-state mask) of the pattern's DFA."""
    lo, hi = C.c_uint32(0), C.c_uint32(0)
    rc = lib().pq_regex_dfa_sinks(pattern.encode(), C.byref(lo), C.byref(hi))
    return rc, (hi.value << 32) | lo.value


def regex_match_host_dfa(pattern: str, s: bytes) -> int:
    """The GPU kernel's DFA run on the host (-8: DFA over its size cap)."""
    return lib().pq_regex_match_host_dfa(pattern.encode(), _buf(s), len(s))


def canonical_dump(col: HostColumn) -> bytes:
    """Canonical dump: u8 is_null + payload; INT96 rendered as the
    reference's "INT96(hi:lo)" string (column_reader.cpp:257-264)."""
    n = col.num_rows
    t = col.type
    if t == BYTE_ARRAY:
        offsets = col.offsets
        data = col.data
        var = True
    elif t == INT96:
        raw = col.data.reshape(-1, 12) if n else np.zeros((0, 12), np.uint8)
        strs = []
        for i in range(n):
            if col.validity[i]:
                lo = int(np.frombuffer(raw[i, :8].tobytes(), "<i8")[0])
                hi = int(np.frombuffer(raw[i, 8:].tobytes(), "<i4")[0])
                strs.append(f"INT96({hi}:{lo})".encode())
            else:
                strs.append(b"")
        lens = np.array([len(s) for s in strs], dtype=np.int64)
        offsets = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        data = np.frombuffer(b"".join(strs), dtype=np.uint8)
        var = True
    else:
        w = WIDTH[t]
        offsets = np.arange(n + 1, dtype=np.int64) * w
        data = col.data
        var = False
    valid = col.validity
    lens = np.where(valid != 0, np.diff(offsets), 0).astype(np.int64)
    rec = 1 + lens + (4 * (valid != 0) if var else 0)
    out = np.zeros(int(rec.sum()), dtype=np.uint8)
    starts = np.concatenate([[0], np.cumsum(rec)[:-1]]).astype(np.int64) if n else np.zeros(0, np.int64)
    out[starts] = (valid == 0).astype(np.uint8)
    nz = np.nonzero(valid)[0]
    if len(nz):
        pay = starts[nz] + 1
        if var:
            l32 = lens[nz].astype("<u4").view(np.uint8).reshape(-1, 4)
            for k in range(4):
                out[pay + k] = l32[:, k]
            pay = pay + 4
        L = lens[nz]
        tot = int(L.sum())
        if tot:
            cs = np.concatenate([[0], np.cumsum(L)[:-1]])
            ar = np.arange(tot, dtype=np.int64)
            out[np.repeat(pay - cs, L) + ar] = np.asarray(data, np.uint8)[np.repeat(offsets[nz] - cs, L) + ar]
    return out.tobytes()
