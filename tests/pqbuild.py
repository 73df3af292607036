"""Hand-built Parquet pages for edge-case tests (test helper, pure Python).

Lets a test write exactly the bytes a malformed or unusual page holds:
zero-count runs, bit width 0, truncated payloads, pages past EOF, unknown
page types.  The footer is minimal but readable by the reference reader.
"""
from __future__ import annotations

import struct


def varint(v: int) -> bytes:
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def zigzag(v: int) -> bytes:
    return varint((v << 1) ^ (v >> 63) if v < 0 else v << 1)


class TW:
    """Thrift compact writer."""

    def __init__(self):
        self.b = bytearray()
        self.last = 0
        self.stack = []

    def field(self, fid: int, t: int):
        d = fid - self.last
        if 0 < d <= 15:
            self.b.append((d << 4) | t)
        else:
            self.b.append(t)
            self.b += zigzag(fid)
        self.last = fid

    def i32(self, fid, v):
        self.field(fid, 5)
        self.b += zigzag(v)
        return self

    def i64(self, fid, v):
        self.field(fid, 6)
        self.b += zigzag(v)
        return self

    def string(self, fid, s: bytes):
        self.field(fid, 8)
        self.b += varint(len(s)) + s
        return self

    def begin(self, fid):
        self.field(fid, 12)
        self.stack.append(self.last)
        self.last = 0
        return self

    def end(self):
        self.b.append(0)
        self.last = self.stack.pop()
        return self

    def list_begin(self, fid, et, n):
        self.field(fid, 9)
        self.b.append((n << 4) | et if n < 15 else 0xF0 | et)
        if n >= 15:
            self.b += varint(n)
        return self

    def push(self):
        self.stack.append(self.last)
        self.last = 0

    def pop(self):
        self.last = self.stack.pop()

    def stop(self):
        self.b.append(0)
        return self


def data_header(size: int, nvals: int, enc: int = 0, ptype: int = 0, with_dph: bool = True,
                usize: int | None = None) -> bytes:
    """usize: uncompressed_page_size when it differs (compressed pages)."""
    t = TW().i32(1, ptype).i32(2, size if usize is None else usize).i32(3, size)
    if with_dph:
        t.begin(5).i32(1, nvals).i32(2, enc).i32(3, 3).i32(4, 3).end()
    return bytes(t.stop().b)


def dict_header(size: int, nvals: int) -> bytes:
    return bytes(TW().i32(1, 2).i32(2, size).i32(3, size).begin(7).i32(1, nvals).i32(2, 2).end().stop().b)


def rle(count: int, value: int, bw: int) -> bytes:
    return varint(count << 1) + value.to_bytes((bw + 7) // 8, "little")


def bitpack(values, bw: int, groups: int | None = None) -> bytes:
    g = groups if groups is not None else (len(values) + 7) // 8
    vals = list(values) + [0] * (8 * g - len(values))
    bits = 0
    for i, v in enumerate(vals):
        bits |= (v & ((1 << bw) - 1)) << (i * bw)
    nbytes = (len(vals) * bw + 7) // 8
    return varint((g << 1) | 1) + bits.to_bytes(nbytes, "little")


def levels_section(stream: bytes) -> bytes:
    return struct.pack("<I", len(stream)) + stream


def plain_ba(values) -> bytes:
    return b"".join(struct.pack("<I", len(v)) + v for v in values)


def build_file(pages: list[bytes], ptype: int, optional: bool, num_values: int,
               dict_at_start: bool = False, name: bytes = b"c", pad_footer: bool = True, codec: int = 0,
               nested: str | None = None):
    """pages: list of (header + payload) blobs laid out back to back.
    nested: None (one flat leaf: max_def = optional, max_rep 0), "repeated"
    (a REPEATED leaf: max_def 1, max_rep 1) or "list" (the LIST shape
    optional group a / repeated group list / leaf element: max_def 2 +
    optional, max_rep 1), levels as ParquetReader::build_columns_recursive
    counts them (parquet_reader.cpp:495-543).
    Returns (file bytes, chunk dict for the oracle/C ABI)."""
    body = b"PAR1"
    start = len(body)
    for p in pages:
        body += p
    end = len(body)
    t = TW()
    t.i32(1, 1)
    if nested == "list":
        t.list_begin(2, 12, 4)
        t.push(); t.string(4, b"schema"); t.i32(5, 1); t.stop(); t.pop()
        t.push(); t.i32(3, 1); t.string(4, b"a"); t.i32(5, 1); t.i32(6, 3); t.stop(); t.pop()
        t.push(); t.i32(3, 2); t.string(4, b"list"); t.i32(5, 1); t.stop(); t.pop()
        t.push(); t.i32(1, ptype); t.i32(3, 1 if optional else 0); t.string(4, name); t.stop(); t.pop()
        path = [b"a", b"list", name]
        max_def, max_rep = 2 + (1 if optional else 0), 1
    else:
        t.list_begin(2, 12, 2)
        t.push(); t.string(4, b"schema"); t.i32(5, 1); t.stop(); t.pop()
        rep = 2 if nested == "repeated" else (1 if optional else 0)
        t.push(); t.i32(1, ptype); t.i32(3, rep); t.string(4, name); t.stop(); t.pop()
        path = [name]
        max_def, max_rep = (1, 1) if nested == "repeated" else (1 if optional else 0, 0)
    t.i64(3, num_values)
    t.list_begin(4, 12, 1)
    t.push()
    t.list_begin(1, 12, 1)
    t.push()
    t.i64(2, start)
    t.begin(3)
    t.i32(1, ptype)
    t.list_begin(2, 5, 1)
    t.b += zigzag(0)
    t.list_begin(3, 8, len(path))
    for seg in path:
        t.b += varint(len(seg)) + seg
    t.i32(4, codec)
    t.i64(5, num_values)
    t.i64(6, end - start)
    t.i64(7, end - start)
    t.i64(9, start)
    if dict_at_start:
        t.i64(11, start)
    t.end()
    t.stop()
    t.pop()
    t.i64(2, end - start)
    t.i64(3, num_values)
    t.stop()
    t.pop()
    if pad_footer:
        t.string(6, b"pqbuild " + b"." * 300)
    t.stop()
    footer = bytes(t.b)
    data = body + footer + struct.pack("<I", len(footer)) + b"PAR1"
    chunk = dict(num_values=num_values, data_page_offset=start,
                 dictionary_page_offset=start if dict_at_start else None, codec=codec, type=ptype,
                 max_def=max_def, max_rep=max_rep)
    return data, chunk
