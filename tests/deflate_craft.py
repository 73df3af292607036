"""A hand-built DEFLATE dynamic-Huffman block (RFC 1951 3.2.7) whose
code-length sequence uses code 16 right after a 17/18 zero run, the shape
zlib itself rarely emits (zopfli does).  Code 16 repeats the last length
written, which is 0 after a zero run.  Test input only; Python's zlib is the
check that the stream is valid."""
from __future__ import annotations

import struct
import zlib


class BitWriter:
    def __init__(self):
        self.bits = 0
        self.n = 0
        self.out = bytearray()

    def put(self, v: int, nb: int):  # LSB-first fields
        self.bits |= (v & ((1 << nb) - 1)) << self.n
        self.n += nb
        while self.n >= 8:
            self.out.append(self.bits & 0xFF)
            self.bits >>= 8
            self.n -= 8

    def put_code(self, code: int, length: int):  # Huffman codes: MSB first
        rev = int(format(code, f"0{length}b")[::-1], 2) if length else 0
        self.put(rev, length)

    def done(self) -> bytes:
        if self.n:
            self.out.append(self.bits & 0xFF)
        return bytes(self.out)


def canonical(lengths: list[int]) -> list[int]:
    """Canonical Huffman codes for the lengths (RFC 1951 3.2.2)."""
    mx = max(lengths)
    bl = [0] * (mx + 1)
    for l in lengths:
        if l:
            bl[l] += 1
    code, nxt = 0, [0] * (mx + 2)
    for b in range(1, mx + 1):
        code = (code + bl[b - 1]) << 1
        nxt[b] = code
    out = [0] * len(lengths)
    for i, l in enumerate(lengths):
        if l:
            out[i] = nxt[l]
            nxt[l] += 1
    return out


CL_ORDER = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]


def deflate_16_after_zero_run(data: bytes) -> bytes:
    """One final dynamic block coding `data` as literals.  Every byte value of
    the data gets a literal length of 4 or 5 (a complete code with EOB); the
    runs of unused symbols between them are coded 18/17 followed by 16."""
    used = sorted(set(data))
    assert 2 <= len(used) <= 15
    syms = used + [256]
    k = len(syms)
    # complete prefix code over k symbols: lengths L and L + 1
    L = k.bit_length() - 1   # 2^L <= k < 2^(L+1)
    n_short = (2 << L) - k   # symbols at length L, the rest at L + 1: Kraft sum 1
    lit = [0] * 257
    for i, sym in enumerate(syms):
        lit[sym] = L if i < n_short else L + 1
    dist = [1]  # one distance code, never used
    seq = lit + dist
    # code-length symbols: zero runs as 18 or 17, then 16 (repeat the last
    # length written = 0) for up to 6 more; other lengths literally
    cl_syms = []  # (symbol, extra value, extra bits)
    i = 0
    while i < len(seq):
        if seq[i] != 0:
            cl_syms.append((seq[i], 0, 0))
            i += 1
            continue
        j = i
        while j < len(seq) and seq[j] == 0:
            j += 1
        run = j - i
        if run >= 14:
            first = min(run - 3, 138)  # leave >= 3 for a 16 after the 18
            cl_syms.append((18, first - 11, 7))
            rest = run - first
        elif run >= 6:
            first = min(run - 3, 10)
            cl_syms.append((17, first - 3, 3))
            rest = run - first
        else:
            cl_syms.extend([(0, 0, 0)] * run)
            rest = 0
        while rest >= 3:
            r = min(rest, 6)
            if rest - r in (1, 2):
                r = rest - 3 if rest - 3 >= 3 else rest
            cl_syms.append((16, r - 3, 2))
            rest -= r
        cl_syms.extend([(0, 0, 0)] * rest)
        i = j
    assert any(a[0] == 16 for a in cl_syms)
    # code-length code: complete code over the symbols used
    used_cl = sorted({a[0] for a in cl_syms})
    m = len(used_cl)
    Lc = m.bit_length() - 1
    ns = (2 << Lc) - m
    cl_len = [0] * 19
    for t, sym in enumerate(used_cl):
        cl_len[sym] = Lc if t < ns else Lc + 1
    if m == 1:
        cl_len[used_cl[0]] = 1
    cl_code = canonical(cl_len)
    hclen = 19
    while hclen > 4 and cl_len[CL_ORDER[hclen - 1]] == 0:
        hclen -= 1
    w = BitWriter()
    w.put(1, 1)  # BFINAL
    w.put(2, 2)  # dynamic
    w.put(257 - 257, 5)
    w.put(1 - 1, 5)
    w.put(hclen - 4, 4)
    for t in range(hclen):
        w.put(cl_len[CL_ORDER[t]], 3)
    for sym, ev, eb in cl_syms:
        w.put_code(cl_code[sym], cl_len[sym])
        if eb:
            w.put(ev, eb)
    lit_code = canonical(lit)
    for b in data:
        w.put_code(lit_code[b], lit[b])
    w.put_code(lit_code[256], lit[256])
    raw = w.done()
    assert zlib.decompress(raw, -15) == data
    return raw


def gzip_member(raw_deflate: bytes, data: bytes, crc: int | None = None) -> bytes:
    c = zlib.crc32(data) if crc is None else crc
    return b"\x1f\x8b\x08\x00\x00\x00\x00\x00\x00\xff" + raw_deflate + struct.pack("<II", c & 0xFFFFFFFF, len(data))
