"""CPU: known-answer tests for the hybrid RLE/bit-packed decoder (R-RLE).

Expected values come from an independent pure-Python model of the Parquet
hybrid encoding for well-formed streams, plus hand-derived answers for the
reference's quirks (include/reader/rle_decoder.hpp:17-95): zero-fill after
exhaustion, int32 truncation, zero-count runs wrapping the literal counter.
"""
import random

import pytest

import pqbuild as B
from oracle import oracle as O


def model_decode(stream: bytes, bw: int, count: int):
    """Spec model for well-formed streams (no zero-count runs)."""
    out, pos = [], 0
    while len(out) < count and pos < len(stream):
        ind, shift = 0, 0
        while pos < len(stream):
            b = stream[pos]
            pos += 1
            ind |= (b & 0x7F) << shift
            if not b & 0x80:
                break
            shift += 7
        if ind & 1:
            n = (ind >> 1) * 8
            nbytes = n * bw // 8
            bits = int.from_bytes(stream[pos:pos + nbytes], "little")
            for i in range(n):
                out.append((bits >> (i * bw)) & ((1 << bw) - 1))
            pos += nbytes
        else:
            n = ind >> 1
            nb = (bw + 7) // 8
            v = int.from_bytes(stream[pos:pos + nb], "little")
            pos += nb
            out += [v] * n
    out = out[:count] + [0] * max(0, count - len(out))
    return [((v & 0xFFFFFFFF) ^ 0x80000000) - 0x80000000 for v in out]


def check(stream, bw, count, expected=None):
    rc, got = O.rle_decode(stream, bw, count)
    assert rc == 0
    assert got == (expected if expected is not None else model_decode(stream, bw, count))


@pytest.mark.parametrize("bw", list(range(0, 33)))
def test_single_group_and_rle_runs(bw):
    rng = random.Random(bw)
    vals = [rng.getrandbits(bw) if bw else 0 for _ in range(8)]
    stream = B.rle(5, vals[0], bw) + B.bitpack(vals, bw) + B.rle(3, vals[-1], bw)
    check(stream, bw, 16)


@pytest.mark.parametrize("bw", [1, 3, 10, 17, 32])
def test_63_group_bitpacked_run(bw):
    rng = random.Random(100 + bw)
    vals = [rng.getrandbits(bw) for _ in range(63 * 8)]
    check(B.bitpack(vals, bw), bw, len(vals))


def test_padded_final_group_and_partial_read():
    vals = [1, 2, 3]
    stream = B.bitpack(vals, 2)  # one group, 5 zero pads
    check(stream, 2, 3, [1, 2, 3])
    check(stream, 2, 8, [1, 2, 3, 0, 0, 0, 0, 0])


def test_multibyte_varint_headers():
    stream = B.rle(1000, 7, 3) + B.rle(20000, 1, 3)
    check(stream, 3, 21000)


def test_exhaustion_zero_fills():
    check(B.rle(3, 9, 4), 4, 10, [9, 9, 9] + [0] * 7)
    check(b"", 4, 5, [0] * 5)


def test_int32_truncation():
    # bw 32 value with the top bit set becomes negative (static_cast<int32_t>)
    check(B.rle(2, 0xFFFFFFFE, 32), 32, 2, [-2, -2])
    # bw 40: the low 32 bits are kept
    check(B.bitpack([(1 << 39) | 5, 3], 40), 40, 2, [5, 3])


def test_zero_group_literal_run_wraps():
    # header 0x01 = bit-packed with 0 groups: literal_count_ wraps, the rest of
    # the batch is read as consecutive bw-bit fields right after the header
    stream = B.rle(2, 1, 2) + bytes([0x01, 0b11100100, 0x1B])
    check(stream, 2, 10, [1, 1, 0, 1, 2, 3, 3, 2, 1, 0])


def test_zero_count_rle_run_after_literal_reuses_cursor():
    # literal run [1,2,3,0,1,2,3,0] then an RLE header with count 0: later
    # values continue from the literal cursor (the next stream bytes)
    stream = B.bitpack([1, 2, 3, 0, 1, 2, 3, 0], 2) + B.rle(0, 3, 2) + bytes([0x1B])
    rc, got = O.rle_decode(stream, 2, 12)
    assert rc == 0
    # bytes after the 2-byte literal payload: 0x00 (rle header), 0x03 (value), 0x1B
    assert got == [1, 2, 3, 0, 1, 2, 3, 0, 0, 0, 0, 0]


def test_zero_count_without_literal_is_out_of_scope():
    rc, _ = O.rle_decode(B.rle(0, 1, 2) + B.rle(3, 1, 2), 2, 3)
    assert rc == -8  # PQO_ERR_UNSUPPORTED: the reference dereferences NULL


def test_random_wellformed_streams():
    rng = random.Random(7)
    for _ in range(200):
        bw = rng.randrange(1, 33)
        stream, total = b"", 0
        for _ in range(rng.randrange(1, 12)):
            if rng.random() < 0.5:
                n = rng.randrange(1, 300)
                stream += B.rle(n, rng.getrandbits(bw), bw)
                total += n
            else:
                g = rng.randrange(1, 64)
                stream += B.bitpack([rng.getrandbits(bw) for _ in range(8 * g)], bw)
                total += 8 * g
        check(stream, bw, total + rng.randrange(0, 20))
