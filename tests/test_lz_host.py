"""CPU: the codec pass's SNAPPY and LZ4 command-stream parsers
(csrc/kernels/lz.hpp) built for the host (tools/lz_check.cpp, with k_codec's
queue checks and an exact-size output) and pinned against pyarrow's snappy and
lz4_raw: literals of every length encoding, copies with 1-, 2- and 4-byte
offsets, overlapping copies, LZ4's 255-byte length extensions, Hadoop-framed
LZ4 (several blocks), V2-style pages that end exactly on the last sequence;
and damaged payloads, which must end in a status.  The GPU runs the same
source (tests/test_gpu_ext.py decodes pyarrow SNAPPY / LZ4 pages).  Codecs are
outside the reference's parity scope (column_reader.cpp:13-15)."""
import ctypes as C
import os
import random
import struct
import subprocess

import numpy as np
import pytest

pa = pytest.importorskip("pyarrow")

PKG = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "duckdb-parquet-parser_amd")
LIB = os.path.join(PKG, "pqgpu", "liblz_check.so")
SNAPPY, LZ4, LZ4_RAW = 1, 5, 7
OK, CORRUPT, SIZE = 0, 1, 2


@pytest.fixture(scope="module")
def lz():
    subprocess.run(["make", "-C", PKG, "pqgpu/liblz_check.so"], check=True, stdout=subprocess.DEVNULL)
    return C.CDLL(LIB)


def dec(lz, codec, b: bytes, n: int, ring=65536):
    out = (C.c_uint8 * (n + 16))()
    ol = C.c_uint32(0)
    rc = lz.lz_decompress(codec, b, len(b), out, n, ring, C.byref(ol))
    return rc, bytes(out[:ol.value])


def inputs():
    rng = random.Random(1)
    g = np.random.default_rng(7)
    words = [b"carefully ", b"quickly ", b"special ", b"requests ", b"the ", b"final ", b"deposits "]
    yield b"a"
    yield b"hello hello hello hello world" * 100
    yield bytes(range(256)) * 50
    yield bytes(rng.randrange(256) for _ in range(5000))  # literals of every length class
    yield b"".join(rng.choice(words) for _ in range(40000))
    yield g.integers(0, 1000, 200000).astype(np.int64).tobytes()
    yield b"ab" * 70000  # overlapping copies, long lengths
    yield b"\0" * 300000
    blk = g.integers(0, 256, 40_000).astype(np.uint8).tobytes()
    yield blk + g.integers(0, 256, 20_000).astype(np.uint8).tobytes() + blk  # a copy 60 KB back (2-byte offsets)
    yield np.sort(g.integers(0, 10**9, 300000)).astype(np.int64).tobytes()


def hadoop(raw: bytes, block=65536) -> bytes:
    """Hadoop's LZ4 framing: [u32 BE raw][u32 BE packed][LZ4 block] per block."""
    c = pa.Codec("lz4_raw")
    out = b""
    for i in range(0, max(len(raw), 1), block):
        part = raw[i:i + block]
        z = c.compress(part, asbytes=True)
        out += struct.pack(">II", len(part), len(z)) + z
    return out


@pytest.mark.parametrize("codec", [SNAPPY, LZ4_RAW, LZ4])
def test_lz_vs_pyarrow(lz, codec):
    for i, d in enumerate(inputs()):
        if codec == SNAPPY:
            z = pa.Codec("snappy").compress(d, asbytes=True)
        elif codec == LZ4_RAW:
            z = pa.Codec("lz4_raw").compress(d, asbytes=True)
        else:
            z = hadoop(d)
        rc, got = dec(lz, codec, z, len(d))
        assert rc == OK and got == d, (codec, i, rc, len(got), len(d))


def test_snappy_four_byte_offsets_and_literal_lengths(lz):
    """Hand-made SNAPPY streams for the tags compressors rarely emit: a
    literal with a 1..4-byte length and a copy with a 4-byte offset."""
    lit = bytes(range(200))
    for nb in (1, 2, 3, 4):  # literal tag 60 + nb: length - 1 in nb bytes
        z = bytes([len(lit)]) + bytes([(59 + nb) << 2]) + (len(lit) - 1).to_bytes(nb, "little") + lit
        assert dec(lz, SNAPPY, bytes([0xC8, 0x01]) + z[1:], 200) == (OK, lit)
    # 8 literal bytes, then a 4-byte-offset copy of 8 bytes from 8 back
    body = bytes([(8 - 1) << 2]) + b"abcdefgh" + bytes([((8 - 1) << 2) | 3]) + (8).to_bytes(4, "little")
    assert dec(lz, SNAPPY, bytes([16]) + body, 16) == (OK, b"abcdefgh" * 2)


def test_lz_damaged(lz):
    """Statuses of damaged payloads: a copy before the first byte, a copy
    farther back than the ring, an output longer than the page, a cut
    stream, a wrong declared length."""
    # copy of 4 from distance 1 with no history
    assert dec(lz, SNAPPY, bytes([4, (0 << 2) | 1, 1]), 4)[0] == CORRUPT
    assert dec(lz, LZ4_RAW, bytes([0x00, 1, 0]), 4)[0] == CORRUPT
    # a distance past the 8 KiB small-page ring
    r = np.random.default_rng(3).integers(0, 256, 10000).astype(np.uint8).tobytes()
    z = pa.Codec("lz4_raw").compress(r + r[:4000], asbytes=True)  # one copy from 10,000 back
    assert dec(lz, LZ4_RAW, z, len(r) + 4000, ring=65536) == (OK, r + r[:4000])
    assert dec(lz, LZ4_RAW, z, len(r) + 4000, ring=8192)[0] == CORRUPT
    d = bytes(range(256)) * 40
    # the output is one byte short of the stream
    z = pa.Codec("lz4_raw").compress(d, asbytes=True)
    assert dec(lz, LZ4_RAW, z, len(d) - 1)[0] == SIZE
    assert dec(lz, LZ4_RAW, z, len(d) + 1)[0] == SIZE  # does not fill the page
    # snappy's declared length disagrees with the page
    z = pa.Codec("snappy").compress(d, asbytes=True)
    assert dec(lz, SNAPPY, z, len(d) + 1)[0] == SIZE
    # cut streams
    for cut in (1, 2, len(z) // 2, len(z) - 1):
        assert dec(lz, SNAPPY, z[:cut], len(d))[0] != OK
    zh = hadoop(d, 4096)
    for cut in (3, 8, 9, len(zh) // 2):
        assert dec(lz, LZ4, zh[:cut], len(d))[0] != OK
    # a Hadoop block whose raw size disagrees with its content
    bad = bytearray(zh)
    bad[3] ^= 1
    assert dec(lz, LZ4, bytes(bad), len(d))[0] == SIZE
    # an empty LZ4_RAW block is corrupt (a block holds at least its token)
    assert dec(lz, LZ4_RAW, b"", 0)[0] == CORRUPT


def test_lz_random_mutants_end_in_status(lz):
    """Thousands of mutants (flipped bytes, cut tails) decode to a status and
    never more bytes than the page holds (the ASan/UBSan build of the same
    harness runs in test_fuzz_host.py)."""
    rng = random.Random(5)
    base = b"".join(rng.choice([b"alpha ", b"beta ", b"gamma ", b"delta "]) for _ in range(3000))
    streams = [(SNAPPY, pa.Codec("snappy").compress(base, asbytes=True)),
               (LZ4_RAW, pa.Codec("lz4_raw").compress(base, asbytes=True)),
               (LZ4, hadoop(base, 8192))]
    for codec, z in streams:
        for _ in range(400):
            m = bytearray(z)
            if rng.random() < 0.2:
                m = m[:rng.randrange(1, len(m))]
            else:
                for _ in range(rng.randint(1, 4)):
                    m[rng.randrange(len(m))] = rng.randrange(256)
            rc, got = dec(lz, codec, bytes(m), len(base))
            assert rc in (OK, CORRUPT, SIZE) and len(got) <= len(base)
