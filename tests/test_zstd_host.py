"""CPU: the codec pass's ZSTD decoder (csrc/kernels/zstd.hpp, RFC 8878) built
for the host (tools/zstd_check.cpp) and pinned against
pyarrow's zstd: frames of several shapes (raw / RLE / compressed blocks,
Huffman 1- and 4-stream literals, FSE-compressed and direct Huffman weights,
predefined / RLE / FSE / repeat sequence tables, repeat offsets, matches
farther back than 64 KiB, multi-block frames) at compression levels -5..22,
and damaged frames that must end in a status, never a fault.  The GPU runs
the same source (tests/test_gpu_ext.py decodes pyarrow ZSTD pages).  Codecs
are outside the reference's parity scope (column_reader.cpp:13-15)."""
import ctypes as C
import os
import random
import subprocess

import numpy as np
import pytest

pa = pytest.importorskip("pyarrow")
if not pa.Codec.is_available("zstd"):
    pytest.skip("pyarrow without zstd", allow_module_level=True)

PKG = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "duckdb-parquet-parser_amd")
LIB = os.path.join(PKG, "pqgpu", "libzstd_check.so")


@pytest.fixture(scope="module")
def zs():
    subprocess.run(["make", "-C", PKG, "pqgpu/libzstd_check.so"], check=True, stdout=subprocess.DEVNULL)
    return C.CDLL(LIB)


def dec(zs, b: bytes, n: int):
    out = (C.c_uint8 * (n + 16))()
    ol = C.c_uint32(0)
    rc = zs.zs_decompress(b, len(b), out, n, C.byref(ol))
    return rc, bytes(out[:ol.value])


def inputs():
    rng = random.Random(1)
    g = np.random.default_rng(7)
    words = [b"carefully ", b"quickly ", b"special ", b"requests ", b"the ", b"final ", b"deposits "]
    yield b"a"
    yield b"hello hello hello hello world" * 100
    yield bytes(range(256)) * 50
    yield bytes(rng.randrange(256) for _ in range(5000))
    yield b"".join(rng.choice(words) for _ in range(40000))
    yield g.integers(0, 1000, 200000).astype(np.int64).tobytes()
    yield b"ab" * 70000
    yield g.integers(0, 50, 1_500_000).astype(np.uint8).tobytes()
    blk = g.integers(0, 256, 100_000).astype(np.uint8).tobytes()
    yield blk + g.integers(0, 256, 300_000).astype(np.uint8).tobytes() + blk  # a match 300 KiB back
    yield np.sort(g.integers(0, 10**9, 300000)).astype(np.int64).tobytes()


@pytest.mark.parametrize("level", [-5, 1, 3, 9, 19, 22])
def test_zstd_vs_pyarrow(zs, level):
    c = pa.Codec("zstd", compression_level=level)
    for i, d in enumerate(inputs()):
        rc, got = dec(zs, c.compress(d, asbytes=True), len(d))
        assert rc == 0 and got == d, (level, i, rc, len(got), len(d))


def test_zstd_concatenated_frames(zs):
    c = pa.Codec("zstd", compression_level=3)
    a, b = b"first frame " * 500, b"second " * 900
    rc, got = dec(zs, c.compress(a, asbytes=True) + c.compress(b, asbytes=True), len(a) + len(b))
    assert rc == 0 and got == a + b


def test_zstd_damaged_frames_end_in_a_status(zs):
    rng = random.Random(5)
    d = b"".join(rng.choice([b"alpha ", b"beta ", b"gamma%d " % rng.randrange(999)]) for _ in range(4000))
    clean = pa.Codec("zstd", compression_level=3).compress(d, asbytes=True)
    rejected = 0
    for _ in range(400):
        b = bytearray(clean)
        for _ in range(rng.randint(1, 4)):
            b[rng.randrange(len(b))] = rng.randrange(256)
        rc, _ = dec(zs, bytes(b), len(d))
        assert rc in (0, 1, 2, 3)
        rejected += rc != 0
    assert rejected > 300
    rc, _ = dec(zs, clean[: len(clean) // 2], len(d))  # truncated
    assert rc != 0
    rc, _ = dec(zs, clean, len(d) - 1)  # the slot one byte short
    assert rc == 2


def _bits_le(fields):
    """(value, nbits) fields packed LSB first."""
    acc = n = 0
    for v, nb in fields:
        acc |= v << n
        n += nb
    return acc.to_bytes((n + 7) // 8, "little")


def test_zstd_huffman_weights_zero_run_past_alphabet(zs):
    """A compressed-literals block whose FSE-coded Huffman weight table
    declares one symbol of probability 0 followed by a run of 66 more zeros:
    past the 12 weight symbols zstd allows (RFC 8878 4.2.1.2), and past the
    decoder's 64-entry count table.  Must end in a status (round-5 advice:
    such a run used to write past the table)."""
    hdesc = _bits_le([(0, 4), (1, 5)] + [(3, 2)] * 22 + [(0, 2)])
    hb = len(hdesc) + 3
    huf = bytes([hb]) + hdesc + b"\x00" * 3
    regen, comp = 100, len(huf) + 8
    lit_hdr = (2 | (0 << 2) | (regen << 4) | (comp << 14)).to_bytes(3, "little")
    body = lit_hdr + huf + b"\x55" * 8 + b"\x00"  # then no sequences
    block = (1 | (2 << 1) | (len(body) << 3)).to_bytes(3, "little") + body
    frame = bytes([0x28, 0xB5, 0x2F, 0xFD, 0x20, regen]) + block
    rc, _ = dec(zs, frame, regen)
    assert rc != 0
