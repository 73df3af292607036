"""Codec edge cases outside pyarrow's output (codec.hip):
a DEFLATE dynamic block whose code-length sequence has code 16 right after a
17/18 zero run (RFC 1951: 16 repeats the last length written, 0 there), and
GZIP member trailers whose CRC-32 does not match the data (must fail, not
decode silently).  Built by tests/deflate_craft.py, checked by Python's zlib."""
import struct

import numpy as np
import pytest

import deflate_craft as D
import pqbuild as B
from pqgpu import capi
from util import to_desc

pytestmark = pytest.mark.gpu

VALUES = [3, 1, 4, 1, 5, 9, 2, 6, 5, 3, 5, 8, 9, 7, 9, 3, 2, 3, 8, 4] * 13


def gzip_int32_file(crc=None):
    data = b"".join(struct.pack("<i", v) for v in VALUES)
    member = D.gzip_member(D.deflate_16_after_zero_run(data), data, crc)
    page = B.data_header(len(member), len(VALUES), usize=len(data)) + member
    f, ch = B.build_file([page], capi.INT32, False, len(VALUES), codec=2)
    d = to_desc(ch)
    d.ext_flags = capi.EXT_CODECS
    return f, d


def test_code16_after_zero_run(ctx):
    f, d = gzip_int32_file()
    dc = ctx.upload(f, [d])
    try:
        dc.decode()
        h = dc.to_host()
    finally:
        dc.free()
    assert np.array_equal(np.frombuffer(h.data.tobytes(), dtype="<i4"), np.array(VALUES, dtype=np.int32))
    assert h.validity.all()


def test_gzip_crc_mismatch_fails(ctx):
    import zlib
    data = b"".join(struct.pack("<i", v) for v in VALUES)
    f, d = gzip_int32_file(crc=zlib.crc32(data) ^ 0x10)
    with pytest.raises(capi.PqError) as ei:
        dc = ctx.upload(f, [d])
        dc.free()
    assert ei.value.code == -9 and "corrupt" in ei.value.msg  # PQ_ERR_DECOMPRESS
