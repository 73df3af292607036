"""CPU check of the hand-built DEFLATE fixture (tests/deflate_craft.py): the
stream is valid per zlib and really uses code 16 after a zero run."""
import struct
import zlib

import deflate_craft as D


def test_crafted_stream_is_valid_and_uses_16_after_zero_run():
    data = b"".join(struct.pack("<i", v) for v in [3, 1, 4, 1, 5, 9, 2, 6] * 40)
    raw = D.deflate_16_after_zero_run(data)   # asserts the 16-after-run shape itself
    assert zlib.decompress(raw, -15) == data
    member = D.gzip_member(raw, data)
    assert zlib.decompress(member, 16 + 15) == data
