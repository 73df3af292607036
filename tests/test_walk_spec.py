"""CPU: the speculative parallel page walk (format.cpp
walk_chunk) yields exactly the serial walk's page table, status and message —
the serial walk being ColumnReader::read_all's header loop
(/root/reference/src/reader/column_reader.cpp:18-71), pinned to the compiled
reference by test_oracle_golden.py.  A chunk of >= 4 MiB with
total_compressed_size set walks speculatively (one thread per MiB); 0
forces the serial walk."""
import ctypes as C

import numpy as np
import pytest

from pqgpu import capi, gen


def _walk(f, ch, total):
    d = capi.ChunkDesc()
    C.memmove(C.byref(d), C.byref(ch), C.sizeof(ch))
    d.total_compressed_size = total
    rc, msg, t = capi.build_page_table(f, d)
    return rc, msg, bytes(t)


def _check(f, ch, totals=None):
    serial = _walk(f, ch, 0)
    for tot in totals or [ch.total_compressed_size]:
        assert _walk(f, ch, tot) == serial, tot
    return serial


def _files():
    return {
        "c3_ref": gen.build(gen.c3_cols(), 500_000, 1, seed=3),
        "c2_ref": gen.build(gen.c2_cols(), 12_000_000, 1, seed=2),
        "c3_arrow": gen.build(gen.c3_cols(), 500_000, 1, seed=3, layout=gen.ARROW_LAYOUT, rows_per_page=3000),
    }


@pytest.mark.parametrize("name", ["c3_ref", "c2_ref", "c3_arrow"])
def test_spec_walk_equals_serial(name):
    f = _files()[name]
    ch = capi.File(f).chunk(0, 0)
    assert ch.total_compressed_size >= 8 << 20
    rc, msg, t = _check(f, ch, [ch.total_compressed_size, ch.total_compressed_size // 2,
                                ch.total_compressed_size * 2, 8 << 20])
    assert rc == 0


@pytest.mark.parametrize("seed", range(6))
def test_spec_walk_corrupted_bytes(seed):
    """Random byte damage inside the chunk (headers and payload alike): both
    walks meet the same pages, then the same error text."""
    base = _files()["c3_ref" if seed % 2 == 0 else "c3_arrow"]
    ch = capi.File(base).chunk(0, 0)
    rng = np.random.default_rng(seed)
    b = bytearray(base)
    lo, hi = 4, 4 + ch.total_compressed_size
    for pos in rng.integers(lo + (hi - lo) // 4, hi, size=3 + seed):
        b[int(pos)] = int(rng.integers(0, 256))
    # and a header's compressed size at a page boundary of the true chain
    rc0, msg0, t = capi.build_page_table(base, ch)
    mid = t[len(t) // 2]
    b[mid.header_offset + 6] = 0x7F
    _check(bytes(b), ch)


def test_spec_walk_truncated_file():
    f = _files()["c3_ref"]
    ch = capi.File(f).chunk(0, 0)
    cut = f[: int(len(f) * 0.6)]
    rc, msg, t = _check(cut, ch)
    assert rc != 0 or len(t) > 0


def test_spec_walk_pyarrow_statistics(tmp_path):
    pa = pytest.importorskip("pyarrow")
    pq = pytest.importorskip("pyarrow.parquet")
    rng = np.random.default_rng(5)
    words = np.array([b"alpha", b"beta", b"gamma", b"delta", b"epsilon"])
    vals = [b" ".join(rng.choice(words, size=int(k))).decode() for k in rng.integers(1, 9, size=400_000)]
    p = tmp_path / "s.parquet"
    pq.write_table(pa.table({"s": vals}), p, compression="NONE", data_page_version="1.0", use_dictionary=False,
                   write_statistics=True, data_page_size=4096)
    f = p.read_bytes()
    ch = capi.File(f).chunk(0, 0)
    assert ch.total_compressed_size >= 8 << 20
    rc, msg, t = _check(f, ch)
    assert rc == 0 and len(t) > 100


def test_header_field8_not_struct_is_skipped():
    """PageHeader field 8 with a non-struct wire type (an i32 here) is skipped
    like any unknown field (metadata.cpp:149-151): the walk finds the same
    pages and header sizes as the reference, whose decode is unaffected."""
    import struct
    import pqbuild as B
    from oracle import oracle as O
    from util import to_oracle_chunk
    vals = [b"ab", b"cde", b"f"]
    pay = B.plain_ba(vals)
    hdr = bytes(B.TW().i32(1, 0).i32(2, len(pay)).i32(3, len(pay)).begin(5).i32(1, 3).i32(2, 0).i32(3, 3)
                .i32(4, 3).end().i32(8, 12345).stop().b)
    f, ch = B.build_file([hdr + pay, hdr + pay], gen.BYTE_ARRAY, False, 6)
    rc_o, msg_o, col = O.read_all(f, to_oracle_chunk(ch))
    assert rc_o == 0, msg_o
    rc, msg, t = capi.build_page_table(f, _desc(ch))
    assert rc == 0, msg
    assert len(t) == 2 and [p.num_values for p in t] == [3, 3]
    assert t[0].payload_offset - t[0].header_offset == len(hdr)
    assert t[1].header_offset == t[0].payload_offset + len(pay)


def _desc(ch):
    from util import to_desc
    return to_desc(ch)
