"""GPU: mutated fixtures through every decode path and the regex scan
(SURVEY §5 "fuzz the decoder").  The mutants are test_fuzz_host.py's (page
headers and payload bytes of the small golden fixtures, seeded); the GPU
decode must report the oracle's status and, on success, its exact canonical
dump; the page filter must report the oracle's page set or the same error.
(The oracle is pinned to the compiled reference on these same mutants by
test_fuzz_host.py wherever the reference's behaviour is defined.)"""
import numpy as np
import pytest

from oracle import oracle as O
from pqgpu import capi
from test_fuzz_host import _mutants
from util import gpu_read_column, to_desc

pytestmark = pytest.mark.gpu

MUTANTS = _mutants(240, seed=23)


def _chunk(c):
    return O.Chunk(*c)


def _pages_with_e(f, ch):
    """1 per data page none of whose non-NULL values holds the byte 'e'
    (pattern "e"; mutated payloads are not UTF-8, so a bytes search)."""
    rc, msg, col = O.read_all(f, ch)
    assert rc == 0, msg
    out = []
    for (_, ptype, _, first, nrows) in col.pages:
        if ptype != 0:
            continue
        sat = any(col.valid[r] and b"e" in bytes(col.data[col.offsets[r]:col.offsets[r + 1]])
                  for r in range(first, first + nrows))
        out.append(0 if sat else 1)
    return np.array(out, dtype=np.uint8)


@pytest.mark.parametrize("part", range(4))
def test_mutants_decode(ctx, path, part):
    for i, (name, f, c) in enumerate(MUTANTS):
        if i % 4 != part:
            continue
        ch = _chunk(c)
        rc_o, msg_o, col = O.read_all(f, ch)
        rc_g, msg_g, d_g = gpu_read_column(ctx, f, [to_desc(ch)])
        assert rc_g == rc_o, (name, i, path, rc_g, msg_g, rc_o, msg_o)
        if rc_o == 0:
            assert d_g == O.dump_column(col), (name, i, path)
        elif rc_o in (-2, -4):
            assert msg_g == msg_o, (name, i, path)


def test_mutants_regex(ctx, kernel):
    n = 0
    for i, (name, f, c) in enumerate(MUTANTS):
        ch = _chunk(c)
        if ch.type != capi.BYTE_ARRAY:
            continue
        rc_o, msg_o, _ = O.read_all(f, ch)
        dc = None
        try:
            dc = ctx.upload(f, [to_desc(ch)])
            if rc_o != 0:
                try:
                    dc.regex_pages("e", False)
                    raised = None
                except capi.PqError as e2:
                    raised = e2
                assert raised is not None, (name, i, kernel, rc_o, msg_o)
                assert raised.code == rc_o, (name, i, kernel, raised.msg, msg_o)
            else:
                got = dc.regex_pages("e", False)
                assert np.array_equal(got, _pages_with_e(f, ch)), (name, i, kernel)
            n += 1
        except capi.PqError as e:  # the upload's walk failed: the oracle failed the same way
            assert rc_o == e.code, (name, i, e.msg, msg_o)
        finally:
            if dc is not None:
                dc.free()
    assert n > 20
