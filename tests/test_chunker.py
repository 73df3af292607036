"""The example driver's 4 KiB string chunker (/root/reference/src/main.cpp:17-32,
SURVEY §8f rank 3).  CPU: the oracle's C restatement (pqo_chunk_assign)
against a line-by-line Python restatement of the loop on hand-made and
generated columns (the reference's driver hard-codes its input path, so it
cannot be run here: parity is pinned to the restatement of its loop).  GPU:
pq_chunk_assign on the decoded column against the oracle, bit-exact."""
import numpy as np
import pytest

from oracle import oracle as O
from pqgpu import capi, gen
from util import to_oracle_chunk


def loop_restated(valid, offsets, chunk_size):
    """main.cpp:17-32 as written: chunk is a string; only its size matters."""
    n = len(valid)
    out = [0] * n
    size, chunk_id = 0, 0
    for r in range(n):
        if not valid[r]:
            continue
        if size >= chunk_size:
            size = 0
            chunk_id += 1
        ln = int(offsets[r + 1] - offsets[r])
        size += len(str(ln)) + ln
        out[r] = chunk_id
    return np.asarray(out, dtype=np.int64), chunk_id + 1


def _col(lens, nulls):
    valid = np.asarray([0 if i in nulls else 1 for i in range(len(lens))], dtype=np.uint8)
    L = np.where(valid == 1, np.asarray(lens, dtype=np.int64), 0)
    offs = np.concatenate([[0], np.cumsum(L)]).astype(np.int64)
    return O.Column(valid, offs, np.zeros(int(offs[-1]), np.uint8), [], capi.BYTE_ARRAY)


@pytest.mark.parametrize("chunk", [0, 1, 5, 12, 4096])
def test_oracle_chunker_vs_loop(chunk):
    rng = np.random.default_rng(chunk)
    cases = [_col([], set()), _col([3], set()), _col([3], {0}), _col([0, 0, 0, 9, 10, 99, 100, 1000], {2}),
             _col(rng.integers(0, 300, size=5000).tolist(), set(rng.integers(0, 5000, size=400).tolist()))]
    for col in cases:
        got, k = O.chunk_assign(col, chunk)
        exp, ke = loop_restated(col.valid, col.offsets, chunk)
        assert k == ke and np.array_equal(got, exp)


def test_oracle_chunker_known_answer():
    # weights: "3"+3 = 4 bytes each; chunk 8 -> strings 0,1 | 2,3 | 4
    col = _col([3, 3, 3, 3, 3], set())
    got, k = O.chunk_assign(col, 8)
    assert got.tolist() == [0, 0, 1, 1, 2] and k == 3
    # 10-byte string weighs 12; chunk 12 closes after each string
    got, k = O.chunk_assign(_col([10, 10, 1], {1}), 12)
    assert got.tolist() == [0, 0, 1] and k == 2


def _oracle_column(f, ch):
    rc, msg, col = O.read_all(f, to_oracle_chunk(ch))
    assert rc == 0, msg
    return col


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,rows,chunk", [("c3", 100_000, 4096), ("c2", 100_000, 4096), ("c3", 20_000, 0),
                                            ("c2", 20_000, 1), ("c3", 20_000, 100), ("c2", 20_000, 1 << 30),
                                            ("c3", 3_000_000, 4096), ("c2", 3_000_000, 65536)])
def test_gpu_chunker_vs_oracle(ctx, cfg, rows, chunk):
    cols = gen.c3_cols() if cfg == "c3" else gen.c2_cols()
    f = gen.build(cols, rows, 1, seed=11)
    ch = capi.File(f).chunk(0, 0)
    dc = ctx.upload(f, [ch])
    dc.decode()
    got, k = dc.chunk_assign(chunk)
    dc.free()
    exp, ke = O.chunk_assign(_oracle_column(f, ch), chunk)
    assert k == ke and np.array_equal(got, exp)


@pytest.mark.gpu
@pytest.mark.parametrize("null_frac", [1.0, 0.9])
def test_gpu_chunker_mostly_null(ctx, null_frac):
    cols = [gen.Col("s", gen.DICT_STRINGS, gen.BYTE_ARRAY, optional=True, null_frac=null_frac, dict_size=50,
                    len_min=0, len_max=300, max_run=3)]
    f = gen.build(cols, 30_000, 1, seed=5)
    ch = capi.File(f).chunk(0, 0)
    dc = ctx.upload(f, [ch])
    dc.decode()
    got, k = dc.chunk_assign(4096)
    dc.free()
    exp, ke = O.chunk_assign(_oracle_column(f, ch), 4096)
    assert k == ke and np.array_equal(got, exp)


@pytest.mark.gpu
@pytest.mark.slow
def test_gpu_chunker_c3_full_size(ctx):
    f = gen.build(gen.c3_cols(), 10_000_000, 1, seed=gen.CONFIG_SEEDS["C3"])
    ch = capi.File(f).chunk(0, 0)
    dc = ctx.upload(f, [ch])
    dc.decode()
    got, k = dc.chunk_assign(4096)
    dc.free()
    exp, ke = O.chunk_assign(_oracle_column(f, ch), 4096)
    assert k == ke and np.array_equal(got, exp)
