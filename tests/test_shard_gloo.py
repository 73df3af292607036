"""CPU: the multi-GPU shard plan, single process and with
world_size-2 gloo.

Shards are contiguous, byte-balanced ranges of a chunk's data pages (the
product's page table from pq_build_page_table → shard.data_page_ranges), each
decoded independently given the chunk's dictionary
(/root/reference/src/reader/column_reader.cpp:140-225), with no collective on
the data path; row offsets are a host exclusive scan.  Without a GPU the
shard's bytes (shard.extract_range: its data pages + the dictionary pages
they use) are decoded by the oracle (the checker); the -m gpu twin in
test_gpu_shard.py decodes the same ranges with pq_chunk_upload_range.  The
concatenation of shard dumps must equal the unsharded dump byte for byte.
"""
import hashlib
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from pqgpu import capi, gen
from pqgpu.shard import (data_page_ranges, data_page_ranges_py, extract_range, page_ranges, range_rows,
                         rank_row_groups, shard_row_offsets)


def test_page_ranges_cover_and_balance():
    rng = np.random.default_rng(1)
    for world in (1, 2, 3, 4, 8):
        sizes = rng.integers(200, 1200, size=2000)
        rs = page_ranges(sizes, world)
        assert len(rs) == world
        assert rs[0][0] == 0 and rs[-1][1] == len(sizes)
        for (a, b), (c, d) in zip(rs, rs[1:]):
            assert b == c and a <= b
        loads = [sizes[a:b].sum() for a, b in rs]
        assert max(loads) - min(loads) <= 2 * sizes.max()


def test_page_ranges_degenerate():
    assert page_ranges([], 4) == [(0, 0)] * 4
    assert page_ranges([5], 2)[0][0] == 0 and page_ranges([5], 2)[-1][1] == 1


def test_c_planner_equals_numpy_plan():
    """pq_plan_page_ranges (the library planner ParquetReader::read_column's
    device sharding uses) == the numpy plan, on random tables with dictionary
    pages interleaved, empty tables and world > pages."""
    rng = np.random.default_rng(5)
    for trial in range(60):
        n = int(rng.integers(0, 300))
        table = []
        for i in range(n):
            dict_page = bool(rng.random() < 0.05)
            table.append(capi.PageDesc(payload_size=int(rng.integers(0, 1 << int(rng.integers(1, 22)))),
                                       page_type=2 if dict_page else 0))
        for world in (1, 2, 3, 5, 8, 17, 400):
            assert data_page_ranges(table, world) == data_page_ranges_py(table, world), (trial, world)
    with pytest.raises(capi.PqError):
        capi.plan_page_ranges([], 0)


def test_c_planner_on_real_tables():
    for name, f, ch in _cases():
        rc, msg, table = capi.build_page_table(f, ch)
        assert rc == 0, msg
        for world in (2, 4, 8):
            assert data_page_ranges(table, world) == data_page_ranges_py(table, world), name


def test_rank_row_groups_partition():
    for nrg in (1, 7, 10, 100):
        for world in (1, 2, 4, 8):
            got = sum((rank_row_groups(nrg, r, world) for r in range(world)), [])
            assert got == list(range(nrg))


def test_shard_row_offsets():
    assert shard_row_offsets([3, 0, 5]).tolist() == [0, 3, 3]


def _cases():
    """(name, file, chunk) — C2 ref/arrow layout, C4's dictionary and PLAIN
    string columns and an OPTIONAL DOUBLE, small enough for the oracle."""
    c2r = gen.build(gen.c2_cols(), 30000, 1, seed=2, layout=gen.REF_LAYOUT)
    c2a = gen.build(gen.c2_cols(), 30000, 1, seed=2, layout=gen.ARROW_LAYOUT, rows_per_page=1500)
    c4 = gen.build(gen.c4_cols(), 12000, 1, seed=4, layout=gen.ARROW_LAYOUT, rows_per_page=700)
    out = [("c2_ref", c2r, capi.File(c2r).chunk(0, 0)), ("c2_arrow", c2a, capi.File(c2a).chunk(0, 0))]
    F4 = capi.File(c4)
    for ci in (3, 6, 7):
        out.append((f"c4_c{ci}", c4, F4.chunk(0, ci)))
    return out


def _oracle_dump(file, desc):
    from oracle import oracle as O
    from util import to_oracle_chunk
    rc, msg, col = O.read_all(file, to_oracle_chunk(desc))
    assert rc == 0, msg
    return O.dump_column(col), len(col.valid)


@pytest.mark.parametrize("world", [2, 3, 8])
def test_page_range_shards_equal_whole_chunk(world):
    for name, f, ch in _cases():
        rc, msg, table = capi.build_page_table(f, ch)
        assert rc == 0, msg
        whole, nrows = _oracle_dump(f, ch)
        ranges = data_page_ranges(table, world)
        parts, rows = [], []
        for a, b in ranges:
            sub, d = extract_range(f, ch, table, a, b)
            if b > a:
                dump, n = _oracle_dump(sub, d)
            else:
                dump, n = b"", 0
            first, cnt = range_rows(table, a, b)
            assert n == cnt, (name, a, b)
            parts.append(dump)
            rows.append(n)
        assert shard_row_offsets(rows).tolist() == [range_rows(table, a, b)[0] for a, b in ranges]
        assert sum(rows) == nrows
        assert b"".join(parts) == whole, name


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    """One rank: the product's page table and shard plan, its own range only."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = {}
    for name, f, ch in _cases():
        rc, msg, table = capi.build_page_table(f, ch)
        assert rc == 0, msg
        a, b = data_page_ranges(table, world)[rank]
        sub, d = extract_range(f, ch, table, a, b)
        dump, n = _oracle_dump(sub, d) if b > a else (b"", 0)
        out[name] = (n, hashlib.sha256(dump).hexdigest(), dump if len(dump) < (1 << 20) else None)
    gathered = [None] * world
    dist.all_gather_object(gathered, out)
    if rank == 0:
        q.put(gathered)
    dist.destroy_process_group()


def test_gloo_two_ranks_page_shards_equal_single():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    gathered = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for name, f, ch in _cases():
        whole, nrows = _oracle_dump(f, ch)
        rows = [gathered[r][name][0] for r in range(world)]
        offs = shard_row_offsets(rows)
        assert offs[-1] + rows[-1] == nrows
        parts = [gathered[r][name][2] for r in range(world)]
        assert all(p is not None for p in parts)
        assert b"".join(parts) == whole, name


def test_row_page_range_partitions_pages():
    """Ranks with disjoint row ranges covering a multi-row-group column own
    every data page exactly once (bench.py C4 leg)."""
    from pqgpu.shard import row_page_range
    rg_rows = 9000
    f = gen.build(gen.c4_cols(), rg_rows, 3, seed=4, layout=gen.ARROW_LAYOUT, rows_per_page=700)
    F = capi.File(f)
    for ci in (0, 3, 6, 7):
        tables = []
        for g in range(3):
            rc, msg, t = capi.build_page_table(f, F.chunk(g, ci))
            assert rc == 0, msg
            tables.append(t)
        for world in (1, 2, 3, 5, 8):
            per = -(-3 * rg_rows // world)
            owned = [0] * 3
            for r in range(world):
                lo, hi = per * r, min(per * (r + 1), 3 * rg_rows)
                for g in range(3):
                    a, b = row_page_range(tables[g], g * rg_rows, lo, hi)
                    assert a == owned[g]  # contiguous, in rank order
                    owned[g] = b
            assert owned == [sum(1 for p in t if p.page_type == 0) for t in tables]
