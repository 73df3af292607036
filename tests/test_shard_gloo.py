"""CPU: the multi-GPU sharding plan with world_size-2 gloo.

Shards are contiguous page ranges / row-group blocks with no collective on
the data path; the only exchange is the host-side gather of per-shard
results.  The union of shard results must equal the 1-GPU (here: oracle)
result, byte for byte and in order.
"""
import hashlib
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from pqgpu import gen
from pqgpu.shard import page_ranges, rank_row_groups, shard_row_offsets


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


def test_rank_row_groups_partition():
    for nrg in (1, 7, 10, 100):
        for world in (1, 2, 4, 8):
            got = sum((rank_row_groups(nrg, r, world) for r in range(world)), [])
            assert got == list(range(nrg))


def test_shard_row_offsets():
    assert shard_row_offsets([3, 0, 5]).tolist() == [0, 3, 3]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle as O
    from pqgpu import capi
    from util import to_oracle_chunk
    cols = gen.c4_cols()
    f = gen.build(cols, 1500, 5, seed=4, layout=gen.ARROW_LAYOUT, rows_per_page=400)
    F = capi.File(f)
    mine = rank_row_groups(F.num_row_groups, rank, world)
    digests = {}
    for ci in range(len(cols)):
        parts = []
        for rg in mine:
            rc, msg, col = O.read_all(f, to_oracle_chunk(F.chunk(rg, ci)))
            assert rc == 0, msg
            parts.append(O.dump_column(col))
        digests[ci] = (mine, [hashlib.sha256(p).hexdigest() for p in parts])
    gathered = [None] * world
    dist.all_gather_object(gathered, digests)
    if rank == 0:
        q.put(gathered)
    dist.destroy_process_group()


def test_gloo_two_ranks_union_equals_single():
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
    # single-process reference: every row group in order
    from oracle import oracle as O
    from pqgpu import capi
    from util import to_oracle_chunk
    cols = gen.c4_cols()
    f = gen.build(cols, 1500, 5, seed=4, layout=gen.ARROW_LAYOUT, rows_per_page=400)
    F = capi.File(f)
    for ci in range(len(cols)):
        single = []
        for rg in range(F.num_row_groups):
            rc, msg, col = O.read_all(f, to_oracle_chunk(F.chunk(rg, ci)))
            single.append(hashlib.sha256(O.dump_column(col)).hexdigest())
        union = []
        for r in range(world):
            rgs, ds = gathered[r][ci]
            union += ds
        assert union == single
