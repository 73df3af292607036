"""Page-range / row-group sharding across GPUs.

Every data page decodes independently (column_reader.cpp:140-225 needs only
the page, its header, the max levels and the chunk's dictionary), so the
multi-GPU plan is embarrassingly parallel: contiguous ranges of the global
page order, balanced by payload bytes, one range per GPU, no collective on
the data path.  Row offsets of each shard are a host prefix sum.
"""
from __future__ import annotations

import numpy as np


def page_ranges(page_bytes, world: int) -> list[tuple[int, int]]:
    """Split pages [0, n) into `world` contiguous ranges with near-equal byte
    totals (cut where the running total crosses k/world of the sum)."""
    b = np.asarray(page_bytes, dtype=np.int64)
    n = len(b)
    if world <= 1 or n == 0:
        return [(0, n)] + [(n, n)] * max(0, world - 1)
    cum = np.cumsum(b)
    total = int(cum[-1]) if n else 0
    cuts = [0]
    for k in range(1, world):
        target = total * k / world
        c = int(np.searchsorted(cum, target, side="left")) + 1
        cuts.append(min(max(c, cuts[-1]), n))
    cuts.append(n)
    return [(cuts[i], cuts[i + 1]) for i in range(world)]


def rank_row_groups(nrg: int, rank: int, world: int) -> list[int]:
    """Contiguous block of row groups for `rank` (C4/C5: 10 / 100 row groups)."""
    base, extra = divmod(nrg, world)
    start = rank * base + min(rank, extra)
    cnt = base + (1 if rank < extra else 0)
    return list(range(start, start + cnt))


def shard_row_offsets(rows_per_shard) -> np.ndarray:
    """Global first row of each shard (host exclusive scan, no collective)."""
    r = np.asarray(rows_per_shard, dtype=np.int64)
    return np.concatenate([[0], np.cumsum(r)[:-1]]) if len(r) else r
