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


def data_page_ranges(table, world: int) -> list[tuple[int, int]]:
    """Byte-balanced contiguous ranges of a chunk's DATA pages (ordinals in walk
    order, the unit pq_chunk_upload_range takes) from its page table
    (capi.build_page_table): the library's planner, pq_plan_page_ranges
    (csrc/capi.hip).  Dictionary pages are not counted: every shard that needs
    one gets it replicated."""
    from . import capi
    return capi.plan_page_ranges(table, world)


def data_page_ranges_py(table, world: int) -> list[tuple[int, int]]:
    """The same plan in numpy (page_ranges): the cross-check of the C planner."""
    sizes = [p.payload_size for p in table if p.page_type == 0]
    return page_ranges(sizes, world)


def row_page_range(table, chunk_first_row: int, lo: int, hi: int) -> tuple[int, int]:
    """Data-page range [a, b) of a chunk (page table from build_page_table)
    owned by the shard whose global rows are [lo, hi): the pages whose first
    row, offset by the chunk's global first row, falls in [lo, hi).  Shards
    with disjoint row ranges covering the column own every page exactly once,
    and every rank plans its part from its own row groups' tables (C4 leg of
    bench.py: rows balanced instead of bytes, no rank generates another's
    row groups)."""
    firsts = [chunk_first_row + p.first_row for p in table if p.page_type == 0]
    a = sum(1 for x in firsts if x < lo)
    b = sum(1 for x in firsts if x < hi)
    return a, b


def range_rows(table, begin: int, end: int) -> tuple[int, int]:
    """(first chunk row, row count) of data pages [begin, end)."""
    data = [p for p in table if p.page_type == 0]
    if begin >= end:
        first = data[begin].first_row if begin < len(data) else sum(p.num_values for p in data)
        return first, 0
    return data[begin].first_row, sum(p.num_values for p in data[begin:end])


def extract_range(file: bytes, chunk, table, begin: int, end: int):
    """The bytes one shard needs, as a standalone column chunk: the header and
    payload of data pages [begin, end) and of every dictionary page they use,
    in walk order, plus a chunk descriptor that walks exactly those pages.
    (What a rank reads from storage for its range; the tests decode it with
    the oracle to check a shard plan without a GPU.)  Returns (bytes, desc)."""
    from .capi import ChunkDesc
    data_pos = [i for i, p in enumerate(table) if p.page_type == 0]
    pick = set(data_pos[begin:end])
    dicts = {table[i].dict_page for i in pick if table[i].dict_page >= 0}
    out = bytearray()
    first_data = None
    nvals = 0
    for i, p in enumerate(table):
        if i not in pick and i not in dicts:
            continue
        if i in pick and first_data is None:
            first_data = len(out)
        lo, hi = p.header_offset, p.payload_offset + p.payload_size
        piece = file[lo:min(hi, len(file))]
        out += piece + bytes(hi - lo - len(piece))
        if i in pick:
            nvals += p.num_values
    d = ChunkDesc()
    d.num_values = nvals
    d.data_page_offset = first_data if first_data is not None else len(out)
    d.dictionary_page_offset = 0
    d.has_dictionary_page_offset = 1 if dicts else 0
    d.codec = chunk.codec
    d.type = chunk.type
    d.max_def_level = chunk.max_def_level
    d.max_rep_level = chunk.max_rep_level
    return bytes(out), d


def column_page_shards(page_index, col: int, world: int) -> list[list[tuple[int, int, int]]]:
    """Global data-page sharding of one column across row groups (R-PAGEIDX
    order, build_page_index parquet_reader.cpp:559-605): the column's pages
    split into `world` contiguous byte-balanced ranges; each rank's range as
    pieces (row_group, first data page, end data page) with page ordinals
    local to that row group's chunk (what pq_chunk_upload_range takes).
    `page_index` is File.page_index(): rows (data_offset, data_size, rg, col)."""
    pi = np.asarray(page_index, dtype=np.int64).reshape(-1, 4)
    mine = pi[pi[:, 3] == col]
    rgs = mine[:, 2]
    # ordinal of every page inside its row group's chunk
    local = np.zeros(len(mine), dtype=np.int64)
    for rg in np.unique(rgs):
        sel = np.nonzero(rgs == rg)[0]
        local[sel] = np.arange(len(sel))
    out = []
    for a, b in page_ranges(mine[:, 1], world):
        pieces = []
        i = a
        while i < b:
            rg = int(rgs[i])
            j = i
            while j < b and rgs[j] == rg:
                j += 1
            pieces.append((rg, int(local[i]), int(local[j - 1]) + 1))
            i = j
        out.append(pieces)
    return out
