"""Shared helpers: run the oracle (checker) and the HIP path on the same input."""
from __future__ import annotations

from oracle import oracle as O
from pqgpu import capi


def to_oracle_chunk(d) -> O.Chunk:
    if isinstance(d, O.Chunk):
        return d
    if isinstance(d, dict):
        return O.Chunk(d["num_values"], d["data_page_offset"], d["dictionary_page_offset"],
                       d["codec"], d["type"], d["max_def"], d["max_rep"])
    return O.Chunk(d.num_values, d.data_page_offset,
                   d.dictionary_page_offset if d.has_dictionary_page_offset else None, d.codec,
                   d.type, d.max_def_level, d.max_rep_level)


def to_desc(c) -> capi.ChunkDesc:
    if isinstance(c, capi.ChunkDesc):
        return c
    if isinstance(c, dict):
        c = to_oracle_chunk(c)
    d = capi.ChunkDesc()
    d.num_values = c.num_values
    d.data_page_offset = c.data_page_offset
    d.has_dictionary_page_offset = 1 if c.dictionary_page_offset is not None else 0
    d.dictionary_page_offset = c.dictionary_page_offset or 0
    d.codec = c.codec
    d.type = c.type
    d.max_def_level = c.max_def
    d.max_rep_level = c.max_rep
    return d


def oracle_read_column(file: bytes, chunks) -> tuple[int, str, bytes | None]:
    """ParquetReader::read_column semantics: chunks decoded in order and
    concatenated; the first failing chunk ends the read."""
    out = []
    for ch in chunks:
        rc, msg, col = O.read_all(file, to_oracle_chunk(ch))
        if rc != 0:
            return rc, msg, None
        out.append(O.dump_column(col))
    return 0, "", b"".join(out)


def gpu_read_column(ctx, file: bytes, chunks) -> tuple[int, str, bytes | None]:
    descs = [to_desc(c) for c in chunks]
    try:
        dc = ctx.upload(file, descs)
    except capi.PqError as e:
        return e.code, e.msg, None
    try:
        dc.decode()
    except capi.PqError as e:
        dc.free()
        return e.code, e.msg, None
    host = dc.to_host()
    dc.free()
    return 0, "", capi.canonical_dump(host)


def file_chunks(file: bytes, col: int):
    F = capi.File(file)
    return [F.chunk(rg, col) for rg in range(F.num_row_groups)]
