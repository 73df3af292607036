#!/usr/bin/env python3
"""Writes tests/golden/bench_expect.json: expected regex page sets of the
bench's full-size legs, computed HERE (CPU) with the oracle's decode
(oracle/pq_oracle.c, pinned to the compiled reference) and Python `re`
(the R-REGEX contract), so bench.py can validate its GPU results
on the box without the reference.  Stored as sha256 of the 0/1 page-flag
bytes plus the reported count.  Decode results are validated in bench.py
against the generator's own value dump (pinned to the oracle by
tests/test_host_cpu.py), which needs no stored expectation."""
import hashlib
import json
import os
import re
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "duckdb-parquet-parser_amd"), os.path.join(ROOT, "tests")]
from oracle import oracle as O  # noqa: E402
from pqgpu import capi, gen  # noqa: E402
from util import to_oracle_chunk  # noqa: E402


def page_flags(f: bytes, ch, pattern: str, neg: bool = False) -> np.ndarray:
    rc, msg, col = O.read_all(f, to_oracle_chunk(ch))
    assert rc == 0, msg
    rc, msg, table = capi.build_page_table(f, ch)
    assert rc == 0, msg
    valid = np.asarray(col.valid)
    off = np.asarray(col.offsets)
    data = bytes(col.data)
    rx = re.compile(pattern, re.ASCII)
    cache = {}
    flags = []
    for p in table:
        if p.page_type != 0:
            continue
        rep = True
        for r in range(p.first_row, p.first_row + p.num_values):
            if not valid[r]:
                continue
            s = data[off[r]:off[r + 1]]
            m = cache.get(s)
            if m is None:
                m = cache[s] = rx.search(s.decode("utf-8", "surrogateescape")) is not None
            if m != neg:
                rep = False
                break
        flags.append(1 if rep else 0)
    return np.asarray(flags, dtype=np.uint8)


def entry(flags: np.ndarray) -> dict:
    return {"pages": int(len(flags)), "reported": int(flags.sum()),
            "sha256": hashlib.sha256(flags.tobytes()).hexdigest()}


ROWS = 10_000_000
# four patterns, each with and without --neg-regex
C3_PATTERNS = ["special.*requests", "^(carefully|quickly) ", "[0-9]", "e"]
C5_PATTERNS = ["^qx"]


def c3_job(rank: int) -> dict:
    """bench.py c3_legs on rank `rank`: its own 10M-row row group (first_rg=rank)."""
    f = gen.build(gen.c3_cols(), ROWS, 1, seed=gen.CONFIG_SEEDS["C3"], first_rg=rank)
    ch = capi.File(f).chunk(0, 0)
    out = {}
    for pat in C3_PATTERNS:
        for neg in (0, 1):
            out[f"c3|{ROWS}|rg{rank}|{pat}|{neg}"] = entry(page_flags(f, ch, pat, bool(neg)))
    return out


def c5_job(rg: int, layout: int = gen.ARROW_LAYOUT) -> dict:
    """bench.py c5_leg: row group `rg` of the C5 column (rank r holds row
    groups [r * c5_rgs, (r + 1) * c5_rgs)), arrow or reference layout."""
    f = gen.build(gen.c2_cols(), ROWS, 1, seed=gen.CONFIG_SEEDS["C5"], layout=layout, first_rg=rg)
    ch = capi.File(f).chunk(0, 0)
    key = "c5" if layout == gen.ARROW_LAYOUT else "c5ref"
    return {f"{key}|{ROWS}|rg{rg}|{pat}": entry(page_flags(f, ch, pat)) for pat in C5_PATTERNS}


def c5ref_job(rg: int) -> dict:
    return c5_job(rg, gen.REF_LAYOUT)


def main():
    """usage: make_bench_expect.py [ranks] [c5_rgs_per_rank] [processes]"""
    import multiprocessing as mp
    ranks = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    c5_rgs = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    procs = int(sys.argv[3]) if len(sys.argv) > 3 else 6
    only = os.environ.get("ONLY", "c3,c5,c5ref").split(",")
    jobs = ([(c3_job, r) for r in range(ranks)] if "c3" in only else []) + \
           ([(c5_job, g) for g in range(ranks * c5_rgs)] if "c5" in only else []) + \
           ([(c5ref_job, g) for g in range(ranks * c5_rgs)] if "c5ref" in only else [])
    path = os.path.join(ROOT, "tests", "golden", "bench_expect.json")
    out = json.load(open(path)) if os.path.exists(path) else {}
    with mp.get_context("fork").Pool(procs) as pool:
        for d in pool.imap_unordered(_run, jobs):
            out.update(d)
            print(len(out), flush=True)
    with open(path, "w") as fh:
        json.dump(out, fh, indent=0, sort_keys=True)


def _run(job):
    fn, arg = job
    return fn(arg)


if __name__ == "__main__":
    main()
