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


def main():
    out = {}
    rows = 10_000_000
    c3 = gen.build(gen.c3_cols(), rows, 1, seed=gen.CONFIG_SEEDS["C3"])
    ch = capi.File(c3).chunk(0, 0)
    for pat in ("special.*requests",):
        out[f"c3|{rows}|{pat}"] = entry(page_flags(c3, ch, pat))
    del c3
    c5_rgs = int(os.environ.get("C5_RGS", "4"))
    c5 = gen.build(gen.c2_cols(), rows, c5_rgs, seed=gen.CONFIG_SEEDS["C5"], layout=gen.ARROW_LAYOUT)
    F = capi.File(c5)
    for pat in sys.argv[1:] or ["^qx"]:
        fl = np.concatenate([page_flags(c5, F.chunk(rg, 0), pat) for rg in range(c5_rgs)])
        out[f"c5|{rows}x{c5_rgs}|{pat}"] = entry(fl)
        print(pat, out[f"c5|{rows}x{c5_rgs}|{pat}"], flush=True)
    path = os.path.join(ROOT, "tests", "golden", "bench_expect.json")
    old = json.load(open(path)) if os.path.exists(path) else {}
    old.update(out)
    with open(path, "w") as fh:
        json.dump(old, fh, indent=1, sort_keys=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
