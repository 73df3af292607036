"""GPU: full-size C3 regex parity (10M rows, ~293k pages).

The page sets of the four §8(d) patterns, each with and without --neg-regex,
must equal the committed digests of the oracle's page sets
(tests/golden/bench_expect.json, made by scripts/make_bench_expect.py from the
oracle's decode and Python `re`), on a cold scan (every scan walks the length
chains and files the string index, regex_index=2) and on the warm scans that
read the filed index.  The reported-page rule is the build's R-REGEX contract
(README.md:54-64): a page is reported iff no non-null value matches (with
neg: iff no non-null value fails to match)."""
import hashlib
import json
import os

import pytest

from pqgpu import capi, gen

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROWS = 10_000_000
PATTERNS = ("special.*requests", "^(carefully|quickly) ", "[0-9]", "e")


@pytest.fixture(scope="module")
def c3_chunk(ctx):
    f = gen.build(gen.c3_cols(), ROWS, 1, seed=gen.CONFIG_SEEDS["C3"])
    dc = ctx.upload(f, [capi.File(f).chunk(0, 0)])
    yield dc
    dc.free()


@pytest.fixture(scope="module")
def expect():
    with open(os.path.join(ROOT, "tests", "golden", "bench_expect.json")) as fh:
        return json.load(fh)


@pytest.mark.parametrize("neg", [False, True])
@pytest.mark.parametrize("pattern", PATTERNS)
def test_c3_full_size_page_sets(ctx, c3_chunk, expect, pattern, neg):
    e = expect[f"c3|{ROWS}|rg0|{pattern}|{int(neg)}"]
    for cold in (True, False):
        ctx.set_option("regex_index", 2 if cold else 1)
        try:
            flags = c3_chunk.regex_pages(pattern, neg)
        finally:
            ctx.set_option("regex_index", 1)
        assert len(flags) == e["pages"]
        assert int(flags.sum()) == e["reported"], (pattern, neg, cold)
        assert hashlib.sha256(flags.astype("u1").tobytes()).hexdigest() == e["sha256"], (pattern, neg, cold)
