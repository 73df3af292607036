"""CPU: the C-ABI library, the host format layer, the regex compiler and the
generator — everything that runs without a GPU."""
import hashlib
import json
import os
import random
import zlib
import re

import pytest

from oracle import oracle as O
from pqgpu import capi, gen

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def declared_symbols():
    with open(os.path.join(ROOT, "include", "pq_gpu.h")) as fh:
        src = fh.read()
    return sorted(set(re.findall(r"\b(pq_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    L = capi.lib()
    names = declared_symbols()
    assert len(names) >= 30
    missing = [n for n in names if not hasattr(L, n)]
    assert missing == []


def test_context_create_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(capi.PqError):
        capi.Context(0)


def test_file_open_errors():
    with pytest.raises(capi.PqError, match="too small"):
        capi.File(b"PAR1")
    with pytest.raises(capi.PqError, match="magic"):
        capi.File(b"XXXX" + b"\0" * 20)


# ── regex compiler vs Python re (the R-REGEX golden) ───────────────────────
PATTERNS = ["special.*requests", "^(carefully|quickly) ", "[0-9]", "e", "a|b", "^$", "x*",
            "ab{2,3}c", "(?:foo|ba+r)$", "[^a-z ]", r"\d+\s", r"\w\W", "^abc$", "q.u", "a.c", ".",
            "^.$", "é", "[^x]y", "(a|)b", "ab?c", "a{2}", "a{1,}b", "[]a]", "[a-]x", r"\.",
            "(a*)*b", "^(a|b)*$", "c$|^d", "(?P<w>ab)+", "a+?b", r"\S\s\S", r"[\d\-]+", "$", "^",
            "a^b", "b$c", r"\Aab", r"ab\Z", "é.$", "[^é]"[:0] + "[^q]+$", "(ab|a)(bc|c)", ".*",
            "fo{0}x", "s{1}p", "(x|y|z){2,4}"]
ALPHABET = "abcdqxyz éè.-_]!09 \t"


def random_strings(seed, n=300):
    rng = random.Random(seed)
    out = ["", "a", "ab", "abc", "special requests", "quickly x", "carefully ", "é", "aéc", "qéu"]
    for _ in range(n):
        out.append("".join(rng.choice(ALPHABET) for _ in range(rng.randrange(0, 12))))
    return out


@pytest.mark.parametrize("pattern", PATTERNS)
def test_regex_host_matches_python_re(pattern):
    rc, msg = capi.regex_check(pattern)
    assert rc == 0, msg
    rx = re.compile(pattern, re.ASCII)
    for s in random_strings(zlib.crc32(pattern.encode()) & 0xFFFF):
        exp = rx.search(s) is not None
        assert bool(capi.regex_match_host(pattern, s.encode())) == exp, (pattern, s)


@pytest.mark.parametrize("pattern", PATTERNS)
def test_regex_dfa_matches_python_re(pattern):
    """The subset-construction DFA the page kernel runs equals Python re."""
    rx = re.compile(pattern, re.ASCII)
    if capi.regex_match_host_dfa(pattern, b"") == -8:
        pytest.skip("DFA over its size cap: the NFA kernel runs this pattern")
    for s in random_strings(zlib.crc32(pattern.encode()) & 0xFFFF):
        exp = rx.search(s) is not None
        assert capi.regex_match_host_dfa(pattern, s.encode()) == int(exp), (pattern, s)


@pytest.mark.parametrize("pattern", PATTERNS + ["zebra|quartz", "x[0-9]q", "(?:jq|qj)k", "^q", "Q.*Z"])
def test_regex_dfa_sinks_absorb(pattern):
    """The absorbing-state mask k_regex_plain<true> stops a batch on holds
    DEAD and ACCEPT."""
    rc, sinks = capi.regex_dfa_sinks(pattern)
    if rc == -8:
        pytest.skip("DFA over its size cap")
    assert rc == 0
    assert sinks & 0b11 == 0b11  # DEAD and ACCEPT


@pytest.mark.parametrize("pattern,why", [
    ("a**", "multiple repeat"), ("(", "missing )"), ("a{,3}", "{,n}"), (r"\b", "escape"),
    ("(?=a)", "group construct"), ("[é]", "non-ASCII"), ("*a", "nothing to repeat"),
    ("^*", "nothing to repeat"), (r"(a)\1", "escape"), ("a" * 70, "64 positions"),
])
def test_regex_rejects_outside_subset(pattern, why):
    rc, msg = capi.regex_check(pattern)
    assert rc == -22 and why in msg


# ── generator ──────────────────────────────────────────────────────────────
def test_generator_is_deterministic_against_committed_fixtures():
    """Byte-identical regeneration of committed inputs (portable PRNG, no libm)."""
    cases = {
        "c1_int32_ref": lambda: gen.build(gen.c1_cols(), 10000, 1, seed=1),
        "c2_dict_arrow": lambda: gen.build(gen.c2_cols(), 20000, 1, seed=2, layout=gen.ARROW_LAYOUT,
                                           rows_per_page=5000),
        "c4_mixed_arrow": lambda: gen.build(gen.c4_cols(), 2000, 2, seed=4, layout=gen.ARROW_LAYOUT,
                                            rows_per_page=600),
    }
    for name, fn in cases.items():
        with open(os.path.join(GOLDEN, name + ".parquet"), "rb") as fh:
            assert fn() == fh.read(), name


def test_c1_file_size_matches_survey_probe():
    # INT32 PLAIN 10,000 rows, ref-layout = 40 pages, 40,882 B (without footer pad)
    f = gen.build(gen.c1_cols(), 10000, 1, seed=1, footer_pad=False)
    assert len(f) == 40882
    assert capi.File(f).page_index().shape[0] == 40


@pytest.mark.skipif(not O.have_ref(), reason="reference harness not built")
@pytest.mark.parametrize("cols,n", [(gen.c2_cols(), 6000), (gen.c3_cols(), 800), (gen.c4_cols(), 700)])
def test_ref_layout_equals_reference_writer(tmp_path, cols, n):
    f = gen.build(cols, n, 1, seed=5, footer_pad=False)
    path = str(tmp_path / "w.parquet")
    O.ref_write(path, [(c.name, c.type, 1 if c.optional else 0, 0 if c.type == gen.BYTE_ARRAY else -1,
                        gen.values_dump(c, i, n, 0, 5)) for i, c in enumerate(cols)], n)
    with open(path, "rb") as fh:
        assert fh.read() == f


def test_generator_values_match_oracle_decode():
    cols = gen.c4_cols()
    f = gen.build(cols, 1500, 1, seed=8, layout=gen.ARROW_LAYOUT, rows_per_page=400)
    F = capi.File(f)
    from util import to_oracle_chunk
    for ci, c in enumerate(cols):
        rc, msg, col = O.read_all(f, to_oracle_chunk(F.chunk(0, ci)))
        assert rc == 0, msg
        assert O.dump_column(col) == gen.values_dump(c, ci, 1500, 0, 8)
