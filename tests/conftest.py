"""Test configuration: `gpu` marker, import paths, shared helpers."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "duckdb-parquet-parser_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running full-size case")


@pytest.fixture(scope="session")
def ctx():
    from pqgpu import capi
    c = capi.Context(0)
    yield c
    c.close()


# Kernel-path fixtures shared by the GPU parity tests.
@pytest.fixture(params=["default", "big", "fused", "generic", "serial"])
def path(request, ctx):
    """Every kernel path that ships: "default" = what a chunk takes with the
    default options (dictionary BYTE_ARRAY on dict_pipe.hip: the run-table
    passes k_pipe_runs + k_pipe_codes3 + k_pipe_write; two-pass
    PLAIN BYTE_ARRAY, plain_ba.hip; tile-parallel PLAIN fixed width,
    fixed_fast.hip; the fused and generic kernels for chunks neither
    takes); "big" puts every page of a dictionary chunk through k_pipe_big
    (the large-page kernel) so it also meets small pages; "fused" forces the
    per-page fused BYTE_ARRAY kernel (dict_fused.hip) onto every BYTE_ARRAY
    chunk it can take; "generic" forces decode.hip's rows/scan/gather and
    per-page k_fixed (dictionary chunks: rows by k_wide_rows, a workgroup per
    page); "serial" is "generic" with the wave-per-page k_ba_rows, the byte-wise
    gather and k_fixed_levels2's large-LDS form.  PLAIN BYTE_ARRAY chunks take the one-pass kernel
    (k_plain_fused) under "default" and the two passes under "big"."""
    p = request.param
    ctx.set_option("big_all", int(p == "big"))
    ctx.set_option("dict_pipe", int(p in ("default", "big")))
    ctx.set_option("plain_ba", int(p in ("default", "big")))
    ctx.set_option("fused_ba", int(p not in ("generic", "serial")))
    ctx.set_option("fixed_plain", int(p not in ("generic", "serial")))
    ctx.set_option("wide_rows", int(p != "serial"))
    ctx.set_option("gather_rows", int(p != "serial"))
    ctx.set_option("levels_small", int(p != "serial"))
    ctx.set_option("plain_fused", int(p != "big"))
    ctx.set_option("fixed_fused", int(p == "big"))
    yield p
    for k in ("dict_pipe", "plain_ba", "fused_ba", "fixed_plain", "plain_fused"):
        ctx.set_option(k, 1)
    ctx.set_option("fixed_fused", 0)
    ctx.set_option("big_all", 0)
    ctx.set_option("wide_rows", 1)
    ctx.set_option("gather_rows", 1)
    ctx.set_option("levels_small", 1)


@pytest.fixture(params=["window", "codes", "lanes", "nfa"])
def kernel(request, ctx):
    """Every page kernel: windowed DFA (default for chunks without dictionary
    pages), match bits over the pipe decode's codes (default for dictionary
    chunks the pipe path takes; "codes" with the run-table passes' codes), lane-per-page
    DFA (other dictionary chunks) and wave-per-page NFA (patterns whose DFA is
    over its size cap)."""
    ctx.set_option("regex_dfa", int(request.param != "nfa"))
    ctx.set_option("regex_plain", int(request.param == "window"))
    ctx.set_option("regex_codes", int(request.param in ("window", "codes")))
    yield request.param
    ctx.set_option("regex_dfa", 1)
    ctx.set_option("regex_plain", 1)
    ctx.set_option("regex_codes", 1)
