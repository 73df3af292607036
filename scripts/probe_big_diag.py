"""k_pipe_big step-5 diagnostics (fused_debug bit 27): per page, the def /
index record counts, header-list lengths, error flag, segments and def
record capacity, reported through the page error record."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "duckdb-parquet-parser_amd")]
from pqgpu import capi, gen  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
col = gen.Col("s", gen.DICT_STRINGS, gen.BYTE_ARRAY, optional=True, null_frac=0.05, dict_size=100_000,
              len_min=4, len_max=9, max_run=16)
f = gen.build([col], rows, 1, seed=gen.CONFIG_SEEDS["C2"], layout=gen.ARROW_LAYOUT)
ctx = capi.Context(0)
ctx.set_option("fused_debug", 1 << 27)
dc = ctx.upload(f, [capi.File(f).chunk(0, 0)])
try:
    dc.decode()
    print("no error reported")
except capi.PqError as e:
    print("diag:", e.msg)
