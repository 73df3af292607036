"""k_pipe_big diagnostics (fused_debug bit 27): the first page (walk order)
that a step would send to the exact decoder, as pos = the step (1 shape,
2 prologue, 3 header lists, 4 records [+16 flag, +32 no def records, +64 no
index records], 8 levels above max_def), need = the page, size = its bytes."""
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
