#!/usr/bin/env python3
"""A/B of ColumnReader::read_all (std::vector<Value> out) on the C2 chunk at
10M and 1M rows: tools/api_check time_read_all from this tree and from the
builds named in argv (directories holding pqgpu/api_check + libpqgpu.so)."""
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "duckdb-parquet-parser_amd")]
from pqgpu import gen  # noqa: E402

tools = [os.path.join(ROOT, "duckdb-parquet-parser_amd", "pqgpu", "api_check")] + \
    [os.path.join(d, "pqgpu", "api_check") for d in sys.argv[1:]]
with tempfile.TemporaryDirectory() as td:
    for rows in (10_000_000, 1_000_000):
        path = os.path.join(td, f"c2_{rows}.parquet")
        with open(path, "wb") as fh:
            fh.write(gen.build(gen.c2_cols(), rows, 1, seed=gen.CONFIG_SEEDS["C2"]))
        for rnd in range(2):
            for tool in tools:
                r = subprocess.run([tool, path, "time_read_all", "0", "0", "7", os.path.join(td, "d")],
                                   stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=600)
                js = json.loads(r.stdout.decode().strip().splitlines()[-1]) if r.returncode == 0 else {"err": r.stderr.decode()[-300:]}
                print(json.dumps({"tool": os.path.relpath(tool, ROOT), "rows": rows, "round": rnd,
                                  "read_all_ms": js.get("read_all_ms"), "Mvalues_per_s": round(rows / js["read_all_ms"] / 1e3, 1) if "read_all_ms" in js else None,
                                  "phases": js.get("phases_ms"), "samples": js.get("read_all_samples")}), flush=True)
