#!/usr/bin/env python3
"""Per-kernel VGPRs / scratch / occupancy of one HIP source (hipcc
-Rpass-analysis=kernel-resource-usage).  usage: kres.py FILE.hip [-o out.o]"""
import re
import subprocess
import sys

src = sys.argv[1]
pkg = "/root/repo/duckdb-parquet-parser_amd"
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", f"-I{pkg}/../include",
       f"-I{pkg}/csrc", f"-I{pkg}/include", "-c", src, "-o", "/tmp/kres.o", "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, stderr=subprocess.PIPE, stdout=subprocess.PIPE, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"remark:\s+(Function Name|VGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\S+)", line)
    if not m:
        continue
    k, v = m.group(1), m.group(2)
    if k == "Function Name":
        cur = re.sub(r"^_ZN3pqk12_GLOBAL__N_1\d+", "", v)[:48]
        rows[cur] = {}
    elif cur:
        rows[cur][k.split()[0]] = v
for n, r in rows.items():
    print(f"{n:50s} vgpr {r.get('VGPRs', '?'):>4s} scratch {r.get('ScratchSize', '?'):>4s} occ {r.get('Occupancy', '?'):>3s} lds {r.get('LDS', '?')}")
