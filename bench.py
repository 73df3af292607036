#!/usr/bin/env python3
"""Benchmark: decoded values/s (RLE + dictionary BYTE_ARRAY) and regex pages/s.

Workload (BASELINE.json configs[1] = SURVEY §8d C2): one BYTE_ARRAY UTF8
OPTIONAL column, 1000-entry dictionary, runs of 1+U[0,16) rows, 5% NULL,
reference-writer page layout (512 rows/page, bit width 10), synthetic data
from the deterministic generator.  One step = one full
ColumnReader::read_all-equivalent decode of a rank's pages on the GPU
(validity bitmap + int64 offsets + chars, all kernels), inputs resident in
HBM.

Multi-GPU: the job is the C2 column at N x 10M rows in N row
groups of 10M rows; rank r generates, decodes and validates row group r only
(the global page order cut at row-group boundaries).  Weak scaling, no
collective on the data path.  `python bench.py --gpus N` launches the N ranks itself
(torch.distributed.run) when WORLD_SIZE is not set; the driver's own
torch.distributed.run launch is used as is.  With N > 1 a strong-scaling
figure (the 10M-row chunk split N ways) is reported beside it.

Timing: W untimed warmup steps, then R = --repeats timed regions of exactly
K steps, each bracketed by barrier + device sync on both sides; per region
the max over ranks; `value` comes from the median region.

Further legs (not `value`): C3 regex page filter (configs[2]) and PLAIN
decode, C4 8 mixed columns, C5 dictionary decode + regex, end-to-end (host
walk + H2D + decode), CPU baselines.  Every leg's result is checked against
the generator's own value dump (pinned to the oracle by the CPU tests) or the
committed regex page-set digests (tests/golden/bench_expect.json).

Rank 0 prints ONE JSON line (contract in the task statement).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import socket
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "duckdb-parquet-parser_amd")
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md
# kernel timers (HIP events on the decode stream, capi.hip Timed)
KERNELS = ("dict_index", "dict_entries", "pipe_runs", "pipe_big", "wide_chars", "pipe_count", "pipe_codes", "pipe_write",
           "ba_fused", "ba_rows", "scan", "ba_gather", "plain_spec", "plain_ba", "fixed_plain", "fixed", "plain_opt")
REGEX_KERNELS = ("regex_dict", "regex_codes", "regex_lanes", "regex_plain", "regex_pages")
ROWS = 10_000_000
C3_PATTERNS = ("special.*requests", "^(carefully|quickly) ", "[0-9]", "e")
C5_PATTERN = "^qx"  # splits C5's pages (≈7% reported): not an all-miss scan


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--repeats", type=int, default=5, help="timed regions of --steps steps (median reported)")
    ap.add_argument("--rows", type=int, default=ROWS, help="C2 rows per GPU")
    ap.add_argument("--layout", choices=["ref", "arrow"], default="ref")
    ap.add_argument("--no-regex", action="store_true")
    ap.add_argument("--regex-rows", type=int, default=ROWS)
    ap.add_argument("--pattern", default="special.*requests")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-c4", action="store_true")
    ap.add_argument("--c4-rows", type=int, default=ROWS, help="C4 rows per row group")
    ap.add_argument("--c4-rows-per-gpu", type=int, default=12_500_000, help="C4: 100M rows / 8 GPUs")
    ap.add_argument("--cpu-seconds", type=float, default=5.0, help="per CPU-baseline sample")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0: the box's CPU share (<= 16)")
    ap.add_argument("--no-c5", action="store_true")
    ap.add_argument("--c5-rgs", type=int, default=12, help="C5 row groups of 10M rows per GPU (1B rows / 8 GPUs = 12.5)")
    ap.add_argument("--c5-pattern", default=C5_PATTERN)
    ap.add_argument("--no-c5-ref", action="store_true", help="skip C5 in the reference writer's layout")
    ap.add_argument("--c5-streams", type=int, default=2,
                    help="contexts (HIP streams) the C5 row groups alternate over: one row group's "
                         "run/code kernels overlap another's write pass")
    ap.add_argument("--no-validate", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--no-wide", action="store_true", help="skip the 100k-entry dictionary leg")
    ap.add_argument("--no-ext", action="store_true", help="skip the compressed / DATA_PAGE_V2 leg (SURVEY §8f rank 4)")
    ap.add_argument("--cpu-only", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo: rehearse N ranks on fewer GPUs (control path only; the data path has no collective)")
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "pmc_latest.json"))
    ap.add_argument("--full-json", default=os.path.join(ROOT, "gpurun_out", "bench_full.json"),
                    help="every leg's full record goes here; stdout gets the compact headline line")
    ap.add_argument("--opt", action="append", default=[],
                    help="context option key=value set before any upload (repeatable), e.g. write_waves=8")
    return ap.parse_args()


# ── launch ────────────────────────────────────────────────────────────────
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def maybe_spawn(args):
    """--gpus N without a launcher: start N ranks as CHILD processes (one per
    GPU, torch.distributed.run) and exit with their status.  Nothing here has
    touched the GPU yet."""
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        env = dict(os.environ)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
        sys.exit(subprocess.call(cmd, env=env))


# ── measurement plumbing ──────────────────────────────────────────────────
class Job:
    def __init__(self, rank, world, local, dist, ctx):
        self.rank, self.world, self.local, self.dist, self.ctx = rank, world, local, dist, ctx

    def barrier(self):
        import torch
        if self.dist is not None:
            self.dist.barrier()
        torch.cuda.synchronize()
        self.ctx.sync()

    def _reduce(self, xs, op):
        if self.dist is None:
            return list(xs)
        import torch
        dev = "cpu" if self.dist.get_backend() == "gloo" else f"cuda:{self.local}"
        t = torch.tensor(list(xs), dtype=torch.float64, device=dev)
        self.dist.all_reduce(t, op=op)
        return t.tolist()

    def max_all(self, xs):
        return self._reduce(xs, self.dist.ReduceOp.MAX if self.dist else None)

    def sum_all(self, xs):
        return self._reduce(xs, self.dist.ReduceOp.SUM if self.dist else None)

    def gather(self, obj):
        if self.dist is None:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def timed(self, step, check, steps, repeats, warmup=0, kernels=KERNELS):
        """`repeats` regions of exactly `steps` steps, each bracketed by a
        barrier + sync; seconds per region (max over ranks), then the same
        steps once more with per-kernel HIP events (events perturb the wall
        clock, so they stay outside the timed regions)."""
        import torch
        for _ in range(warmup):
            step()
        self.ctx.sync()
        check()
        secs = []
        for _ in range(repeats):
            self.barrier()
            t0 = time.perf_counter()
            for _ in range(steps):
                step()
            self.ctx.sync()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            self.barrier()
            secs.append(t1 - t0)
        check()
        secs = self.max_all(secs)
        self.ctx.timing(True)
        self.ctx.timing_reset()
        for _ in range(steps):
            step()
        self.ctx.sync()
        self.ctx.timing(False)
        check()
        kern = {}
        for name in kernels:
            ms, n = self.ctx.timing_get(name)
            if n:
                kern[name] = {"ms_per_launch": ms / n, "ms_per_step": ms / steps, "launches_per_step": n / steps}
        return secs, kern


def kernel_source_hash() -> str:
    """sha256 over the sources of the C2 pipe kernels a PMC summary measures
    (dict_pipe.hip and every header it includes, recursively): the summary's
    traffic figure applies to a run only when these are unchanged."""
    import re
    h = hashlib.sha256()
    base = os.path.join(PKG, "csrc")
    seen, todo = set(), ["kernels/dict_pipe.hip"]
    while todo:
        rel = todo.pop()
        if rel in seen:
            continue
        seen.add(rel)
        path = os.path.join(base, rel) if os.path.exists(os.path.join(base, rel)) else os.path.join(ROOT, "include", rel)
        if not os.path.exists(path):
            continue
        with open(path, "rb") as fh:
            src = fh.read()
        for inc in re.findall(rb'#include "([^"]+)"', src):
            todo.append(inc.decode())
    for rel in sorted(seen):
        for path in (os.path.join(base, rel), os.path.join(ROOT, "include", rel)):
            if os.path.exists(path):
                with open(path, "rb") as fh:
                    h.update(rel.encode())
                    h.update(fh.read())
                break
    return h.hexdigest()[:16]


def pmc_traffic(path: str, kernel: str):
    """HBM bytes per launch of `kernel` from a rocprofv3 --pmc summary
    (scripts/pmc_summary.py: separate FETCH_SIZE / WRITE_SIZE passes,
    corrected per MI355X_MICROARCH.md), used only when it was taken on these
    same kernel sources; else None."""
    if not path or not os.path.exists(path):
        return None, "no PMC summary"
    with open(path) as fh:
        d = json.load(fh)
    if d.get("kernel_src_sha") != kernel_source_hash():
        return None, f"PMC summary {d.get('source')} was taken on other kernel sources"
    k = d.get("kernels", {}).get(kernel)
    return (k.get("hbm_bytes_per_launch") if k else None), d.get("source")


def pmc_step_traffic(path: str, kern: dict):
    """HBM bytes of one whole step: each step kernel's PMC bytes per launch
    (a C2-only PMC summary, scripts/gpu_pmc_c2.sh) x its launches per step
    (the bench's own HIP-event timers); None unless every timed kernel of
    the step has a PMC figure taken on these kernel sources."""
    if not path or not os.path.exists(path):
        return None
    with open(path) as fh:
        d = json.load(fh)
    if d.get("kernel_src_sha") != kernel_source_hash():
        return None
    pk = d.get("kernels", {})
    total, parts = 0.0, {}
    for name, v in kern.items():
        e = next((pk[c] for c in (name, name + "3", name.replace("pipe_codes", "pipe_codes3")) if c in pk), None)
        if not e or "hbm_bytes_per_launch" not in e:
            return None
        parts[name] = e["hbm_bytes_per_launch"] * v["launches_per_step"]
        total += parts[name]
    return {"bytes": total, "per_kernel": parts, "source": d.get("source")}


def sha(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


def expectations():
    p = os.path.join(ROOT, "tests", "golden", "bench_expect.json")
    if os.path.exists(p):
        with open(p) as fh:
            return json.load(fh)
    return {}


def cpu_share(args) -> int:
    if args.cpu_threads > 0:
        return args.cpu_threads
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


# ── CPU baselines (rank 0, N=1; run before anything touches the GPU) ─────
def _regex_pages_cpu_worker(job):
    """Oracle decode (C) of a page range + Python `re` per value (the R-REGEX
    contract): reported flag per page."""
    import re

    import numpy as np
    from oracle import oracle as O
    sub, desc, pattern, first_rows, counts = job
    rc, msg, col = O.read_all(sub, desc)
    assert rc == 0, msg
    valid = np.asarray(col.valid)
    off = np.asarray(col.offsets)
    data = bytes(col.data)
    rx = re.compile(pattern, re.ASCII)
    flags = []
    r = 0
    for n in counts:
        rep = 1
        for i in range(r, r + n):
            if valid[i] and rx.search(data[off[i]:off[i + 1]].decode("utf-8", "surrogateescape")):
                rep = 0
                break
        flags.append(rep)
        r += n
    return flags


def cpu_baselines(args):
    from oracle import oracle as O
    from pqgpu import capi, gen
    from pqgpu.shard import data_page_ranges, extract_range
    threads = cpu_share(args)
    out = {"host_cpu": _cpu_model(), "cores_used": threads,
           "cores_note": "threads = min(16, sched_getaffinity): the box's CPU share for one GPU"}
    if not O.have_ref():
        return None
    layout = gen.REF_LAYOUT if args.layout == "ref" else gen.ARROW_LAYOUT
    rows = 1_000_000
    f = gen.build(gen.c2_cols(), rows, 1, seed=gen.CONFIG_SEEDS["C2"], layout=layout)
    ch = capi.File(f).chunk(0, 0)
    def ochunk(d):
        return O.Chunk(d.num_values, d.data_page_offset,
                       d.dictionary_page_offset if d.has_dictionary_page_offset else None, d.codec, d.type,
                       d.max_def_level, d.max_rep_level)
    och = ochunk(ch)

    def reps_for(fn):
        s, _ = fn(1)
        return max(1, int(args.cpu_seconds / max(s, 1e-3)))

    one = lambda reps: O.ref_time_read_all(f, och, reps=reps, threads=1)  # noqa: E731
    reps = reps_for(one)
    s, nv = one(reps)
    out["single_thread"] = {"value": nv / s, "unit": "values/s", "cores": 1, "seconds": s,
                            "sample": f"{reps} x ColumnReader::read_all of a {rows}-row C2 chunk"}
    chunkp = lambda reps: O.ref_time_read_all(f, och, reps=reps, threads=threads)  # noqa: E731
    reps = reps_for(chunkp)
    s, nv = chunkp(reps)
    out["chunk_parallel"] = {"value": nv / s, "unit": "values/s", "cores": threads, "seconds": s,
                             "sample": f"{threads} ColumnReaders x {reps} reads of the {rows}-row C2 chunk "
                                       "(one reader per chunk: the reference API's parallelism)"}
    rc, msg, table = capi.build_page_table(f, ch)
    shards = []
    for a, b in data_page_ranges(table, 4 * threads):
        sub, d = extract_range(f, ch, table, a, b)
        shards.append((sub, ochunk(d)))
    pagep = lambda reps: O.ref_time_read_all_multi(shards, ch.type, ch.max_def_level, ch.max_rep_level,  # noqa: E731
                                                   reps=reps, threads=threads)
    reps = reps_for(pagep)
    s, nv = pagep(reps)
    out["page_parallel"] = {"value": nv / s, "unit": "values/s", "cores": threads, "seconds": s,
                            "sample": f"the {rows}-row C2 chunk as {len(shards)} page-range shards "
                                      f"(dictionary replicated), {threads} threads, {reps} rounds"}
    # regex: oracle decode + Python re (RE2 is absent on the box), page-parallel processes
    rrows = 2_000_000
    rf = gen.build(gen.c3_cols(), rrows, 1, seed=gen.CONFIG_SEEDS["C3"])
    rch = capi.File(rf).chunk(0, 0)
    rc, msg, rtable = capi.build_page_table(rf, rch)
    jobs = []
    for a, b in data_page_ranges(rtable, 4 * threads):
        sub, d = extract_range(rf, rch, rtable, a, b)
        dp = [p for p in rtable if p.page_type == 0][a:b]
        jobs.append((sub, ochunk(d), args.pattern, [p.first_row for p in dp],
                     [p.num_values for p in dp]))
    # native: the reference's ColumnReader::read_all per page-range shard,
    # values tested with the build's host DFA (regex_host.cpp, the table
    # k_regex_plain walks), page-parallel on `threads` threads, at C3's full size
    nrows_n = args.regex_rows
    nf = gen.build(gen.c3_cols(), nrows_n, 1, seed=gen.CONFIG_SEEDS["C3"])
    nch = capi.File(nf).chunk(0, 0)
    rc, msg, ntable = capi.build_page_table(nf, nch)
    ndata = [p for p in ntable if p.page_type == 0]
    nshards, ncounts = [], []
    for a, b in data_page_ranges(ntable, 8 * threads):
        sub, d = extract_range(nf, nch, ntable, a, b)
        nshards.append((sub, ochunk(d)))
        ncounts.append([p.num_values for p in ndata[a:b]])
    del nf
    nat = {}
    for neg in (False, True):
        run = lambda reps: O.ref_time_regex_pages_multi(nshards, nch.type, nch.max_def_level,  # noqa: E731
                                                        nch.max_rep_level, ncounts, args.pattern, neg,
                                                        reps=reps, threads=threads)
        s1, _ = run(1)
        reps = max(1, int(args.cpu_seconds / max(s1, 1e-3)))
        s, fl = run(reps)
        nat["neg" if neg else "pos"] = {"value": len(ndata) * reps / s, "unit": "pages/s", "seconds": s,
                                        "reps": reps, "reported_pages": int(fl.sum())}
    out["regex_native"] = {**nat["pos"], "cores": threads, "kind": "reference",
                           "neg": nat["neg"],
                           "sample": f"C3 {nrows_n} rows ({len(ndata)} pages), pattern {args.pattern!r}: the "
                                     "reference ColumnReader::read_all (oracle/_ref) per page-range shard, "
                                     "values tested with the build's host DFA (regex_host.cpp) until one "
                                     f"satisfies the predicate, {threads} threads"}
    del nshards
    import multiprocessing as mp
    with mp.get_context("fork").Pool(threads) as pool:
        t0 = time.perf_counter()
        flags = sum(pool.map(_regex_pages_cpu_worker, jobs, chunksize=1), [])
        s = time.perf_counter() - t0
    out["regex"] = {"value": len(flags) / s, "unit": "pages/s", "cores": threads, "seconds": s, "kind": "port",
                    "sample": f"C3 {rrows} rows ({len(flags)} pages), pattern {args.pattern!r}: oracle decode "
                              "+ Python re.search per value, page-range shards on a process pool",
                    "reported_pages": int(sum(flags))}
    return out


# ── legs ──────────────────────────────────────────────────────────────────
def c2_leg(J, args, exp):
    """The headline: the (N x rows)-row C2 column as N row groups, one per
    rank (the global page order cut at row-group boundaries); every rank
    generates, decodes and validates only its own row group (first_rg=rank)."""
    from pqgpu import capi, gen
    layout = gen.REF_LAYOUT if args.layout == "ref" else gen.ARROW_LAYOUT
    t0 = time.perf_counter()
    f = gen.build(gen.c2_cols(), args.rows, 1, seed=gen.CONFIG_SEEDS["C2"], layout=layout, first_rg=J.rank)
    gen_s = time.perf_counter() - t0
    ch = capi.File(f).chunk(0, 0)
    t0 = time.perf_counter()
    rc, msg, table = capi.build_page_table(f, ch)
    walk_s = time.perf_counter() - t0
    assert rc == 0, msg
    t0 = time.perf_counter()
    dc = J.ctx.upload(f, [ch])
    upload_s = time.perf_counter() - t0
    dc.decode()
    nrows = dc.num_rows
    host = dc.to_host()
    nonnull = int(host.validity.sum())
    chars = int(dc.out.num_bytes)
    valid = None
    want = None
    if not args.no_validate:
        # this rank's row group against the generator's dump of it
        want = sha(gen.values_dump(gen.c2_cols()[0], 0, args.rows, J.rank, gen.CONFIG_SEEDS["C2"]))
        ok = sha(capi.canonical_dump(host)) == want
        valid = all(J.gather(bool(ok)))
    del host
    secs, kern = J.timed(dc.decode_async, dc.decode_check, args.steps, args.repeats, warmup=args.warmup)
    rows_all = J.sum_all([nrows])[0]
    med = statistics.median(secs)
    res = {"secs": secs, "median_s": med, "value": rows_all * args.steps / med, "nrows": nrows,
           "rows_all": rows_all, "nonnull": nonnull, "chars": chars, "payload": dc.payload_bytes,
           "pages": dc.num_pages, "kern": kern, "validated": valid, "row_group": J.rank,
           "gen_s": gen_s}
    if not args.no_e2e and J.rank == 0:
        # end to end from host file bytes: host page walk + image build + H2D
        # (+ allocation) + one decode, each the median of 3 (reported
        # separately from the device-resident rate)
        payload = dc.payload_bytes
        dc.free()

        def e2e_runs(device_walk: int):
            w, u, d = [], [], []
            J.ctx.set_option("device_walk", device_walk)
            J.ctx.timing(True)
            J.ctx.timing_reset()
            for _ in range(3):
                t0 = t1 = time.perf_counter()
                x = J.ctx.upload(f, [ch])  # pq_chunk_upload walks the chunk itself
                t2 = time.perf_counter()
                x.decode()
                t3 = time.perf_counter()
                x.free()
                w.append(t1 - t0), u.append(t2 - t1), d.append(t3 - t2)
            J.ctx.timing(False)
            J.ctx.set_option("device_walk", 0)
            phases = upload_phases(J.ctx, 3)
            wk = J.ctx.timing_get("walk")
            if wk[1]:
                phases["walk_kernels"] = {"ms": wk[0] / 3, "calls_per_upload": wk[1] / 3}
            return statistics.median(w), statistics.median(u), statistics.median(d), phases

        wm, um, dm, phases = e2e_runs(0)
        res["e2e"] = {"table_ms": wm * 1e3, "upload_ms": um * 1e3, "first_decode_ms": dm * 1e3,
                      "total_ms": (wm + um + dm) * 1e3, "values_per_s": nrows / (wm + um + dm),
                      "file_bytes": len(f), "upload_phases": phases,
                      "note": "from host file bytes: upload (walk, planning, allocation, "
                              "pinned H2D of the raw chunk bytes overlapped with the walk, GPU relayout) + first decode "
                              "(includes output allocation)"}
        wm, um, dm, phases = e2e_runs(1)
        res["e2e"]["device_walk"] = {
            "upload_ms": um * 1e3, "first_decode_ms": dm * 1e3, "total_ms": (wm + um + dm) * 1e3,
            "values_per_s": nrows / (wm + um + dm), "upload_phases": phases,
            "note": "option device_walk: the page walk runs on the GPU (walk.hip) once the raw chunk bytes are in HBM "
                    "(up_walk then covers the H2D wait, the walk kernels and the page table's copy back)"}
    else:
        dc.free()
    res["walk_s"] = walk_s
    res["upload_s"] = upload_s
    if not args.no_e2e and J.rank == 0:
        res["api_read_all"] = api_read_all_leg(f, want)
        # the same call on cpu_baseline's 1M-row chunk (like for like with its
        # page_parallel / chunk_parallel rates)
        from pqgpu import gen as _gen
        layout = _gen.REF_LAYOUT if args.layout == "ref" else _gen.ARROW_LAYOUT
        f1 = _gen.build(_gen.c2_cols(), 1_000_000, 1, seed=_gen.CONFIG_SEEDS["C2"], layout=layout)
        want1 = sha(_gen.values_dump(_gen.c2_cols()[0], 0, 1_000_000, 0, _gen.CONFIG_SEEDS["C2"]))
        res["api_read_all"]["chunk_1m"] = api_read_all_leg(f1, want1, reps=9)
    del f
    return res


def api_read_all_leg(f: bytes, want, reps: int = 5):
    """What a drop-in caller of the reference API gets (the
    std::vector<Value> path): pqgpu::ColumnReader::read_all on the C2 chunk,
    host file bytes in, std::vector<Value> out (range read, upload, decode,
    copy-out, the Value build on up to 16 host threads), timed in the C++ tool
    (tools/api_check.cpp time_read_all, median of 3 after a warm-up), its
    values checked against the generator's dump."""
    import tempfile
    tool = os.path.join(ROOT, "duckdb-parquet-parser_amd", "pqgpu", "api_check")
    with tempfile.TemporaryDirectory() as td:
        path, dump = os.path.join(td, "c2.parquet"), os.path.join(td, "c2.dump")
        with open(path, "wb") as fh:
            fh.write(f)
        r = subprocess.run([tool, path, "time_read_all", "0", "0", str(reps), dump], stdout=subprocess.PIPE,
                           stderr=subprocess.PIPE, timeout=600)
        if r.returncode != 0:
            return {"error": r.stderr.decode(errors="replace")[-500:]}
        js = json.loads(r.stdout.decode().strip().splitlines()[-1])
        with open(dump, "rb") as fh:
            got = hashlib.sha256(fh.read()).hexdigest()
    n = js["values"]
    return {"values_per_s": n / (js["read_all_ms"] * 1e-3), "read_all_ms": js["read_all_ms"],
            "read_columnar_ms": js["read_columnar_ms"], "to_values_ms": js["to_values_ms"],
            "to_values_per_s": n / (js["to_values_ms"] * 1e-3), "threads": js["threads"], "values": n,
            "read_all_samples_ms": js.get("read_all_samples"), "to_values_samples_ms": js.get("to_values_samples"),
            "phases_ms": js.get("phases_ms"),
            "validated": (got == want) if want else None,
            "note": "ColumnReader::read_all from host file bytes to std::vector<Value>; compare cpu_baseline."
                    "chunk_parallel (the reference's read_all, one thread per chunk) and single_thread"}


def strong_leg(J, args):
    """Strong scaling: the 10M-row C2 chunk split into N page ranges."""
    from pqgpu import capi, gen
    from pqgpu.shard import data_page_ranges
    layout = gen.REF_LAYOUT if args.layout == "ref" else gen.ARROW_LAYOUT
    f = gen.build(gen.c2_cols(), args.rows, 1, seed=gen.CONFIG_SEEDS["C2"], layout=layout)
    ch = capi.File(f).chunk(0, 0)
    rc, msg, table = capi.build_page_table(f, ch)
    a, b = data_page_ranges(table, J.world)[J.rank]
    dc = J.ctx.upload_range(f, ch, table, a, b)
    dc.decode()
    valid = None
    if not args.no_validate:
        # this shard's dump sits in the whole column's dump after the shards before it
        mine = capi.canonical_dump(dc.to_host())
        sizes = J.gather(len(mine))
        start = sum(sizes[:J.rank])
        whole = gen.values_dump(gen.c2_cols()[0], 0, args.rows, 0, gen.CONFIG_SEEDS["C2"])
        ok = whole[start:start + len(mine)] == mine and (J.rank != J.world - 1 or start + len(mine) == len(whole))
        valid = all(J.gather(bool(ok)))
        del whole, mine
    secs, kern = J.timed(dc.decode_async, dc.decode_check, args.steps, args.repeats, warmup=args.warmup)
    dc.free()
    med = statistics.median(secs)
    return {"rows_total": args.rows, "ms_per_step": med / args.steps * 1e3, "page_range_rank0": J.gather([a, b])[0],
            "values_per_s": args.rows * args.steps / med, "scaling": "strong", "validated": valid}


def c3_legs(J, args, exp):
    from pqgpu import capi, gen
    rows = args.regex_rows
    rfile = gen.build(gen.c3_cols(), rows, 1, seed=gen.CONFIG_SEEDS["C3"], first_rg=J.rank)
    RF = capi.File(rfile)
    rch = RF.chunk(0, 0)
    rdc = J.ctx.upload(rfile, [rch])
    flags = rdc.regex_pages(args.pattern)
    rsteps = max(3, args.steps // 2)
    step = lambda: rdc.regex_pages_async(args.pattern)  # noqa: E731
    npages = rdc.num_pages

    def scan_stats(secs, kern):
        med = statistics.median(secs)
        k = next((k for k in ("regex_plain", "regex_lanes", "regex_pages") if k in kern), None)
        kms = kern[k]["ms_per_launch"] if k else None
        return {"pages_per_s": npages * rsteps * J.world / med, "ms_per_scan": med / rsteps * 1e3,
                "repeats_ms": [x / rsteps * 1e3 for x in secs], "kernel": k, "kernel_ms": kms,
                "payload_GBs": rdc.payload_bytes / (kms * 1e-3) / 1e9 if kms else None,
                "roofline_frac": rdc.payload_bytes / (kms * 1e-3) / 1e9 / HBM_PEAK_GBS if kms else None}
    # the metric: a cold single scan, what --regex-column does once per file:
    # option regex_index=2 makes every timed scan a first scan (walk the
    # length chains and file the chunk's string index again)
    J.ctx.set_option("regex_index", 2)
    try:
        cold = scan_stats(*J.timed(step, rdc.regex_pages_result, rsteps, args.repeats, warmup=max(1, args.warmup // 2),
                                   kernels=REGEX_KERNELS))
    finally:
        J.ctx.set_option("regex_index", 1)
    # warm: repeat scans of the same chunk read the index the first scan filed
    secs, kern = J.timed(step, rdc.regex_pages_result, rsteps, args.repeats, warmup=max(1, args.warmup // 2),
                         kernels=REGEX_KERNELS)
    warm = scan_stats(secs, kern)

    def check(fl, pat, neg):
        e = exp.get(f"c3|{rows}|rg{J.rank}|{pat}|{int(neg)}")
        ok = (sha(fl.astype("u1").tobytes()) == e["sha256"]) if e else None
        oks = J.gather(ok)
        return None if any(o is None for o in oks) else all(oks)

    regex = {**cold, "scan": "cold: every timed scan is a first scan (regex_index=2: chain walk + index filed)",
             "pages_per_gpu": npages, "pattern": args.pattern, "reported_pages": int(flags.sum()),
             "validated": check(flags, args.pattern, False),
             "warm": {**warm, "scan": "warm: repeat scans read the string index the first scan filed"}}
    if not args.no_e2e and J.rank == 0:
        u, r = [], []
        J.ctx.timing(True)
        J.ctx.timing_reset()
        for _ in range(3):
            t1 = time.perf_counter()
            x = J.ctx.upload(rfile, [rch])
            t2 = time.perf_counter()
            x.regex_pages(args.pattern)
            t3 = time.perf_counter()
            x.free()
            u.append(t2 - t1), r.append(t3 - t2)
        J.ctx.timing(False)
        phases = upload_phases(J.ctx, 3)
        um, rm = statistics.median(u), statistics.median(r)
        regex["e2e"] = {"upload_ms": um * 1e3, "first_scan_ms": rm * 1e3, "total_ms": (um + rm) * 1e3,
                        "pages_per_s": npages / (um + rm), "upload_phases": phases,
                        "payload_bytes": rdc.payload_bytes,
                        "note": "from host file bytes: pq_chunk_upload (speculative page walk, device planning, "
                                "allocation, pinned multi-buffered H2D) + one regex scan incl. pattern compile"}
    # the four patterns, each with and without --neg-regex,
    # timed and checked against the oracle's page sets (make_bench_expect.py)
    sweep = {}
    for pat in C3_PATTERNS:
        for neg in (False, True):
            fl = rdc.regex_pages(pat, neg)
            st = lambda p=pat, n=neg: rdc.regex_pages_async(p, n)  # noqa: E731
            J.ctx.set_option("regex_index", 2)  # cold scans first, then warm (see above)
            try:
                c = scan_stats(*J.timed(st, rdc.regex_pages_result, rsteps, 3, warmup=1, kernels=REGEX_KERNELS))
            finally:
                J.ctx.set_option("regex_index", 1)
            w = scan_stats(*J.timed(st, rdc.regex_pages_result, rsteps, 3, warmup=1, kernels=REGEX_KERNELS))
            sweep[f"{pat}{' (neg)' if neg else ''}"] = {
                "pages_per_s": c["pages_per_s"], "ms_per_scan": c["ms_per_scan"], "kernel": c["kernel"],
                "kernel_ms": c["kernel_ms"], "roofline_frac": c["roofline_frac"],
                "warm": {k: w[k] for k in ("pages_per_s", "ms_per_scan", "kernel", "kernel_ms", "roofline_frac")},
                "reported_pages": int(fl.sum()), "validated": check(fl, pat, neg)}
    regex["patterns"] = sweep
    regex["all_validated"] = all(v["validated"] for v in sweep.values()) and bool(regex["validated"])
    # C3 PLAIN decode on the same upload
    dsteps = max(3, args.steps // 2)
    rdc.decode()
    ok = None
    if not args.no_validate:
        ok = sha(capi.canonical_dump(rdc.to_host())) == sha(
            gen.values_dump(gen.c3_cols()[0], 0, rows, J.rank, gen.CONFIG_SEEDS["C3"]))
    secs, dkern = J.timed(rdc.decode_async, rdc.decode_check, dsteps, args.repeats, warmup=2)
    med = statistics.median(secs)
    c3d = {"ms_per_decode": med / dsteps * 1e3, "values_per_s": rows * dsteps * J.world / med,
           "payload_bytes": rdc.payload_bytes, "kernel_ms": {k: v["ms_per_step"] for k, v in dkern.items()},
           "validated": ok}
    # the example driver's 4 KiB chunker over the decoded column (main.cpp:17-32)
    rdc.decode()
    ct = []
    for _ in range(3):
        t0 = time.perf_counter()
        ids, nchunks = rdc.chunk_assign(4096)
        ct.append(time.perf_counter() - t0)
    c3d["chunker"] = {"ms": statistics.median(ct) * 1e3, "chunks": nchunks,
                      "note": "pq_chunk_assign incl. the tuple_to_chunk copy to host (80 MB)"}
    rdc.free()
    # the same strings OPTIONAL with 5 % NULLs in 20,000-row pages (the shape
    # pyarrow writes by default): levels, then the value sections on the
    # PLAIN kernels
    ocol = gen.Col("comment", gen.COMMENT, gen.BYTE_ARRAY, optional=True, null_frac=0.05, len_min=10, len_max=44)
    ofile = gen.build([ocol], rows, 1, seed=gen.CONFIG_SEEDS["C3"], layout=gen.ARROW_LAYOUT, first_rg=J.rank)
    OF = capi.File(ofile)
    odc = J.ctx.upload(ofile, [OF.chunk(0, 0)])
    odc.decode()
    ok = None
    if not args.no_validate:
        ok = sha(capi.canonical_dump(odc.to_host())) == sha(gen.values_dump(ocol, 0, rows, J.rank, gen.CONFIG_SEEDS["C3"]))
    secs, okern = J.timed(odc.decode_async, odc.decode_check, dsteps, args.repeats, warmup=2)
    med = statistics.median(secs)
    c3d["optional_arrow"] = {"ms_per_decode": med / dsteps * 1e3, "values_per_s": rows * dsteps * J.world / med,
                             "pages": odc.num_pages, "null_frac": 0.05,
                             "kernel_ms": {k: v["ms_per_step"] for k, v in okern.items()}, "validated": ok}
    odc.free()
    return regex, c3d


def _rows_slice(h, r0: int, r1: int):
    """Rows [r0, r1) of a host column (offsets rebased)."""
    from pqgpu import capi
    if h.offsets is not None:
        o = h.offsets[r0:r1 + 1]
        return capi.HostColumn(h.type, h.validity[r0:r1], h.data[o[0]:o[-1]], o - o[0])
    w = len(h.data) // max(h.num_rows, 1)
    return capi.HostColumn(h.type, h.validity[r0:r1], h.data[r0 * w:r1 * w], None)


def _piece_alg_bytes(p, optional: bool) -> int:
    """SURVEY §8(d) algorithmic bytes of one decoded device chunk: its page
    payloads, its values (BYTE_ARRAY: 8(n+1) offsets + chars; else n x width)
    and, for OPTIONAL columns, its validity bitmap."""
    from pqgpu import capi
    n = p.num_rows
    o = p.out
    vals = o.num_bytes + (8 * (n + 1) if o.type == capi.BYTE_ARRAY else 0)
    return p.payload_bytes + vals + ((n + 7) // 8 if optional else 0)


def c4_leg(J, args):
    """the 8-column mixed file at --c4-rows-per-gpu x N rows
    (100M at N = 8) in row groups of --c4-rows rows, data pages sharded across
    the ranks: rank r owns the pages whose first row falls in its row range
    (shard.row_page_range; ranges cross row-group boundaries), generates only
    the row groups those pages live in and uploads each column's pages with
    pq_chunk_upload_range.  Validation: every touched row group decoded whole
    against the generator's dump, and every shard against its rows of that."""
    from pqgpu import capi, gen
    from pqgpu.shard import row_page_range
    cols = gen.c4_cols()
    seed = gen.CONFIG_SEEDS["C4"]
    rg_rows, per_gpu = args.c4_rows, args.c4_rows_per_gpu
    total = per_gpu * J.world
    lo, hi = per_gpu * J.rank, per_gpu * (J.rank + 1)
    ctxs = [J.ctx] + [capi.Context(J.local) for _ in range(max(1, args.c5_streams) - 1)]
    pieces = {ci: [] for ci in range(len(cols))}  # column -> its shard pieces (device chunks)
    ok = True
    nrg = 0
    for g in range(lo // rg_rows, (hi - 1) // rg_rows + 1):
        n_g = min(rg_rows, total - g * rg_rows)
        f = gen.build(cols, n_g, 1, seed=seed, layout=gen.ARROW_LAYOUT, first_rg=g)
        F = capi.File(f)
        nrg += 1
        for ci, col in enumerate(cols):
            ch = F.chunk(0, ci)
            rc, msg, table = capi.build_page_table(f, ch)
            assert rc == 0, msg
            a, b = row_page_range(table, g * rg_rows, lo, hi)
            if a == b:
                continue
            dc = ctxs[ci % len(ctxs)].upload_range(f, ch, table, a, b)
            dc.decode()
            if not args.no_validate:
                whole = J.ctx.upload(f, [ch])
                whole.decode()
                h = whole.to_host()
                whole.free()
                ok &= sha(capi.canonical_dump(h)) == sha(gen.values_dump(col, ci, n_g, g, seed))
                r0 = dc.first_row
                ok &= capi.canonical_dump(dc.to_host()) == capi.canonical_dump(_rows_slice(h, r0, r0 + dc.num_rows))
                del h
            pieces[ci].append(dc)
        del f, F
    steps = max(3, args.steps // 4)
    out, total_ms = {}, 0.0
    for ci, col in enumerate(cols):
        ps = pieces[ci]
        st = lambda ps=ps: [p.decode_async() for p in ps]  # noqa: E731
        ck = lambda ps=ps: [p.decode_check() for p in ps]  # noqa: E731
        secs, kern = J.timed(st, ck, steps, args.repeats, warmup=2)
        ms = statistics.median(secs) / steps * 1e3
        # SURVEY §8(d) C4 algorithmic bytes of the column's shard: page payloads
        # in; values (fixed width: n x width; strings: 8(n+1) offsets + chars)
        # and the validity bitmap (OPTIONAL columns) out
        b_alg = sum(_piece_alg_bytes(p, col.optional) for p in ps)
        gbs = b_alg / (ms * 1e-3) / 1e9
        out[col.name] = {"ms": ms, "pieces": len(ps), "kernels_ms": {k: v["ms_per_step"] for k, v in kern.items()},
                         "roofline": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                      "frac": gbs / HBM_PEAK_GBS, "algorithmic_bytes": b_alg}}
        total_ms += ms
    # the rank's whole share: every column's pieces alternated over
    # --c5-streams contexts (HIP streams), all queued before any check, so
    # latency-bound kernels of one column overlap bandwidth-bound ones of another
    alld = [p for ci in pieces for p in pieces[ci]]

    def rg_step():
        for p in alld:
            p.decode_async()

    def rg_check():
        for p in alld:
            p.decode_check()

    secs, _ = J.timed(rg_step, rg_check, steps, args.repeats, warmup=2)
    nvals = sum(p.num_rows for p in alld)
    nvals_all = J.sum_all([nvals])[0]
    b_all = sum(_piece_alg_bytes(p, cols[ci].optional) for ci in pieces for p in pieces[ci])
    for p in alld:
        p.free()
    for c in ctxs[1:]:
        c.close()
    ms = statistics.median(secs) / steps * 1e3
    return {"values_per_s": nvals_all / (ms * 1e-3), "rows_per_gpu": nvals // len(cols), "row_groups_touched": nrg,
            "roofline": {"bound": "hbm", "achieved": b_all / (ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": b_all / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, "algorithmic_bytes": b_all,
                         "note": "the rank's whole share per step (all 8 columns), B_alg as SURVEY §8(d) C4"},
            "rows_total": total, "row_group_rows": rg_rows, "ms_per_step": ms, "streams": len(ctxs),
            "serial_ms": total_ms, "serial_values_per_s": nvals_all / (total_ms * 1e-3),
            "note": "values_per_s: the rank's page shards of all 8 columns decoded together over `streams` contexts "
                    "(max over ranks); serial_*: the sum of the columns timed one at a time (`columns`)",
            "columns": out, "layout": "arrow", "sharding": "data pages by global first row (row_page_range)",
            "validated": None if args.no_validate else all(J.gather(bool(ok)))}


UPLOAD_PHASES = ("up_walk", "up_plan", "up_plan_pages", "up_plan_fused", "up_plan_pipe", "up_plan_plain",
                 "up_plan_rest", "up_alloc", "up_h2d", "up_fill", "up_wait")
UPLOAD_PHASES_NOTE = ("host timers per upload (sum over the uploads / uploads): NOT additive and NOT parts of "
                      "upload_ms. up_walk, up_plan (with its up_plan_* parts) and up_alloc are wall times on the "
                      "calling thread; with the raw upload the chunk's bytes go to HBM from a side thread that starts "
                      "before the walk, so up_h2d (the H2D section, which also waits for that thread and copies the "
                      "page tables) overlaps up_walk and up_plan; up_fill is CPU time summed over the threads that "
                      "fill the pinned ring (several at once), up_wait the final wait for its DMA queues; "
                      "calls_per_upload > 1 means the section ran that often per upload")


def upload_phases(ctx, uploads: int) -> dict:
    out = {"note": UPLOAD_PHASES_NOTE}
    for k in UPLOAD_PHASES:
        ms, calls = ctx.timing_get(k)
        if calls:
            out[k] = {"ms": ms / uploads, "calls_per_upload": calls / uploads}
    return out


def wide_dict_leg(J, args):
    """the C2 column shape with a 100,000-entry dictionary
    (1.0 MB dictionary page: pyarrow's 1 MiB dictionary_pagesize_limit,
    17-bit indices, 20,000-row pages), 10M rows per rank (row group = rank).
    Decode timed and checked against the generator's dump; roofline on the
    whole step's algorithmic bytes (payload in, column out)."""
    from pqgpu import capi, gen
    col = gen.Col("s", gen.DICT_STRINGS, gen.BYTE_ARRAY, optional=True, null_frac=0.05, dict_size=100_000,
                  len_min=4, len_max=9, max_run=16)
    rows = args.rows
    f = gen.build([col], rows, 1, seed=gen.CONFIG_SEEDS["C2"], layout=gen.ARROW_LAYOUT, first_rg=J.rank)
    ch = capi.File(f).chunk(0, 0)
    dc = J.ctx.upload(f, [ch])
    del f
    dc.decode()
    h = dc.to_host()
    ok = None
    if not args.no_validate:
        ok = sha(capi.canonical_dump(h)) == sha(gen.values_dump(col, 0, rows, J.rank, gen.CONFIG_SEEDS["C2"]))
        ok = all(J.gather(bool(ok)))
    out_bytes = 8 * (rows + 1) + int(h.offsets[-1]) + (rows + 7) // 8
    del h
    steps = max(3, args.steps // 2)
    secs, kern = J.timed(dc.decode_async, dc.decode_check, steps, args.repeats, warmup=2)
    med = statistics.median(secs) / steps
    b_alg = dc.payload_bytes + out_bytes
    res = {"rows_per_gpu": rows, "dict_entries": 100_000, "dict_page_bytes": None, "pages": dc.num_pages,
           "ms_per_decode": med * 1e3, "values_per_s": rows * J.world / med,
           "b_alg_bytes": b_alg, "b_alg_GBs": b_alg / med / 1e9, "b_alg_frac_of_peak": b_alg / med / 1e9 / HBM_PEAK_GBS,
           "kernel_ms": {k: v["ms_per_step"] for k, v in kern.items()}, "validated": ok}
    pages = dc.pages()
    if pages:
        res["dict_page_bytes"] = int(pages[0].payload_size)
    dc.free()
    return res


def ext_leg(J, args):
    """SURVEY §8f rank 4 (outside the reference's scope): the C3 and C2
    columns as pyarrow writes them with SNAPPY (V1 pages), LZ4_RAW
    (DATA_PAGE_V2) and ZSTD (V1 pages, level 1), 1 MiB pages; upload with PQ_EXT_CODECS | PQ_EXT_PAGE_V2
    (the codec pass rebuilds every page on the GPU, codec.hip), then decode.
    Checked byte for byte against the uncompressed decode of the same column."""
    import io

    import numpy as np
    try:
        import pyarrow as pa
        import pyarrow.parquet as pq
    except ImportError:
        return {"skipped": "pyarrow not importable"}
    from pqgpu import capi, gen
    out = {}
    for name, cols, seed, use_dict, codec, ver in (("c3_snappy_v1", gen.c3_cols(), gen.CONFIG_SEEDS["C3"], False, "SNAPPY", "1.0"),
                                                   ("c2_lz4raw_v2", gen.c2_cols(), gen.CONFIG_SEEDS["C2"], True, "LZ4", "2.0"),
                                                   ("c3_zstd_v1", gen.c3_cols(), gen.CONFIG_SEEDS["C3"], False, "ZSTD", "1.0")):
        rows = args.rows
        f = gen.build(cols, rows, 1, seed=seed, first_rg=J.rank)
        dc = J.ctx.upload(f, [capi.File(f).chunk(0, 0)])
        dc.decode()
        h = dc.to_host()
        dc.free()
        ref = sha(capi.canonical_dump(h))
        valid = np.asarray(h.validity)
        arr = pa.LargeStringArray.from_buffers(
            h.num_rows, pa.py_buffer(np.asarray(h.offsets, np.int64).tobytes()),
            pa.py_buffer(np.asarray(h.data, np.uint8).tobytes()),
            pa.py_buffer(np.packbits(valid.astype(bool), bitorder="little").tobytes()),
            null_count=int(h.num_rows - valid.sum()))
        del h
        b = io.BytesIO()
        pq.write_table(pa.table({"s": arr}), b, compression=codec, data_page_version=ver, use_dictionary=use_dict,
                       row_group_size=rows)
        cf = b.getvalue()
        d = capi.File(cf).chunk(0, 0)
        d.ext_flags = capi.EXT_CODECS | capi.EXT_PAGE_V2
        up, ck = [], []
        for _ in range(3):
            J.ctx.timing(True)
            J.ctx.timing_reset()
            t0 = time.perf_counter()
            x = J.ctx.upload(cf, [d])
            up.append(time.perf_counter() - t0)
            J.ctx.sync()
            ck.append(J.ctx.timing_get("codec")[0])
            J.ctx.timing(False)
            x.free()
        x = J.ctx.upload(cf, [d])
        x.decode()
        ok = sha(capi.canonical_dump(x.to_host())) == ref
        steps = max(3, args.steps // 4)
        secs, kern = J.timed(x.decode_async, x.decode_check, steps, args.repeats, warmup=2)
        ub = x.payload_bytes
        x.free()
        kms = statistics.median(ck)
        out[name] = {"codec": codec, "page_version": ver, "rows": rows, "file_bytes": len(cf), "uncompressed_payload": ub,
                     "codec_kernel_ms": kms, "codec_GBs_out": ub / (kms * 1e-3) / 1e9 if kms else None,
                     "upload_ms": statistics.median(up) * 1e3, "decode_ms": statistics.median(secs) / steps * 1e3,
                     "validated": ok}
    return out


def c5_leg(J, args, exp, layout="arrow"):
    """C5 at --c5-rgs row groups of 10M rows per GPU: every row group is its
    own chunk (ColumnReader is per chunk; each has its own dictionary page).
    Decode all of them, then the regex page filter over all of them
    (dictionary-first: the pattern runs on each dictionary, then pages are
    tested through the codes of the decode that ran before it), then both as
    one step.  layout "ref": the reference writer's 512-row pages (~1.95M
    pages for the whole 1B rows)."""
    from pqgpu import capi, gen
    import numpy as np
    rows = 10_000_000
    rg0 = J.rank * args.c5_rgs
    f = gen.build(gen.c2_cols(), rows, args.c5_rgs, seed=gen.CONFIG_SEEDS["C5"],
                  layout=gen.ARROW_LAYOUT if layout == "arrow" else gen.REF_LAYOUT, first_rg=rg0)
    F = capi.File(f)
    # row groups are independent chunks: alternate them over contexts (one
    # HIP stream each) so latency-bound k_pipe_big of one overlaps the
    # bandwidth-bound k_pipe_write of another; the timed region ends with a
    # device-wide synchronize (torch.cuda.synchronize) covering every stream
    ctxs = [J.ctx] + [capi.Context(J.local) for _ in range(max(1, args.c5_streams) - 1)]
    dcs = [ctxs[rg % len(ctxs)].upload(f, [F.chunk(rg, 0)]) for rg in range(F.num_row_groups)]
    del f
    ok = True
    for i, dc in enumerate(dcs):
        dc.decode()
        if not args.no_validate:
            ok &= sha(capi.canonical_dump(dc.to_host())) == sha(
                gen.values_dump(gen.c2_cols()[0], 0, rows, rg0 + i, gen.CONFIG_SEEDS["C5"]))
        dc.regex_pages(args.c5_pattern)
    steps = max(2, args.steps // 4)

    def dec():
        for dc in dcs:
            dc.decode_async()

    def dec_check():
        for dc in dcs:
            dc.decode_check()

    def rx():
        for dc in dcs:
            dc.regex_pages_async(args.c5_pattern)

    def rx_check():
        for dc in dcs:
            dc.regex_pages_result()

    def both():  # decode + filter in one pass (pq_decode_regex_async)
        for dc in dcs:
            dc.decode_regex_async(args.c5_pattern)

    def both_check():
        for dc in dcs:
            dc.decode_check()
            dc.regex_pages_result()

    dsecs, dkern = J.timed(dec, dec_check, steps, args.repeats, warmup=1)
    rsecs, rkern = J.timed(rx, rx_check, steps, args.repeats, warmup=1, kernels=KERNELS + REGEX_KERNELS)
    bsecs, _ = J.timed(both, both_check, steps, args.repeats, warmup=1)
    dsec = statistics.median(dsecs) / steps
    rsec = statistics.median(rsecs) / steps
    bsec = statistics.median(bsecs) / steps
    nrows = sum(dc.num_rows for dc in dcs)
    npages = sum(dc.num_pages for dc in dcs)
    per_rg = [dc.regex_pages(args.c5_pattern) for dc in dcs]
    flags = np.concatenate(per_rg)
    one_pass = []
    for dc in dcs:
        dc.decode_regex_async(args.c5_pattern)
        dc.decode_check()
        one_pass.append(dc.regex_pages_result())
    same_one_pass = all(bool(np.array_equal(a, b)) for a, b in zip(one_pass, per_rg))
    key = "c5" if layout == "arrow" else "c5ref"
    es = [exp.get(f"{key}|{rows}|rg{rg0 + i}|{args.c5_pattern}") for i in range(len(dcs))]
    rx_ok = None if any(e is None for e in es) else all(
        sha(fl.astype("u1").tobytes()) == e["sha256"] for fl, e in zip(per_rg, es))
    rx_oks = J.gather(rx_ok)
    rx_ok = None if any(o is None for o in rx_oks) else all(rx_oks)
    for dc in dcs:
        dc.free()
    for c in ctxs[1:]:
        c.close()
    return {"rows_per_gpu": nrows, "row_groups_per_gpu": len(dcs), "pages_per_gpu": npages, "layout": layout,
            "streams": len(ctxs),
            "decode_values_per_s": nrows * J.world / dsec, "decode_ms": dsec * 1e3,
            "regex_pages_per_s": npages * J.world / rsec, "regex_ms": rsec * 1e3, "pattern": args.c5_pattern,
            "reported_pages": int(flags.sum()),
            "regex_validated": rx_ok, "one_pass_flags_equal": all(J.gather(same_one_pass)),
            "decode_validated": None if args.no_validate else all(J.gather(bool(ok))),
            "step_values_per_s": nrows * J.world / bsec, "step_ms": bsec * 1e3,
            "step_over_decode": bsec / dsec,
            "step_note": "decode + regex filter of every row group in one pass (pq_decode_regex_async: the pattern runs "
                         "once per dictionary entry, k_pipe_write tests each row's entry as it writes the column)",
            "kernel_ms_note": "HIP events of the first context's row groups only",
            "kernel_ms_per_step": {**{k: v["ms_per_step"] for k, v in dkern.items()},
                                   **{k: v["ms_per_step"] for k, v in rkern.items()}}}


HEADLINE_KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                 "scaling", "vs_baseline", "dtype", "data", "config", "validated")


def _r(x, nd=4):
    return None if x is None else float(f"{x:.{nd}g}")


def compact(res: dict, full_path: str) -> dict:
    """The stdout line: headline keys, roofline, cpu_baseline and one small
    summary per leg (value + roofline fraction).  Every leg's full record is
    in `full_path` (round 5's 20 KB line was past what the driver parses)."""
    out = {k: res[k] for k in HEADLINE_KEYS if k in res}
    rf = res["roofline"]
    out["roofline"] = {k: rf.get(k) for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel",
                                              "kernel_ms", "algorithmic_bytes", "step_traffic",
                                              "step_traffic_over_b_alg")}
    pl = res["pipeline"]
    out["pipeline"] = {"kernel_ms": {k: _r(v) for k, v in pl["kernel_ms"].items()},
                       "b_alg_bytes": pl["b_alg_bytes"], "b_alg_frac_of_peak": _r(pl["b_alg_frac_of_peak"])}
    if "cpu_baseline" in res:
        cb = res["cpu_baseline"]
        out["cpu_baseline"] = {k: cb[k] for k in ("value", "unit", "cores", "kind", "sample") if k in cb}
        for k in ("chunk_parallel", "page_parallel", "regex_native"):
            if k in cb:
                out["cpu_baseline"][k] = {"value": _r(cb[k]["value"]), "unit": cb[k]["unit"],
                                          "cores": cb[k].get("cores")}
    legs = {}
    rx = res.get("regex")
    if rx:
        legs["c3_regex"] = {"pages_per_s": _r(rx["pages_per_s"]), "ms": _r(rx["ms_per_scan"]),
                            "frac": _r(rx["roofline_frac"], 3), "pattern": rx["pattern"],
                            "warm_ms": _r(rx["warm"]["ms_per_scan"]), "warm_frac": _r(rx["warm"]["roofline_frac"], 3),
                            "validated": rx.get("all_validated", rx.get("validated"))}
    cd = res.get("c3_decode")
    if cd:
        legs["c3_plain"] = {"values_per_s": _r(cd["values_per_s"]), "ms": _r(cd["ms_per_decode"]),
                            "validated": cd["validated"]}
    c4 = res.get("c4")
    if c4:
        legs["c4"] = {"values_per_s": _r(c4["values_per_s"]), "ms": _r(c4["ms_per_step"]),
                      "frac": _r(c4["roofline"]["frac"], 3), "validated": c4["validated"]}
    for k in ("c5", "c5_ref"):
        c5 = res.get(k)
        if c5:
            legs[k] = {"values_per_s": _r(c5["decode_values_per_s"]), "ms": _r(c5["decode_ms"]),
                       "step_values_per_s": _r(c5["step_values_per_s"]), "rows_per_gpu": c5["rows_per_gpu"],
                       "validated": bool(c5["decode_validated"] and c5["regex_validated"])}
    wd = res.get("wide_dict")
    if wd:
        legs["wide_dict"] = {"values_per_s": _r(wd["values_per_s"]), "ms": _r(wd["ms_per_decode"]),
                             "frac": _r(wd["b_alg_frac_of_peak"], 3), "validated": wd["validated"]}
    for k, v in (res.get("ext") or {}).items():
        legs[k] = {"codec_GBs_out": _r(v["codec_GBs_out"]), "decode_ms": _r(v["decode_ms"]),
                   "validated": v["validated"]}
    for k, v in (res.get("end_to_end") or {}).items():
        legs["e2e_" + k] = {"total_ms": _r(v["total_ms"])}
        if "device_walk" in v and isinstance(v["device_walk"], dict) and "total_ms" in v["device_walk"]:
            legs["e2e_" + k]["device_walk_total_ms"] = _r(v["device_walk"]["total_ms"])
    if "api_read_all" in res:
        a = res["api_read_all"]
        legs["api_read_all"] = {"values_per_s": _r(a["values_per_s"]), "threads": a.get("threads")}
        if isinstance(a.get("chunk_1m"), dict) and "values_per_s" in a["chunk_1m"]:
            legs["api_read_all"]["chunk_1m_values_per_s"] = _r(a["chunk_1m"]["values_per_s"])
    if "strong" in res:
        legs["strong"] = {k: _r(v) if isinstance(v, float) else v for k, v in res["strong"].items()
                          if not isinstance(v, (dict, list))}
    out["legs"] = legs
    out["full_record"] = os.path.relpath(full_path, ROOT)
    return out


def main():
    args = parse()
    maybe_spawn(args)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and rank == 0:
        print(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)

    if args.cpu_only:  # child of the bench process: CPU baselines only, no GPU
        print(json.dumps(cpu_baselines(args)), flush=True)
        return
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        # in a fresh child interpreter, started before this process touches
        # the GPU (its own process pool forks; nothing GPU-side is shared)
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--cpu-only"] + sys.argv[1:],
                           stdout=subprocess.PIPE, check=True)
        cpu = json.loads(r.stdout.decode().strip().splitlines()[-1])

    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        local = local % max(1, torch.cuda.device_count())  # == LOCAL_RANK unless rehearsing on fewer GPUs
        torch.cuda.set_device(local)
        dist.init_process_group(args.dist_backend)
    from pqgpu import capi
    ctx = capi.Context(local)
    for kv in args.opt:
        k, _, v = kv.partition("=")
        ctx.set_option(k, int(v))
    J = Job(rank, world, local, dist, ctx)
    exp = expectations()

    c2 = c2_leg(J, args, exp)
    nrows = c2["nrows"]
    med = c2["median_s"]
    ms_per_step = med / args.steps * 1e3
    kern = {k: v["ms_per_launch"] for k, v in c2["kern"].items()}
    total_chars = c2["chars"]
    payload = c2["payload"]
    out_bytes = 8 * (nrows + 1) + total_chars + (nrows + 7) // 8
    b_alg = payload + out_bytes  # SURVEY §8d C2 algorithmic bytes per decode
    dom = max(kern, key=kern.get) if kern else "pipe_write"
    dom_ms = kern.get(dom, ms_per_step)
    # algorithmic bytes of one launch of the dominant kernel:
    # pipe_write produces the decoded column (offsets, chars, validity); the
    # u16 codes it reads are this design's intermediate, not algorithmic bytes
    dom_bytes = {"pipe_write": out_bytes, "pipe_codes": payload,
                 "ba_fused": b_alg}.get(dom, payload)
    achieved = dom_bytes / (dom_ms * 1e-3) / 1e9
    traffic, tsrc = pmc_traffic(args.pmc_json, dom)
    step_traffic = pmc_step_traffic(args.pmc_json, c2["kern"])

    result = {
        "metric": "decoded values/sec (RLE+dict BYTE_ARRAY) and regex pages/sec at 1/2/4/8 GPUs",
        "value": c2["value"],
        "unit": "values/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (deterministic splitmix64 generator, SURVEY §8d C2 shape)",
        "config": {"workload": f"C2: dict BYTE_ARRAY OPTIONAL, {args.rows} rows/GPU (one row group per rank of an "
                               f"{args.rows * world}-row column), {args.layout}-layout, 1000-entry dict, 5% NULL",
                   "rows_per_gpu": nrows, "pages_per_gpu": c2["pages"],
                   "parallelism": f"row-group shards x{world} (no collective)"},
        "timing": {"repeats_ms_per_step": [s / args.steps * 1e3 for s in c2["secs"]],
                   "statistic": f"median of {args.repeats} regions of {args.steps} steps, max over ranks"},
        "validated": c2["validated"],
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": tsrc,
                     "kernel": dom, "kernel_ms": dom_ms, "algorithmic_bytes": dom_bytes,
                     "step_traffic": step_traffic["bytes"] if step_traffic else None,
                     "step_traffic_over_b_alg": step_traffic["bytes"] / b_alg if step_traffic else None,
                     "step_traffic_per_kernel": step_traffic["per_kernel"] if step_traffic else None},
        "pipeline": {"kernel_ms": kern,
                     "kernel_ms_note": "HIP events on the decode streams, same steps repeated after the timed "
                                       "regions (events perturb the wall clock)",
                     "sum_kernel_ms": sum(kern.values()),
                     "b_alg_bytes": b_alg, "b_alg_GBs_per_step": b_alg / (ms_per_step * 1e-3) / 1e9,
                     "b_alg_frac_of_peak": b_alg / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS,
                     "nonnull": c2["nonnull"], "chars": total_chars},
    }
    if "e2e" in c2:
        result["end_to_end"] = {"c2": c2["e2e"]}
    if "api_read_all" in c2:
        result["api_read_all"] = c2["api_read_all"]
    if world > 1:
        result["strong"] = strong_leg(J, args)

    if not args.no_regex:
        result["regex"], result["c3_decode"] = c3_legs(J, args, exp)
        if "e2e" in result["regex"]:
            result.setdefault("end_to_end", {})["c3_regex"] = result["regex"].pop("e2e")
    if not args.no_c4:
        result["c4"] = c4_leg(J, args)
    if not args.no_c5:
        result["c5"] = c5_leg(J, args, exp)
        if not args.no_c5_ref:
            result["c5_ref"] = c5_leg(J, args, exp, layout="ref")
    if not args.no_wide:
        result["wide_dict"] = wide_dict_leg(J, args)
    if not args.no_ext:
        result["ext"] = ext_leg(J, args)
    if cpu is not None:
        st = cpu["single_thread"]
        result["cpu_baseline"] = {"value": st["value"], "unit": "values/s", "cores": 1, "kind": "reference",
                                  "sample": st["sample"] + " (the reference's own ColumnReader, oracle/_ref, -O2)",
                                  **{k: v for k, v in cpu.items() if k != "single_thread"}}
    ctx.close()
    if rank == 0:
        path = args.full_json
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "w") as fh:
            json.dump(result, fh, indent=1)
        line = json.dumps(compact(result, path))
        assert len(line) < 6000, f"headline line {len(line)} B: the driver reads ~8 KB of stdout"
        print(line, flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
