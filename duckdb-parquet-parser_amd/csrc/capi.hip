#include <cstdio>
// capi.hip — implementation of the C ABI declared in include/pq_gpu.h.
//
// Host side of the boundary: the page walk runs on the CPU (pqfmt), page
// bytes are uploaded to HBM once per chunk, and the decode is a short,
// allocation-free sequence of launches on the context's stream.  No C++
// exception crosses an extern "C" function.
#include "host/capi_state.hpp"

using namespace pqcapi;

namespace {

// fn(0 .. n-1) on up to hardware_concurrency host threads (inline when n == 1).
template <class Fn>
void parallel_for(int n, Fn&& fn) {
    if (n <= 1) {
        if (n == 1) fn(0);
        return;
    }
    const int nt = std::max(1, std::min<int>(n, static_cast<int>(std::thread::hardware_concurrency())));
    std::atomic<int> next{0};
    std::vector<std::thread> th;
    for (int t = 0; t < nt; t++)
        th.emplace_back([&]() {
            for (int i = next.fetch_add(1); i < n; i = next.fetch_add(1)) fn(i);
        });
    for (auto& x : th) x.join();
}

int set_err(pq_ctx* ctx, int code, const std::string& m) {
    if (ctx) ctx->err = m;
    return code;
}

int hip_check(pq_ctx* ctx, hipError_t e, const char* what) {
    if (e == hipSuccess) return 0;
    return set_err(ctx, PQ_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

// Every entry point that touches the GPU runs on its context's device: a host
// thread may drive contexts on several devices, and HIP's
// current device is per thread.  Restores the caller's device on return.
struct DevGuard {
    int prev = -1;
    explicit DevGuard(const pq_ctx* c) : DevGuard(c ? c->device : -1) {}
    explicit DevGuard(int device) {
        int cur = 0;
        if (device >= 0 && hipGetDevice(&cur) == hipSuccess && cur != device && hipSetDevice(device) == hipSuccess) prev = cur;
    }
    ~DevGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

int plain_width_of(int32_t type) {
    switch (type) {
        case PQ_BOOLEAN: return 1;
        case PQ_INT32: case PQ_FLOAT: return 4;
        case PQ_INT64: case PQ_DOUBLE: return 8;
        case PQ_INT96: return 12;
        default: return 0;
    }
}

// Launch bracket for per-kernel HIP-event timing on the context stream.
struct Timed {
    pq_ctx* ctx;
    PendingTimer t{};
    bool on;
    hipStream_t st;
    Timed(pq_ctx* c, const char* name, hipStream_t s = nullptr) : ctx(c), on(c->timing), st(s ? s : c->stream) {
        if (!on) return;
        t.name = name;
        if (!ctx->free_events.empty()) {
            t.a = ctx->free_events.back().first;
            t.b = ctx->free_events.back().second;
            ctx->free_events.pop_back();
        } else {
            (void)hipEventCreate(&t.a);
            (void)hipEventCreate(&t.b);
        }
        (void)hipEventRecord(t.a, st);
    }
    ~Timed() {
        if (!on) return;
        (void)hipEventRecord(t.b, st);
        ctx->pending.push_back(t);
    }
};

// Host-side phase timer (wall ms) filed under `name` in the same table as the
// kernel timers while timing is on (upload phases: up_walk, up_plan,
// up_alloc, up_h2d).
struct HostTimed {
    pq_ctx* ctx;
    const char* name;
    std::chrono::steady_clock::time_point t0;
    HostTimed(pq_ctx* c, const char* n) : ctx(c), name(n), t0(std::chrono::steady_clock::now()) {}
    ~HostTimed() {
        if (!ctx->timing) return;
        auto& e = ctx->timers[name];
        e.first += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        e.second += 1;
    }
};

void resolve_timers(pq_ctx* ctx) {
    if (ctx->pending.empty()) return;
    (void)hipStreamSynchronize(ctx->stream);
    for (auto& p : ctx->pending) {
        float ms = 0;
        (void)hipEventElapsedTime(&ms, p.a, p.b);
        auto& e = ctx->timers[p.name];
        e.first += ms;
        e.second += 1;
        ctx->free_events.push_back({p.a, p.b});
    }
    ctx->pending.clear();
}

std::string format_error(const DevErr& e) {
    switch (e.code) {
        case PQ_ERR_BUFFER:
            return "ByteBuffer: read beyond end (pos=" + std::to_string(static_cast<uint32_t>(e.pos)) +
                   " need=" + std::to_string(static_cast<uint32_t>(e.need)) +
                   " size=" + std::to_string(static_cast<uint32_t>(e.size)) + ")";
        case PQ_ERR_FLBA: return "FIXED_LEN_BYTE_ARRAY not supported without type_length";
        case PQ_ERR_UNSUPPORTED: return "page encoding outside the supported parity scope";
        default: return "decode error " + std::to_string(e.code);
    }
}

void free_chunk_device(pq_chunk* c) {
    dfree(c->d_bytes);
    dfree(c->d_pages);
    dfree(c->d_dicts);
    dfree(c->d_tiles);
    dfree(c->d_page_tile0);
    dfree(c->d_entries);
    dfree(c->d_dict_count);
    dfree(c->d_page_err);
    dfree(c->d_dict_err);
    if (c->d_zero) {  // d_flags, d_bsum and d_flist live in it
        dfree(c->d_zero);
        c->d_flags = nullptr;
        c->d_bsum = nullptr;
        c->d_flist = nullptr;
    }
    dfree(c->d_flags);
    dfree(c->d_bigd);
    dfree(c->d_rx_index);
    dfree(c->d_row_codes);
    dfree(c->d_tile_chars);
    dfree(c->d_tile_rank);
    dfree(c->d_pwins);
    dfree(c->d_pwbase);
    dfree(c->d_rowinfo);
    dfree(c->d_wchars);
    dfree(c->d_pbsum);
    dfree(c->d_runs);
    dfree(c->d_info);
    dfree(c->d_codes);
    dfree(c->d_tile_nn);
    dfree(c->d_bsum);
    dfree(c->d_flist);
    dfree(c->d_bigp);
    dfree(c->d_chunk_base);
    dfree(c->d_chunks);
    dfree(c->d_cand);
    dfree(c->d_ppages);
    dfree(c->d_page_nn); dfree(c->d_onnv); dfree(c->d_ochv); dfree(c->d_opdense); dfree(c->d_opbase);
    dfree(c->d_otot); dfree(c->d_vpages); dfree(c->d_doffs); dfree(c->d_operr); dfree(c->d_pwpage);
    dfree(c->d_perr);
    dfree(c->d_page_pos);
    dfree(c->d_tile_base);
    dfree(c->d_total);
    dfree(c->d_dflag);
    dfree(c->d_scan_scratch);
    dfree(c->d_page_flags);
    dfree(c->d_dict_match);
    dfree(c->d_dfa);
    dfree(c->d_status);
    dfree(c->d_tickets);
    dfree(c->d_bases);
    if (c->d_prog) { pqre::free_device_program(c->d_prog); c->d_prog = nullptr; }
}

}  // namespace

extern "C" {

int pq_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return n;
}

int pq_plan_page_ranges(const pq_page_desc* table, int64_t ntable, int world, int64_t* ranges) {
    if ((!table && ntable) || ntable < 0 || world <= 0 || !ranges) return PQ_ERR_ARG;
    // cumulative payload bytes of the data pages (shard.py page_ranges)
    std::vector<int64_t> cum;
    cum.reserve(static_cast<size_t>(ntable));
    int64_t acc = 0;
    for (int64_t i = 0; i < ntable; i++) {
        if (table[i].page_type != PQ_DATA_PAGE) continue;
        acc += std::max<int64_t>(table[i].payload_size, 0);
        cum.push_back(acc);
    }
    const int64_t n = static_cast<int64_t>(cum.size());
    int64_t prev = 0;
    for (int k = 0; k < world; k++) {
        int64_t cut = n;
        if (k + 1 < world) {
            if (n == 0) {
                cut = 0;
            } else {
                // first page whose running total reaches (k + 1) / world of the sum, plus one
                // (the float64 quotient of the exact product, as shard.py computes it)
                const double target = static_cast<double>(acc * (k + 1)) / world;
                const int64_t c = static_cast<int64_t>(
                    std::lower_bound(cum.begin(), cum.end(), target,
                                     [](int64_t v, double t) { return static_cast<double>(v) < t; }) -
                    cum.begin()) + 1;
                cut = std::min(std::max(c, prev), n);
            }
        }
        ranges[2 * k] = prev;
        ranges[2 * k + 1] = cut;
        prev = cut;
    }
    return 0;
}

pq_ctx* pq_ctx_create(int device) {
    try {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || n <= device || device < 0) return nullptr;
        DevGuard dg(device);  // the caller's current device comes back on return
        int cur = -1;
        if (hipGetDevice(&cur) != hipSuccess || cur != device) return nullptr;
        auto* c = new pq_ctx();
        c->device = device;
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0)
            c->cus = cus;
        if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
            delete c;
            return nullptr;
        }
        if (hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking) != hipSuccess ||
            hipStreamCreateWithFlags(&c->copy, hipStreamNonBlocking) != hipSuccess ||
            hipStreamCreateWithFlags(&c->copy2, hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming) != hipSuccess) {
            if (c->side) (void)hipStreamDestroy(c->side);
            if (c->copy) (void)hipStreamDestroy(c->copy);
            if (c->copy2) (void)hipStreamDestroy(c->copy2);
            (void)hipStreamDestroy(c->stream);
            delete c;
            return nullptr;
        }
        return c;
    } catch (...) {
        return nullptr;
    }
}

void pq_ctx_destroy(pq_ctx* ctx) {
    if (!ctx) return;
    {
    DevGuard dg(ctx);
    (void)hipStreamSynchronize(ctx->stream);
    for (auto& p : ctx->pending) { (void)hipEventDestroy(p.a); (void)hipEventDestroy(p.b); }
    for (auto& p : ctx->free_events) { (void)hipEventDestroy(p.first); (void)hipEventDestroy(p.second); }
    if (ctx->d_prof) (void)hipFree(ctx->d_prof);
    (void)hipStreamSynchronize(ctx->side);
    (void)hipEventDestroy(ctx->ev_fork);
    (void)hipEventDestroy(ctx->ev_join);
    (void)hipStreamDestroy(ctx->side);
    ctx->stager.release();
    if (ctx->d_raw) (void)hipFree(ctx->d_raw);
    if (ctx->d_walk) (void)hipFree(ctx->d_walk);
    if (ctx->h_walk) (void)hipHostFree(ctx->h_walk);
    if (ctx->d_relay) (void)hipFree(ctx->d_relay);
    if (ctx->d_codec) (void)hipFree(ctx->d_codec);
    if (ctx->d_codec_st) (void)hipFree(ctx->d_codec_st);
    if (ctx->d_zsrc) (void)hipFree(ctx->d_zsrc);
    if (ctx->d_chunker) (void)hipFree(ctx->d_chunker);
    (void)hipStreamSynchronize(ctx->copy);
    (void)hipStreamDestroy(ctx->copy);
    (void)hipStreamSynchronize(ctx->copy2);
    (void)hipStreamDestroy(ctx->copy2);
    (void)hipStreamDestroy(ctx->stream);
    }
    delete ctx;
}

int pq_ctx_set_option(pq_ctx* ctx, const char* key, int64_t value) {
    if (!ctx || !key) return PQ_ERR_ARG;
    DevGuard dg(ctx);
    if (std::strcmp(key, "fused_ba") == 0) { ctx->opt_fused = value != 0; return 0; }
    if (std::strcmp(key, "wide_rows") == 0) { ctx->opt_wide_rows = value != 0; return 0; }
    if (std::strcmp(key, "pipe_wide") == 0) { ctx->opt_pipe_wide = value != 0; return 0; }
    if (std::strcmp(key, "levels_small") == 0) { ctx->opt_levels_small = value != 0; return 0; }
    if (std::strcmp(key, "gather_rows") == 0) { ctx->opt_gather_rows = value != 0; return 0; }
    if (std::strcmp(key, "fused_debug") == 0) { ctx->opt_debug = static_cast<int>(value); return 0; }
    if (std::strcmp(key, "fused_waves") == 0) { ctx->opt_waves = static_cast<int>(value); return 0; }
    if (std::strcmp(key, "fused_claim") == 0) {
        if (value < 1 || value > 64) return set_err(ctx, PQ_ERR_ARG, "fused_claim: 1..64");
        ctx->opt_claim = static_cast<int>(value);
        return 0;
    }
    if (std::strcmp(key, "regex_dfa") == 0) { ctx->opt_regex_dfa = value != 0; return 0; }
    if (std::strcmp(key, "regex_debug") == 0) { ctx->opt_regex_debug = static_cast<int>(value); return 0; }
    if (std::strcmp(key, "regex_plain") == 0) { ctx->opt_regex_plain = value != 0; return 0; }
    if (std::strcmp(key, "regex_codes") == 0) { ctx->opt_regex_codes = value != 0; return 0; }
    if (std::strcmp(key, "regex_reuse") == 0) { ctx->opt_regex_reuse = value != 0; return 0; }
    if (std::strcmp(key, "regex_index") == 0) {
        if (value < 0 || value > 2) return set_err(ctx, PQ_ERR_ARG, "regex_index: 0, 1 or 2");
        ctx->opt_regex_index = static_cast<int>(value);
        return 0;
    }
    if (std::strcmp(key, "zflip") == 0) { ctx->opt_zflip = value != 0; return 0; }
    if (std::strcmp(key, "write_waves") == 0) {
        if (value < 1 || value > 16) return set_err(ctx, PQ_ERR_ARG, "write_waves: 1..16");
        ctx->opt_write_waves = static_cast<int>(value);
        return 0;
    }
    if (std::strcmp(key, "big_all") == 0) { ctx->opt_big_all = value != 0; return 0; }
    if (std::strcmp(key, "fixed_plain") == 0) { ctx->opt_fixed_plain = value != 0; return 0; }
    if (std::strcmp(key, "fixed_fused") == 0) { ctx->opt_fixed_fused = value != 0; return 0; }
    if (std::strcmp(key, "dict_pipe") == 0) { ctx->opt_pipe = value != 0; return 0; }
    if (std::strcmp(key, "plain_ba") == 0) { ctx->opt_plain = value != 0; return 0; }
    if (std::strcmp(key, "plain_fused") == 0) { ctx->opt_plain_fused = value != 0; return 0; }
    if (std::strcmp(key, "pipe_run_dict") == 0) { ctx->opt_run_dict = value != 0; return 0; }
    if (std::strcmp(key, "write_bpc") == 0) {
        if (value < 0 || value > 4) return set_err(ctx, PQ_ERR_ARG, "write_bpc: 0..4");
        ctx->opt_write_bpc = static_cast<int>(value);
        return 0;
    }
    if (std::strcmp(key, "pipe_run_pages") == 0) {
        if (value < 0 || value > 32) return set_err(ctx, PQ_ERR_ARG, "pipe_run_pages: 0 (auto) .. 32");
        ctx->opt_run_pages = static_cast<int>(value);
        return 0;
    }
    if (std::strcmp(key, "stage_bufs") == 0) {
        if (value < 2 || value > pqstage::kMaxBufs) return set_err(ctx, PQ_ERR_ARG, "stage_bufs: 2..16");
        ctx->stager.configure(static_cast<int>(value), ctx->stager.piece());
        ctx->opt_stage_bufs = static_cast<int>(value);
        return 0;
    }
    if (std::strcmp(key, "raw_upload") == 0) { ctx->opt_raw = value != 0; return 0; }
    if (std::strcmp(key, "device_walk") == 0) { ctx->opt_dev_walk = value != 0; return 0; }
    if (std::strcmp(key, "stage_streams") == 0) {
        if (value < 1 || value > 2) return set_err(ctx, PQ_ERR_ARG, "stage_streams: 1..2");
        ctx->opt_stage_streams = static_cast<int>(value);
        return 0;
    }
    if (std::strcmp(key, "stage_piece_kb") == 0) {
        if (value < 64 || value > 65536) return set_err(ctx, PQ_ERR_ARG, "stage_piece_kb: 64..65536");
        ctx->stager.configure(ctx->opt_stage_bufs, static_cast<size_t>(value) << 10);
        return 0;
    }
    if (std::strcmp(key, "regex_win") == 0) {
        if (value < 1024 || value > 32768 || value % 16) return set_err(ctx, PQ_ERR_ARG, "regex_win: 1024..32768, multiple of 16");
        ctx->opt_regex_win = static_cast<int>(value);
        return 0;
    }
    if (std::strcmp(key, "fused_prof") == 0) {
        if (value && !ctx->d_prof) {
            if (hipMalloc(reinterpret_cast<void**>(&ctx->d_prof), 64 * sizeof(uint64_t)) != hipSuccess)
                return set_err(ctx, PQ_ERR_HIP, "hipMalloc failed (prof)");
            (void)hipMemset(ctx->d_prof, 0, 64 * sizeof(uint64_t));
        } else if (!value && ctx->d_prof) {
            (void)hipFree(ctx->d_prof);
            ctx->d_prof = nullptr;
        }
        return 0;
    }
    return set_err(ctx, PQ_ERR_ARG, std::string("unknown option ") + key);
}

const char* pq_last_error(const pq_ctx* ctx) { return ctx ? ctx->err.c_str() : "no context"; }
void* pq_ctx_stream(pq_ctx* ctx) { return ctx ? static_cast<void*>(ctx->stream) : nullptr; }
int pq_ctx_sync(pq_ctx* ctx) {
    if (!ctx) return PQ_ERR_ARG;
    DevGuard dg(ctx);
    return hip_check(ctx, hipStreamSynchronize(ctx->stream), "hipStreamSynchronize");
}

int pq_build_page_table(const uint8_t* file, size_t file_len, const pq_chunk_desc* chunk,
                        pq_page_desc* pages, int64_t cap, int64_t* npages, char* err,
                        size_t errlen) {
    if (!file || !chunk || !npages) return PQ_ERR_ARG;
    try {
        pqfmt::WalkResult w = pqfmt::walk_chunk(file, file_len, *chunk);
        *npages = static_cast<int64_t>(w.pages.size());
        for (int64_t i = 0; i < cap && i < *npages; i++) pages[i] = w.pages[i];
        if (err && errlen) {
            std::strncpy(err, w.message.c_str(), errlen - 1);
            err[errlen - 1] = 0;
        }
        return w.error;
    } catch (...) {
        return PQ_ERR_ALLOC;
    }
}

}  // extern "C" (a C++ helper)

// The device walk (walk.hip) of one chunk over d_bytes = file bytes
// [base, base + len): the page table to `host` (pinned staging, then `sink`)
// and the page count.  PQ_ERR_UNSUPPORTED: refused (the host walk decides).
template <class Sink>
static int device_walk(pq_ctx* ctx, const uint8_t* d_bytes, size_t len, int64_t base, const pq_chunk_desc* chunk,
                       int64_t seg_bytes, int64_t rec_cap, int64_t* npages, Sink&& sink) {
    *npages = 0;
    if (chunk->codec != 0 || chunk->ext_flags != 0 || chunk->num_values <= 0) return PQ_ERR_UNSUPPORTED;
    int64_t off = chunk->data_page_offset;
    if (chunk->has_dictionary_page_offset) off = std::min(off, chunk->dictionary_page_offset);
    if (off < base || off >= base + static_cast<int64_t>(len)) return PQ_ERR_UNSUPPORTED;
    const uint64_t seg = seg_bytes ? static_cast<uint64_t>(seg_bytes) : 8192u;
    if (seg > (1u << 30) || rec_cap < 0 || rec_cap > (int64_t{1} << 20)) return PQ_ERR_UNSUPPORTED;
    const uint32_t rc = static_cast<uint32_t>(rec_cap ? rec_cap : std::max<int64_t>(1, static_cast<int64_t>(seg) / 128));
    const uint64_t start = static_cast<uint64_t>(off), end = static_cast<uint64_t>(base) + len;
    const uint64_t nseg64 = (end - start + seg - 1) / seg;
    if (nseg64 > (1u << 30) / rc) return PQ_ERR_UNSUPPORTED;
    const uint32_t nseg = static_cast<uint32_t>(nseg64);
    pqk::WalkLaunch W{};
    W.bytes = d_bytes; W.base = static_cast<uint64_t>(base); W.len = len;
    W.start = start; W.end = end; W.seg = seg; W.nseg = nseg; W.cap = rc;
    W.num_values = chunk->num_values;
    const size_t nrec = static_cast<size_t>(nseg) * rc;
    // one device buffer, kept by the context: records, segments, links, bases, the page table
    auto al = [](size_t b) { return (b + 255) / 256 * 256; };
    const size_t o_recs = 0, o_segs = o_recs + al(nrec * sizeof(pqk::WalkRec));
    const size_t o_links = o_segs + al(nseg * pqk::walk_seg_bytes());
    const size_t o_bases = o_links + al(nseg * pqk::walk_link_bytes());
    const size_t o_out = o_bases + al(3 * static_cast<size_t>(nseg) * 8);
    const size_t o_pages = o_out + 256, total = o_pages + al(nrec * sizeof(pq_page_desc));
    if (ctx->walk_cap < total) {
        if (ctx->d_walk) (void)hipFree(ctx->d_walk);
        ctx->d_walk = nullptr;
        ctx->walk_cap = 0;
        if (int e = hip_check(ctx, hipMalloc(reinterpret_cast<void**>(&ctx->d_walk), total), "hipMalloc (device walk)")) return e;
        ctx->walk_cap = total;
    }
    uint8_t* mem = ctx->d_walk;
    W.recs = reinterpret_cast<pqk::WalkRec*>(mem + o_recs);
    W.segs = mem + o_segs;
    W.links = mem + o_links;
    W.base_pg = reinterpret_cast<int64_t*>(mem + o_bases);
    W.base_val = W.base_pg + nseg;
    W.dict_in = W.base_val + nseg;
    W.out = reinterpret_cast<int64_t*>(mem + o_out);
    W.pages = reinterpret_cast<pq_page_desc*>(mem + o_pages);
    {
        Timed t(ctx, "walk");
        pqk::launch_walk(ctx->stream, W);
    }
    int64_t res[8] = {-1, -1, 0, 0, 0, 0, 0, 0};
    int rc2 = hip_check(ctx, hipGetLastError(), "walk launch");
    if (!rc2) rc2 = hip_check(ctx, hipMemcpyAsync(res, W.out, sizeof res, hipMemcpyDeviceToHost, ctx->stream), "walk result");
    if (!rc2) rc2 = hip_check(ctx, hipStreamSynchronize(ctx->stream), "walk sync");
    if (std::getenv("PQ_WALK_DEBUG"))
        std::fprintf(stderr, "walk: pages %lld cut %lld entry %lld n %lld exit %lld bad %lld prev_exit %lld first %lld (start %llu seg %llu)\n",
                     (long long)res[0], (long long)res[1], (long long)res[2], (long long)res[3], (long long)res[4],
                     (long long)res[5], (long long)res[6], (long long)res[7], (unsigned long long)start,
                     (unsigned long long)seg);
    if (rc2) return rc2;
    if (res[0] < 0) return PQ_ERR_UNSUPPORTED;
    *npages = res[0];
    const size_t k = static_cast<size_t>(res[0]);
    if (k) {
        if (ctx->h_walk_cap < k) {
            if (ctx->h_walk) (void)hipHostFree(ctx->h_walk);
            ctx->h_walk = nullptr;
            ctx->h_walk_cap = 0;
            if (int e = hip_check(ctx, hipHostMalloc(reinterpret_cast<void**>(&ctx->h_walk), k * sizeof(pq_page_desc)),
                                  "hipHostMalloc (device walk)"))
                return e;
            ctx->h_walk_cap = k;
        }
        if (int e = hip_check(ctx, hipMemcpyAsync(ctx->h_walk, W.pages, k * sizeof(pq_page_desc), hipMemcpyDeviceToHost,
                                                  ctx->stream), "walk copy"))
            return e;
        if (int e = hip_check(ctx, hipStreamSynchronize(ctx->stream), "walk copy sync")) return e;
    }
    sink(ctx->h_walk, k);
    return 0;
}

extern "C" {

int pq_build_page_table_device(pq_ctx* ctx, const uint8_t* d_bytes, size_t len, int64_t base,
                               const pq_chunk_desc* chunk, int64_t seg_bytes, int64_t rec_cap,
                               pq_page_desc* pages, int64_t cap, int64_t* npages) {
    if (!ctx || !chunk || !npages || (!d_bytes && len) || base < 0 || seg_bytes < 0 || seg_bytes > (int64_t{1} << 30) ||
        rec_cap < 0 || rec_cap > (int64_t{1} << 20) || cap < 0 || (cap && !pages))
        return PQ_ERR_ARG;
    *npages = 0;
    DevGuard dg(ctx);
    try {
        return device_walk(ctx, d_bytes, len, base, chunk, seg_bytes, rec_cap, npages,
                           [&](const pq_page_desc* h, size_t k) {
                               std::memcpy(pages, h, std::min<size_t>(k, static_cast<size_t>(cap)) * sizeof(pq_page_desc));
                           });
    } catch (const std::exception& e) {
        return set_err(ctx, PQ_ERR_ALLOC, e.what());
    }
}

int pq_device_buffer(pq_ctx* ctx, const uint8_t* host, size_t n, void** d_out) {
    if (!ctx || !d_out || (!host && n)) return PQ_ERR_ARG;
    DevGuard dg(ctx);
    uint8_t* d = nullptr;
    if (int rc = hip_check(ctx, hipMalloc(reinterpret_cast<void**>(&d), n + 64), "hipMalloc (device buffer)")) return rc;
    int rc = hip_check(ctx, hipMemset(d + n, 0, 64), "device buffer pad");
    if (!rc && n) rc = hip_check(ctx, hipMemcpy(d, host, n, hipMemcpyHostToDevice), "device buffer copy");
    if (rc) {
        (void)hipFree(d);
        return rc;
    }
    *d_out = d;
    return 0;
}

void pq_device_buffer_free(pq_ctx* ctx, void* d) {
    if (!ctx || !d) return;
    DevGuard dg(ctx);
    (void)hipFree(d);
}

// Raw path of an upload: the chunk's byte extents, exactly
// as the file holds them, go to HBM (ctx->d_raw) through the pinned ring on a
// host thread that starts before the page walk, so the H2D overlaps the walk
// and the planning; a GPU pass (k_relayout) then builds the slot image.
struct RawStage {
    std::vector<std::pair<int64_t, int64_t>> ext;  // (file offset, bytes), in d_raw order
    std::vector<int64_t> base;                     // d_raw offset of each extent
    int64_t total = 0;
    std::thread th;
    hipError_t err = hipSuccess;
    bool active = false;
    void join() {
        if (th.joinable()) th.join();
    }
    ~RawStage() { join(); }
};

static void raw_start(pq_ctx* ctx, const uint8_t* file, size_t file_len, RawStage& R) {
    R.active = false;
    if (!ctx->opt_raw || R.ext.empty()) return;
    R.total = 0;
    R.base.clear();
    for (auto& e : R.ext) {
        e.first = std::max<int64_t>(0, e.first);
        e.second = std::max<int64_t>(0, std::min<int64_t>(e.second, static_cast<int64_t>(file_len) - e.first));
        R.base.push_back(R.total);
        R.total += (e.second + 15) / 16 * 16;  // each extent 16-byte aligned in d_raw
    }
    if (R.total <= 0) return;
    const size_t need = static_cast<size_t>(R.total) + 64;
    if (ctx->raw_cap < need) {
        if (ctx->d_raw) (void)hipFree(ctx->d_raw);
        ctx->d_raw = nullptr;
        ctx->raw_cap = 0;
        if (hipMalloc(reinterpret_cast<void**>(&ctx->d_raw), need) != hipSuccess) {
            ctx->d_raw = nullptr;
            return;
        }
        ctx->raw_cap = need;
    }
    R.active = true;
    const int hw = static_cast<int>(std::min(16u, std::max(1u, std::thread::hardware_concurrency())));
    R.th = std::thread([ctx, file, &R, hw]() {
        (void)hipSetDevice(ctx->device);  // a new host thread starts on device 0
        auto fill = [&](uint8_t* dst, size_t a, size_t z) {
            // extents overlapping [a, z) of d_raw
            size_t k = static_cast<size_t>(std::upper_bound(R.base.begin(), R.base.end(), static_cast<int64_t>(a)) -
                                           R.base.begin());
            k = k ? k - 1 : 0;
            size_t at = a;
            for (; k < R.ext.size() && at < z; k++) {
                const size_t b0 = static_cast<size_t>(R.base[k]);
                const size_t b1 = b0 + static_cast<size_t>(R.ext[k].second);
                const size_t b2 = b0 + static_cast<size_t>((R.ext[k].second + 15) / 16 * 16);
                if (b2 <= at) continue;
                if (at < b1) {
                    const size_t e = std::min(z, b1);
                    std::memcpy(dst + (at - a), file + R.ext[k].first + (at - b0), e - at);
                    at = e;
                }
                if (at < z && at < b2) {
                    const size_t e = std::min(z, b2);
                    std::memset(dst + (at - a), 0, e - at);
                    at = e;
                }
            }
            if (at < z) std::memset(dst + (at - a), 0, z - at);
        };
        R.err = ctx->stager.upload(ctx->d_raw, static_cast<size_t>(R.total), ctx->copy, hw, fill,
                                   ctx->opt_stage_streams > 1 ? ctx->copy2 : nullptr);
    });
}


// Builds the device chunk from page walks already made on the host: one walk
// per input chunk (pq_chunk_upload) or one page-range walk (pq_chunk_upload_range).
static int upload_walked(pq_ctx* ctx, const uint8_t* file, size_t file_len, const pq_chunk_desc& desc,
                         std::vector<pqfmt::WalkResult>& walks, int64_t row_offset, pq_chunk** out,
                         RawStage* raw) {
    const int nchunks = static_cast<int>(walks.size());
    try {
        (void)hipSetDevice(ctx->device);
        auto c = std::make_unique<pq_chunk>();
        c->type = desc.type;
        c->max_def = desc.max_def_level;
        c->max_rep = desc.max_rep_level;
        c->plain_width = plain_width_of(c->type);
        c->width = c->plain_width;
        c->row_offset = row_offset;
        std::unique_ptr<HostTimed> plan_timer(new HostTimed(ctx, "up_plan"));
        std::unique_ptr<HostTimed> sub_timer(new HostTimed(ctx, "up_plan_pages"));

        // 1) host walks; every payload gets a 16-byte aligned slot in one image
        // per-page host tables: the context's scratch (capacity kept across
        // uploads, so a reader walking many row groups does not page-fault
        // fresh tables in each time; a context serves one thread at a time)
        PVec<DevPage>& hpages = ctx->s_hpages;
        std::vector<DevDict> hdicts;
        HVec<std::pair<int64_t, int64_t>>& copies = ctx->s_copies;  // (file offset, image offset) per payload
        HVec<int32_t>& copy_size = ctx->s_copy_size;
        hpages.clear();
        copies.clear();
        copy_size.clear();
        int64_t seq = 0, row_base = 0, img = 0;
        {
            size_t tot = 0;
            for (const auto& w : walks) tot += w.pages.size();
            hpages.reserve(tot);
            copies.reserve(tot);
            copy_size.reserve(tot);
            if (nchunks > 1) c->walked.reserve(tot);
            c->page_seq.reserve(tot);
        }
        // pages the codec pass rebuilds (compressed or DATA_PAGE_V2): their slot
        // holds the V1-layout payload; the image build leaves it zero
        std::vector<pqk::CodecEntry> cents;
        std::vector<int64_t> cent_file;  // payload file offset per codec entry
        auto codec_page = [&](const pq_page_desc& p, int32_t* out_len) -> bool {
            if (!(p.flags & (PQ_PAGE_COMPRESSED | PQ_PAGE_V2))) return false;
            const bool v2 = (p.flags & PQ_PAGE_V2) != 0, comp = (p.flags & PQ_PAGE_COMPRESSED) != 0;
            const int64_t lv = v2 ? static_cast<int64_t>(p.v2_def_len) + p.v2_rep_len : 0;
            const int64_t vals = (comp ? static_cast<int64_t>(p.uncompressed_size) : static_cast<int64_t>(p.payload_size)) - lv;
            const int64_t n = vals + (v2 && desc.max_def_level > 0 ? 4 + p.v2_def_len : 0) +
                              (v2 && desc.max_rep_level > 0 ? 4 + p.v2_rep_len : 0);
            if (vals < 0 || n > (1ll << 31) - 64 || p.payload_size < 0)
                throw pqfmt::Error(PQ_ERR_DECOMPRESS, "page header: uncompressed_page_size out of range");
            pqk::CodecEntry e{};
            e.src_len = static_cast<uint32_t>(std::max<int64_t>(0, std::min<int64_t>(p.payload_size, static_cast<int64_t>(file_len) - p.payload_offset)));
            e.out_len = static_cast<uint32_t>(n);
            e.def_len = v2 ? static_cast<uint32_t>(p.v2_def_len) : 0u;
            e.rep_len = v2 ? static_cast<uint32_t>(p.v2_rep_len) : 0u;
            e.codec = comp ? static_cast<uint32_t>((p.flags >> 8) & 0xFF) : 0u;
            e.flags = v2 ? (pqk::kCodecV2 | (desc.max_def_level > 0 ? pqk::kCodecDefPrefix : 0u) |
                            (desc.max_rep_level > 0 ? pqk::kCodecRepPrefix : 0u))
                         : 0u;
            cents.push_back(e);
            cent_file.push_back(p.payload_offset);
            *out_len = static_cast<int32_t>(n);
            return true;
        };
        auto slot = [&](int64_t file_off, int32_t size) {
            int64_t at = img;
            if (!cents.empty() && cents.back().dst == ~0ull) {  // the codec entry just made
                cents.back().dst = static_cast<uint64_t>(at);
                file_off = -1;
            }
            copies.push_back({file_off, at});
            copy_size.push_back(size);
            img += (static_cast<int64_t>(size) + 15) / 16 * 16 + 16;
            return at;
        };
        const int hw_plan = static_cast<int>(std::min(16u, std::max(1u, std::thread::hardware_concurrency())));
        for (int k = 0; k < nchunks; k++) {
            pqfmt::WalkResult& w = walks[static_cast<size_t>(k)];
            pq_chunk::Range rg;
            rg.p0 = static_cast<int32_t>(hpages.size());
            if (plan_pages_parallel(c.get(), desc, w, nchunks > 1, hw_plan, seq, row_base, img, hpages, hdicts, copies,
                                    copy_size)) {
                rg.np = static_cast<int32_t>(hpages.size()) - rg.p0;
                c->ranges.push_back(rg);
                seq += static_cast<int64_t>(w.pages.size());
                if (w.error) {
                    c->walk_error = w.error;
                    c->walk_message = w.message;
                    c->walk_error_seq = seq;
                    break;
                }
                continue;
            }
            std::vector<int32_t> dict_of_walk(w.pages.size(), -1);
            for (size_t i = 0; i < w.pages.size(); i++) {
                pq_page_desc p = w.pages[i];
                int64_t sq = seq + static_cast<int64_t>(i);
                int32_t psize = p.payload_size;
                if ((p.page_type == PQ_DICTIONARY_PAGE || p.page_type == PQ_DATA_PAGE) && codec_page(p, &psize))
                    cents.back().dst = ~0ull;  // placed by slot()
                if (p.page_type == PQ_DICTIONARY_PAGE) {
                    DevDict d{};
                    d.off = static_cast<uint64_t>(slot(p.payload_offset, psize));
                    d.size = psize;
                    d.nvals = p.num_values;
                    d.entry_base = static_cast<int32_t>(c->nentries);
                    c->max_dict_bytes = std::max<uint32_t>(c->max_dict_bytes, static_cast<uint32_t>(std::max(psize, 0)));
                    int64_t cap = c->type == PQ_BYTE_ARRAY
                                      ? std::min<int64_t>(p.num_values, psize / 4 + 1)
                                      : 0;
                    c->nentries += std::max<int64_t>(cap, 0);
                    dict_of_walk[i] = static_cast<int32_t>(hdicts.size());
                    hdicts.push_back(d);
                    c->dict_seq.push_back(sq);
                    c->payload_bytes += psize;
                } else if (p.page_type == PQ_DATA_PAGE) {
                    DevPage d{};
                    d.off = static_cast<uint64_t>(slot(p.payload_offset, psize));
                    d.size = psize;
                    d.nvals = p.num_values;
                    d.first_row = row_base + p.first_row;
                    int dict_dev = p.dict_page >= 0 ? dict_of_walk[p.dict_page] : -1;
                    bool enc_dict = p.encoding == 2 || p.encoding == 8;
                    d.mode = (enc_dict && dict_dev >= 0) ? pqk::MODE_DICT
                             : (c->type == PQ_BOOLEAN ? ((desc.ext_flags && p.encoding == 3) ? pqk::MODE_BOOL_RLE : pqk::MODE_BOOL)
                                                      : pqk::MODE_PLAIN);
                    d.dict = d.mode == pqk::MODE_DICT ? dict_dev : -1;
                    hpages.push_back(d);
                    c->page_seq.push_back(sq);
                    c->payload_bytes += psize;
                }
                p.first_row += row_base;
                if (nchunks > 1) c->walked.push_back(p);
            }
            rg.np = static_cast<int32_t>(hpages.size()) - rg.p0;
            c->ranges.push_back(rg);
            int64_t rows = 0;
            for (const auto& p : w.pages)
                if (p.page_type == PQ_DATA_PAGE) rows += p.num_values;
            row_base += rows;
            seq += static_cast<int64_t>(w.pages.size());
            if (w.error) {  // later chunks are never reached by the reference
                c->walk_error = w.error;
                c->walk_message = w.message;
                c->walk_error_seq = seq;
                break;
            }
        }
        if (nchunks == 1) c->walked = std::move(walks[0].pages);  // rows start at 0: the walk's table as is
        c->nrows = row_base;
        c->nbytes = static_cast<size_t>(img) + 64;
        sub_timer.reset(new HostTimed(ctx, "up_plan_fused"));
        plan_fused(ctx, c.get(), hpages, hdicts);
        sub_timer.reset(new HostTimed(ctx, "up_plan_pipe"));
        plan_pipe(ctx, c.get(), hpages, hdicts);
        sub_timer.reset(new HostTimed(ctx, "up_plan_plain"));
        plan_plain(ctx, c.get(), hpages);
        sub_timer.reset(new HostTimed(ctx, "up_plan_rest"));
        c->npages = static_cast<int>(hpages.size());
        c->ndicts = static_cast<int>(hdicts.size());

        // tiles
        PVec<DevTile>& htiles = ctx->s_htiles;
        PVec<int32_t>& tile0 = ctx->s_tile0;
        // per page range on host threads: tile counts, then the tiles at their
        // indices, with the chunk-wide flags reduced per range
        {
            const size_t NP = hpages.size();
            const int T = static_cast<int>(std::min<size_t>(static_cast<size_t>(hw_plan), std::max<size_t>(1, NP / 16384)));
            const size_t per = (NP + static_cast<size_t>(T) - 1) / static_cast<size_t>(T);
            struct TPart {
                size_t nt = 0;
                bool aligned = true, plain = true;
                uint32_t maxb = 0;
            };
            std::vector<TPart> tp(static_cast<size_t>(T));
            auto ntile = [](const DevPage& pg) {
                return static_cast<size_t>((std::max(pg.nvals, 0) + pqk::kTileRows - 1) / pqk::kTileRows);
            };
            pqfmt::parallel_run(T, T, [&](int t) {
                TPart& P = tp[static_cast<size_t>(t)];
                for (size_t p = static_cast<size_t>(t) * per; p < std::min(NP, (static_cast<size_t>(t) + 1) * per); p++) {
                    P.nt += ntile(hpages[p]);
                    P.maxb = std::max<uint32_t>(P.maxb, static_cast<uint32_t>(std::max(hpages[p].size, 0)));
                    P.plain &= hpages[p].mode == pqk::MODE_PLAIN;
                }
            });
            std::vector<size_t> tb(static_cast<size_t>(T));
            size_t nt = 0;
            for (int t = 0; t < T; t++) {
                tb[static_cast<size_t>(t)] = nt;
                nt += tp[static_cast<size_t>(t)].nt;
            }
            htiles.resize(nt);
            tile0.resize(NP);
            pqfmt::parallel_run(T, T, [&](int t) {
                TPart& P = tp[static_cast<size_t>(t)];
                size_t k = tb[static_cast<size_t>(t)];
                for (size_t p = static_cast<size_t>(t) * per; p < std::min(NP, (static_cast<size_t>(t) + 1) * per); p++) {
                    tile0[p] = static_cast<int32_t>(k);
                    const DevPage& pg = hpages[p];
                    for (int32_t r = 0; r < pg.nvals; r += pqk::kTileRows) {
                        htiles[k++] = DevTile{static_cast<int32_t>(p), r, std::min(pqk::kTileRows, pg.nvals - r), 0};
                        P.aligned &= ((pg.first_row + r) & 31) == 0;
                    }
                }
            });
            c->ntiles = static_cast<int>(nt);
            c->tiles_aligned32 = true;
            // every data page PLAIN, a fixed-width type whose bytes are copied as is
            c->fixed_plain = (c->type == PQ_INT32 || c->type == PQ_INT64 || c->type == PQ_FLOAT ||
                              c->type == PQ_DOUBLE || c->type == PQ_INT96) &&
                             c->width == c->plain_width && c->max_def >= 0 && c->max_rep >= 0;
            for (const auto& P : tp) {
                c->tiles_aligned32 &= P.aligned;
                c->max_page_bytes = std::max(c->max_page_bytes, P.maxb);
                c->fixed_plain &= P.plain;
            }
        }

        sub_timer.reset();
        plan_timer.reset();
        // 2) device allocations + one upload
        std::unique_ptr<HostTimed> alloc_timer(new HostTimed(ctx, "up_alloc"));
        int rc = 0;
        rc |= dalloc(&c->d_bytes, c->nbytes);
        rc |= dalloc(&c->d_pages, hpages.size());
        rc |= dalloc(&c->d_dicts, hdicts.size());
        rc |= dalloc(&c->d_tiles, htiles.size());
        rc |= dalloc(&c->d_page_tile0, tile0.size());
        rc |= dalloc(&c->d_entries, static_cast<size_t>(c->nentries));
        rc |= dalloc(&c->d_dict_count, hdicts.size());
        rc |= dalloc(&c->d_page_err, hpages.size());
        rc |= dalloc(&c->d_dict_err, hdicts.size());
        if (c->pipe) {  // flags | bsum | flist, cleared together
            // (bsum: pipe_grid k_pipe_write workgroup sums)
            const size_t fb = 4 * sizeof(int32_t), bb = static_cast<size_t>(c->pipe_grid) * sizeof(unsigned long long);
            c->z_bsum = fb;
            c->z_flist = (fb + bb + 15) / 16 * 16;
            // cleared per decode (through flist[0]): a multiple of 16 bytes (an
            // odd size takes a second fill kernel for the tail)
            const size_t zb = (c->z_flist + sizeof(int32_t) + 15) / 16 * 16;
            // two such blocks: a decode uses one while its k_pipe_write clears
            // the other for the next decode (no fill kernel per decode)
            const size_t zfull = (std::max(zb, c->z_flist + (hpages.size() + 1) * sizeof(int32_t)) + 255) / 256 * 256;
            rc |= dalloc(&c->d_zero, 2 * zfull);
            if (c->d_zero) {
                c->zfull = zfull;
                c->zsel = 0;
                c->d_flags = reinterpret_cast<int32_t*>(c->d_zero);
                c->d_bsum = reinterpret_cast<unsigned long long*>(c->d_zero + c->z_bsum);
                c->d_flist = reinterpret_cast<int32_t*>(c->d_zero + c->z_flist);
                c->zero_bytes = zb;
            }
        } else {
            rc |= dalloc(&c->d_flags, 4);
        }
        if (c->pipe && !hdicts.empty()) rc |= dalloc(&c->d_dflag, 1);
        {
            size_t off = 0;
            for (size_t i = 0; i < hdicts.size(); i++) {
                const uint32_t sz = static_cast<uint32_t>(std::max(hdicts[i].size, 0));
                if (static_cast<uint64_t>(sz) + 32 <= pqk::kDictLdsCap) continue;
                pq_chunk::BigDict b{static_cast<int>(i), hdicts[i], off, 0, 0};
                off += (pqk::dict_big_scratch(sz) + 255) / 256 * 256;
                // (a dictionary holds at most size / 4 + 1 entries: a corrupt
                // header count must not size these buffers)
                const size_t nv = static_cast<size_t>(std::min<int64_t>(std::max(hdicts[i].nvals, 0), sz / 4 + 1));
                b.lens_off = off;  // entry lengths as bytes (+ 16: k_wide_chars stages whole blocks)
                off += (nv + 16 + 255) / 256 * 256;
                b.pad_off = off;   // 16-byte entry slots (k_pipe_wwide)
                off += (nv * 16 + 255) / 256 * 256;
                c->hbigd.push_back(b);
            }
            if (off) rc |= dalloc(&c->d_bigd, off);
        }
        rc |= dalloc(&c->d_tile_chars, htiles.size());
        if (c->fixed_plain || c->plain_opt) {
            rc |= dalloc(&c->d_tile_rank, htiles.size());
            rc |= dalloc(&c->d_page_pos, hpages.size());
        }
        if (c->plain_opt) {
            const size_t np = hpages.size();
            rc |= dalloc(&c->d_page_nn, np);
            rc |= dalloc(&c->d_onnv, np);
            rc |= dalloc(&c->d_ochv, np);
            rc |= dalloc(&c->d_opdense, np);
            rc |= dalloc(&c->d_opbase, np);
            rc |= dalloc(&c->d_otot, 2);
            rc |= dalloc(&c->d_vpages, np);
            rc |= dalloc(&c->d_doffs, static_cast<size_t>(c->nrows) + 1);
            rc |= dalloc(&c->d_operr, np);
            if (!c->hpwpage.empty()) rc |= dalloc(&c->d_pwpage, c->hpwpage.size());
        }
        rc |= dalloc(&c->d_tile_base, htiles.size());
        rc |= dalloc(&c->d_total, 1);
        rc |= dalloc(&c->d_scan_scratch, std::max(htiles.size(), hpages.size()) / 8192 + 16);
        if (c->type == PQ_BYTE_ARRAY && !c->fused) rc |= dalloc(&c->d_row_codes, static_cast<size_t>(c->nrows));
        if (c->pipe) {
            rc |= dalloc(&c->d_runs, hpages.size() * 2 * pqk::kPipeRunCap);
            rc |= dalloc(&c->d_info, hpages.size());
            // u16 codes, or u32 on the wide pipe (d_codes then holds 2 per row)
            rc |= dalloc(&c->d_codes, static_cast<size_t>(c->nrows) * (c->pipe_wide ? 2 : 1) + 64);
            rc |= dalloc(&c->d_tile_nn, htiles.size());
            if (!c->hbig.empty()) rc |= dalloc(&c->d_bigp, c->hbig.size());
        }
        if (c->plain) {
            rc |= dalloc(&c->d_pwins, c->hpwins.size());
            if (!c->hpwbase.empty()) rc |= dalloc(&c->d_pwbase, c->hpwbase.size());
            rc |= dalloc(&c->d_rowinfo, static_cast<size_t>(c->nrows) + 64);
            rc |= dalloc(&c->d_wchars, c->hpwins.size());
            rc |= dalloc(&c->d_pbsum, static_cast<size_t>(c->plain_grid));
            if (c->plain_spec) {
                const size_t nch = c->hchunks.size();
                rc |= dalloc(&c->d_chunk_base, c->hchunk_base.size());
                rc |= dalloc(&c->d_chunks, nch);
                rc |= dalloc(&c->d_cand, nch * pqk::kPCand);
                rc |= dalloc(&c->d_ppages, nch);
                rc |= dalloc(&c->d_perr, nch);
            }
        }
        if (c->fused) {
            rc |= dalloc(&c->d_status, hpages.size());
            rc |= dalloc(&c->d_tickets, c->ranges.size());
            rc |= dalloc(&c->d_bases, c->ranges.size() + 1);
        }
        if (rc) {
            free_chunk_device(c.get());
            return set_err(ctx, PQ_ERR_HIP, "hipMalloc failed (chunk upload)");
        }
        // payload bytes into their 16-byte slots, zero padding in between and
        // past EOF: written piece by piece straight into pinned buffers by host
        // threads while earlier pieces are in flight to HBM
        alloc_timer.reset();
        HostTimed h2d_timer(ctx, "up_h2d");
        hipStream_t s = ctx->copy;
        const int hw = static_cast<int>(std::min(16u, std::max(1u, std::thread::hardware_concurrency())));
        const int64_t img_end = img;
        auto fill_image = [&](uint8_t* dst, size_t a, size_t z) {
            // first payload whose slot ends after a (slots are in image order)
            size_t k = static_cast<size_t>(std::upper_bound(copies.begin(), copies.end(), static_cast<int64_t>(a),
                                                            [](int64_t v, const std::pair<int64_t, int64_t>& cp) {
                                                                return v < cp.second;
                                                            }) - copies.begin());
            k = k ? k - 1 : 0;
            size_t at = a;
            for (; k < copies.size() && at < z; k++) {
                const int64_t s0 = copies[k].second;
                const int64_t n = copy_size[k];
                const int64_t s1 = s0 + (n + 15) / 16 * 16 + 16;  // slot end
                if (static_cast<size_t>(s1) <= at) continue;
                if (static_cast<size_t>(s0) > at) {  // (no gaps between slots; defensive)
                    const size_t g = std::min(z, static_cast<size_t>(s0)) - at;
                    std::memset(dst + (at - a), 0, g);
                    at += g;
                    if (at >= z) break;
                }
                // payload part [s0, s0 + avail) from the file, rest of the slot zero
                // (codec pages, lo < 0: all zero until the codec pass)
                const int64_t lo = copies[k].first;
                const int64_t avail = lo < 0 ? 0 : std::max<int64_t>(0, std::min<int64_t>(n, static_cast<int64_t>(file_len) - lo));
                const size_t pe = static_cast<size_t>(s0 + avail), se = std::min(z, static_cast<size_t>(s1));
                if (at < pe) {
                    const size_t e = std::min(se, pe);
                    std::memcpy(dst + (at - a), file + lo + (static_cast<int64_t>(at) - s0), e - at);
                    at = e;
                }
                if (at < se) {
                    std::memset(dst + (at - a), 0, se - at);
                    at = se;
                }
            }
            if (at < z) std::memset(dst + (at - a), 0, z - at);  // image tail (past img_end)
            (void)img_end;
        };
        bool relaid = false;
        if (raw && raw->active) {
            raw->join();  // the raw bytes are in HBM (the ring is free again)
            if (raw->err != hipSuccess) {
                rc = hip_check(ctx, raw->err, "raw upload");
            } else {
                PVec<pqk::RelayoutEntry>& ents = ctx->s_ents;
                ents.resize(copies.size());
                std::atomic<bool> inside_all{true};
                {
                    const size_t NC = copies.size();
                    const int T = static_cast<int>(std::min<size_t>(static_cast<size_t>(hw_plan), std::max<size_t>(1, NC / 16384)));
                    const size_t per = (NC + static_cast<size_t>(T) - 1) / static_cast<size_t>(T);
                    pqfmt::parallel_run(T, T, [&](int t) {
                        size_t e = 0;
                        for (size_t k = static_cast<size_t>(t) * per; k < std::min(NC, (static_cast<size_t>(t) + 1) * per); k++) {
                            const int64_t lo = copies[k].first, n = copy_size[k];
                            const int64_t avail = lo < 0 ? 0 : std::max<int64_t>(0, std::min<int64_t>(n, static_cast<int64_t>(file_len) - lo));
                            pqk::RelayoutEntry r{};
                            r.dst = static_cast<uint64_t>(copies[k].second);
                            r.avail = static_cast<uint32_t>(avail);
                            r.slot = static_cast<uint32_t>((n + 15) / 16 * 16 + 16);
                            if (avail > 0) {  // the extent holding the payload (extents and payloads both ascend, mostly)
                                auto in = [&](size_t j) {
                                    return lo >= raw->ext[j].first && lo + avail <= raw->ext[j].first + raw->ext[j].second;
                                };
                                if (!in(e)) {
                                    size_t j = 0;
                                    while (j < raw->ext.size() && !in(j)) j++;
                                    if (j == raw->ext.size()) {
                                        inside_all = false;
                                        return;
                                    }
                                    e = j;
                                }
                                r.src = static_cast<uint64_t>(raw->base[e] + (lo - raw->ext[e].first));
                            }
                            ents[k] = r;
                        }
                    });
                }
                const bool inside = inside_all;
                if (inside) {
                    const size_t need = std::max<size_t>(ents.size(), 1);
                    if (ctx->relay_cap < need) {
                        dfree(ctx->d_relay);
                        ctx->relay_cap = 0;
                        if (dalloc(&ctx->d_relay, need) == 0) ctx->relay_cap = need;
                    }
                    if (ctx->relay_cap >= need) {
                        rc = hip_check(ctx, hipMemcpyAsync(ctx->d_relay, ents.data(), ents.size() * sizeof(pqk::RelayoutEntry),
                                                           hipMemcpyHostToDevice, s),
                                       "upload");
                        if (!rc) {
                            {
                                Timed rt(ctx, "relayout", s);
                                pqk::launch_relayout(s, ctx->d_raw, c->d_bytes, ctx->d_relay, static_cast<int32_t>(ents.size()));
                            }
                            (void)hipMemsetAsync(c->d_bytes + img, 0, c->nbytes - static_cast<size_t>(img), s);
                            relaid = true;
                        }
                    }
                }
            }
        }
        if (!rc && !relaid)
            rc = hip_check(ctx, ctx->stager.upload(c->d_bytes, c->nbytes, s, copies.size() > 64 ? hw : 1, fill_image,
                                                   ctx->opt_stage_streams > 1 ? ctx->copy2 : nullptr),
                           "upload");
        // compressed / DATA_PAGE_V2 pages: their payloads
        // (in d_raw when the raw path holds them, else gathered and uploaded)
        // are rebuilt into their slots by the codec pass (codec.hip)
        if (!rc && !cents.empty()) {
            const uint8_t* csrc = nullptr;
            bool in_raw = relaid && raw && raw->active;
            for (size_t k = 0, e = 0; k < cents.size() && in_raw; k++) {
                const int64_t lo = cent_file[k], n = cents[k].src_len;
                auto in = [&](size_t j) {
                    return lo >= raw->ext[j].first && lo + n <= raw->ext[j].first + raw->ext[j].second;
                };
                if (!in(e)) {
                    size_t j = 0;
                    while (j < raw->ext.size() && !in(j)) j++;
                    if (j == raw->ext.size()) { in_raw = false; break; }
                    e = j;
                }
                cents[k].src = static_cast<uint64_t>(raw->base[e] + (lo - raw->ext[e].first));
            }
            if (in_raw) {
                csrc = ctx->d_raw;
            } else {  // gather the payloads, each 16-byte aligned
                std::vector<int64_t> at(cents.size());
                int64_t tot = 0;
                for (size_t k = 0; k < cents.size(); k++) {
                    at[k] = tot;
                    cents[k].src = static_cast<uint64_t>(tot);
                    tot += (static_cast<int64_t>(cents[k].src_len) + 15) / 16 * 16;
                }
                const size_t need = static_cast<size_t>(tot) + 64;
                if (ctx->zsrc_cap < need) {
                    dfree(ctx->d_zsrc);
                    ctx->zsrc_cap = 0;
                    if (dalloc(&ctx->d_zsrc, need) == 0) ctx->zsrc_cap = need;
                }
                if (ctx->zsrc_cap < need) rc = set_err(ctx, PQ_ERR_HIP, "hipMalloc failed (compressed pages)");
                if (!rc)
                    rc = hip_check(ctx, ctx->stager.upload(ctx->d_zsrc, need, s, cents.size() > 64 ? hw : 1,
                                                           [&](uint8_t* dst, size_t a, size_t z) {
                        size_t k = static_cast<size_t>(std::upper_bound(at.begin(), at.end(), static_cast<int64_t>(a)) - at.begin());
                        k = k ? k - 1 : 0;
                        std::memset(dst, 0, z - a);
                        for (; k < cents.size() && static_cast<size_t>(at[k]) < z; k++) {
                            const size_t b0 = static_cast<size_t>(at[k]), b1 = b0 + cents[k].src_len;
                            const size_t x0 = std::max(a, b0), x1 = std::min(z, b1);
                            if (x0 < x1) std::memcpy(dst + (x0 - a), file + cent_file[k] + (x0 - b0), x1 - x0);
                        }
                    }), "upload");
                csrc = ctx->d_zsrc;
            }
            const size_t n = cents.size();
            if (!rc && ctx->codec_cap < n) {
                dfree(ctx->d_codec);
                dfree(ctx->d_codec_st);
                ctx->codec_cap = 0;
                if (dalloc(&ctx->d_codec, n) == 0 && dalloc(&ctx->d_codec_st, n) == 0) ctx->codec_cap = n;
                else rc = set_err(ctx, PQ_ERR_HIP, "hipMalloc failed (compressed pages)");
            }
            if (!rc)
                rc = hip_check(ctx, ctx->stager.upload(reinterpret_cast<uint8_t*>(ctx->d_codec), n * sizeof(pqk::CodecEntry), s, 1,
                                                       [&](uint8_t* dst, size_t a, size_t z) {
                                                           std::memcpy(dst, reinterpret_cast<const uint8_t*>(cents.data()) + a, z - a);
                                                       }),
                               "upload");
            if (!rc) {
                // every status word starts non-OK: an entry the pass never
                // reached (a failed launch) cannot read as a clean decode
                rc = hip_check(ctx, hipMemsetAsync(ctx->d_codec_st, 0xFF, n * sizeof(uint32_t), s), "codec status");
            }
            if (!rc) {
                Timed ct(ctx, "codec", s);
                const bool gz = std::any_of(cents.begin(), cents.end(), [](const pqk::CodecEntry& e) { return e.codec == 2; });
                const bool other = std::any_of(cents.begin(), cents.end(), [](const pqk::CodecEntry& e) { return e.codec != 2 && e.codec != 0; });
                const bool zstd = std::any_of(cents.begin(), cents.end(), [](const pqk::CodecEntry& e) { return e.codec == 6; });
                const bool zother = std::any_of(cents.begin(), cents.end(), [](const pqk::CodecEntry& e) { return e.codec != 6 && e.codec != 0; });
                if (gz && other) {
                    rc = set_err(ctx, PQ_ERR_CODEC, "GZIP pages mixed with other codecs in one upload");
                } else if (zstd && zother) {
                    rc = set_err(ctx, PQ_ERR_CODEC, "ZSTD pages mixed with other codecs in one upload");
                } else {
                    const int32_t nsmall = static_cast<int32_t>(std::count_if(
                        cents.begin(), cents.end(), [](const pqk::CodecEntry& e) { return e.out_len < pqk::codec_small_bytes(); }));
                    pqk::launch_codec(s, csrc, c->d_bytes, ctx->d_codec, static_cast<int32_t>(n), ctx->d_codec_st, ctx->cus,
                                      gz ? 1 : (zstd ? 2 : 0), nsmall);
                    rc = hip_check(ctx, hipGetLastError(), "codec launch");
                }
            }
        }
        if (ctx->timing) {
            auto& f = ctx->timers["up_fill"];
            f.first += ctx->stager.fill_ms;
            f.second += 1;
            auto& w = ctx->timers["up_wait"];
            w.first += ctx->stager.wait_ms;
            w.second += 1;
        }
        auto put = [&](void* d, const void* h, size_t bytes) {
            if (rc || bytes == 0) return;
            rc = hip_check(ctx, ctx->stager.upload(static_cast<uint8_t*>(d), bytes, s, bytes > (32u << 20) ? hw : 1,
                                                   [&](uint8_t* dst, size_t a, size_t z) {
                                                       std::memcpy(dst, static_cast<const uint8_t*>(h) + a, z - a);
                                                   }),
                           "upload");
        };
        auto put_pinned = [&](void* d, const void* h, size_t bytes) {
            if (rc || bytes == 0) return;
            rc = hip_check(ctx, hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s), "upload");
        };
        put_pinned(c->d_pages, hpages.data(), hpages.size() * sizeof(DevPage));
        put(c->d_dicts, hdicts.data(), hdicts.size() * sizeof(DevDict));
        put_pinned(c->d_tiles, htiles.data(), htiles.size() * sizeof(DevTile));
        put_pinned(c->d_page_tile0, tile0.data(), tile0.size() * sizeof(int32_t));
        if (!rc) (void)hipMemsetAsync(c->d_page_err, 0, std::max<size_t>(hpages.size(), 1) * sizeof(DevErr), s);
        if (!rc) (void)hipMemsetAsync(c->d_dict_err, 0, std::max<size_t>(hdicts.size(), 1) * sizeof(DevErr), s);
        if (!rc && c->d_dflag) (void)hipMemsetAsync(c->d_dflag, 0, sizeof(int32_t), s);
        if (!rc && c->d_zero) {
            (void)hipMemsetAsync(c->d_zero, 0, 2 * c->zfull, s);
            c->next_zeroed = true;
        }
        if (!rc && c->d_chunks) {
            put(c->d_chunks, c->hchunks.data(), c->hchunks.size() * sizeof(uint2));
            put(c->d_chunk_base, c->hchunk_base.data(), c->hchunk_base.size() * sizeof(int32_t));
            if (!rc) (void)hipMemsetAsync(c->d_perr, 0, c->hchunks.size() * sizeof(DevErr), s);
        }
        if (c->d_bigp) put(c->d_bigp, c->hbig.data(), c->hbig.size() * sizeof(int32_t));
        if (c->d_pwins) put(c->d_pwins, c->hpwins.data(), c->hpwins.size() * sizeof(pqk::DevBatch));
        if (c->d_pwbase) put(c->d_pwbase, c->hpwbase.data(), c->hpwbase.size() * sizeof(int64_t));
        if (c->d_pwpage) put(c->d_pwpage, c->hpwpage.data(), c->hpwpage.size() * sizeof(int32_t));
        {  // (also after an error: the pinned tables may still be in flight)
            const hipError_t e = hipStreamSynchronize(s);
            if (!rc) rc = hip_check(ctx, e, "upload sync");
        }
        if (!rc && !cents.empty()) {
            std::vector<uint32_t> st(cents.size());
            rc = hip_check(ctx, hipMemcpy(st.data(), ctx->d_codec_st, st.size() * sizeof(uint32_t), hipMemcpyDeviceToHost),
                           "codec status");
            for (size_t k = 0; k < st.size() && !rc; k++) {
                if (!st[k]) continue;
                static const char* what[] = {"", "corrupt compressed data", "decompressed size differs from the page header",
                                             "unsupported codec", "decompression pass did not run"};
                rc = set_err(ctx, PQ_ERR_DECOMPRESS,
                             "page at file offset " + std::to_string(cent_file[k]) + " (codec " +
                                 std::to_string(cents[k].codec) + "): " + what[std::min<uint32_t>(st[k], 4)]);
            }
        }
        if (rc) {
            free_chunk_device(c.get());
            return rc;
        }
        // output size estimate for BYTE_ARRAY chars: plain pages are bounded
        // by their payload; dictionary pages by rows x mean entry length.
        int64_t est = 0;
        for (const auto& p : hpages) {
            if (p.mode == pqk::MODE_DICT) {
                const DevDict& d = hdicts[p.dict];
                int64_t mean = d.nvals > 0 ? (d.size / d.nvals) + 1 : 1;
                est += static_cast<int64_t>(p.nvals) * mean;
            } else {
                est += p.size;
            }
        }
        c->char_estimate = est + est / 8 + 64;
        *out = c.release();
        return 0;
    } catch (const pqfmt::Error& e) {
        return set_err(ctx, e.code, e.what());
    } catch (const std::exception& e) {
        return set_err(ctx, PQ_ERR_ALLOC, e.what());
    }
}

int pq_chunk_upload(pq_ctx* ctx, const uint8_t* file, size_t file_len, const pq_chunk_desc* chunks,
                    int nchunks, pq_chunk** out) {
    if (!ctx || !file || !chunks || nchunks <= 0 || !out) return PQ_ERR_ARG;
    DevGuard dg(ctx);
    *out = nullptr;
    try {
        // the chunks' page walks are independent: host threads
        std::vector<pqfmt::WalkResult> walks(static_cast<size_t>(nchunks));
        const int hw = static_cast<int>(std::min(16u, std::max(1u, std::thread::hardware_concurrency())));
        const int per = std::max(1, hw / nchunks);  // threads per chunk walk
        // chunk extents known from the footer: their bytes start for HBM now
        RawStage raw;
        bool extents = true;
        for (int k = 0; k < nchunks && extents; k++) {
            int64_t lo = chunks[k].data_page_offset;
            if (chunks[k].has_dictionary_page_offset) lo = std::min(lo, chunks[k].dictionary_page_offset);
            extents = chunks[k].total_compressed_size > 0 && lo >= 0;
            raw.ext.push_back({lo, chunks[k].total_compressed_size});
        }
        if (extents) raw_start(ctx, file, file_len, raw);
        {
            HostTimed ht(ctx, "up_walk");
            // option device_walk: the page walk on the GPU over the raw bytes
            // once they are in HBM (walk.hip); a chunk it refuses (or any
            // chunk the raw upload does not cover) walks on the host, which
            // also reports the reference's errors
            std::vector<char> done(static_cast<size_t>(nchunks), 0);
            if (ctx->opt_dev_walk && raw.active) {
                raw.join();
                if (raw.err == hipSuccess) {
                    for (int k = 0; k < nchunks; k++) {
                        int64_t np = 0;
                        pqfmt::WalkResult& w = walks[static_cast<size_t>(k)];
                        const int rc = device_walk(ctx, ctx->d_raw + raw.base[static_cast<size_t>(k)],
                                                   static_cast<size_t>(raw.ext[static_cast<size_t>(k)].second),
                                                   raw.ext[static_cast<size_t>(k)].first, &chunks[k], 0, 0, &np,
                                                   [&](const pq_page_desc* h, size_t n) { w.pages.assign(h, h + n); });
                        done[static_cast<size_t>(k)] = rc == 0;
                    }
                }
            }
            parallel_for(nchunks, [&](int k) {
                if (!done[static_cast<size_t>(k)]) walks[static_cast<size_t>(k)] = pqfmt::walk_chunk(file, file_len, chunks[k], per);
            });
        }
        return upload_walked(ctx, file, file_len, chunks[0], walks, 0, out, &raw);
    } catch (const std::exception& e) {
        return set_err(ctx, PQ_ERR_ALLOC, e.what());
    }
}

int pq_chunk_upload_range(pq_ctx* ctx, const uint8_t* file, size_t file_len, const pq_chunk_desc* chunk,
                          const pq_page_desc* table, int64_t ntable, int64_t data_begin, int64_t data_end,
                          pq_chunk** out) {
    if (!ctx || !file || !chunk || (!table && ntable) || ntable < 0 || !out || data_begin < 0 ||
        data_end < data_begin)
        return PQ_ERR_ARG;
    DevGuard dg(ctx);
    *out = nullptr;
    try {
        // the data pages of the range, in walk order, and the dictionary pages they use
        std::vector<int64_t> data_idx;
        int64_t k = 0, row0 = -1, rows_before = 0;  // row0: chunk row of data page `data_begin`
        for (int64_t i = 0; i < ntable; i++) {
            if (table[i].page_type != PQ_DATA_PAGE) continue;
            if (k == data_begin) row0 = table[i].first_row;
            if (k >= data_begin && k < data_end) data_idx.push_back(i);
            rows_before = table[i].first_row + table[i].num_values;
            k++;
        }
        if (row0 < 0) row0 = rows_before;  // empty range at the end
        if (data_end > k) return set_err(ctx, PQ_ERR_ARG, "page range past the chunk's data pages");
        std::vector<int32_t> remap(static_cast<size_t>(ntable), -1);
        pqfmt::WalkResult w;
        for (int64_t i : data_idx) {
            const int32_t d = table[i].dict_page;
            if (d < 0) continue;
            if (d >= ntable || d >= i || table[d].page_type != PQ_DICTIONARY_PAGE)
                return set_err(ctx, PQ_ERR_ARG, "page table: bad dictionary page index");
            remap[static_cast<size_t>(d)] = 0;
        }
        for (int64_t i = 0; i < ntable; i++)  // dictionary pages first, in walk order
            if (remap[static_cast<size_t>(i)] == 0) {
                remap[static_cast<size_t>(i)] = static_cast<int32_t>(w.pages.size());
                w.pages.push_back(table[i]);
            }
        for (int64_t i : data_idx) {
            pq_page_desc p = table[i];
            p.first_row -= row0;
            if (p.dict_page >= 0) p.dict_page = remap[static_cast<size_t>(p.dict_page)];
            w.pages.push_back(p);
        }
        // extents: each page's header + payload, contiguous runs merged
        RawStage raw;
        for (const auto& p : w.pages) {
            const int64_t lo = p.header_offset, hi = p.payload_offset + std::max(p.payload_size, 0);
            if (!raw.ext.empty() && raw.ext.back().first + raw.ext.back().second == lo)
                raw.ext.back().second += hi - lo;
            else
                raw.ext.push_back({lo, hi - lo});
        }
        raw_start(ctx, file, file_len, raw);
        std::vector<pqfmt::WalkResult> walks(1);
        walks[0] = std::move(w);
        return upload_walked(ctx, file, file_len, *chunk, walks, row0, out, &raw);
    } catch (const std::exception& e) {
        return set_err(ctx, PQ_ERR_ALLOC, e.what());
    }
}

void pq_chunk_free(pq_ctx* ctx, pq_chunk* c) {
    if (!c) return;
    DevGuard dg(ctx);
    if (ctx) (void)hipStreamSynchronize(ctx->stream);
    free_chunk_device(c);
    delete c;
}

int64_t pq_chunk_num_rows(const pq_chunk* c) { return c ? c->nrows : 0; }
int64_t pq_chunk_first_row(const pq_chunk* c) { return c ? c->row_offset : 0; }
int64_t pq_chunk_num_pages(const pq_chunk* c) { return c ? c->npages : 0; }
int64_t pq_chunk_payload_bytes(const pq_chunk* c) { return c ? c->payload_bytes : 0; }
int pq_chunk_pages(const pq_chunk* c, pq_page_desc* pages, int64_t cap, int64_t* npages) {
    if (!c || !npages) return PQ_ERR_ARG;
    *npages = static_cast<int64_t>(c->walked.size());
    for (int64_t i = 0; i < cap && i < *npages; i++) pages[i] = c->walked[i];
    return 0;
}

static int ensure_output(pq_ctx* ctx, pq_chunk* c, pq_column* out, int64_t char_cap) {
    int64_t rows_needed = c->nrows;
    int64_t bytes_needed = c->type == PQ_BYTE_ARRAY ? char_cap : c->nrows * c->width;
    if (out->capacity_rows < rows_needed + 1 || out->d_validity == nullptr) {
        dfree(out->d_validity);
        dfree(out->d_offsets);
        int64_t cap = rows_needed + 1;
        if (dalloc(&out->d_validity, static_cast<size_t>(cap / 32 + 4)))
            return set_err(ctx, PQ_ERR_HIP, "hipMalloc failed (validity)");
        if (c->type == PQ_BYTE_ARRAY && dalloc(&out->d_offsets, static_cast<size_t>(cap)))
            return set_err(ctx, PQ_ERR_HIP, "hipMalloc failed (offsets)");
        out->capacity_rows = cap;
    }
    if (c->type == PQ_BYTE_ARRAY && out->d_offsets == nullptr) {
        if (dalloc(&out->d_offsets, static_cast<size_t>(out->capacity_rows)))
            return set_err(ctx, PQ_ERR_HIP, "hipMalloc failed (offsets)");
    }
    if (out->capacity_bytes < bytes_needed || out->d_values == nullptr) {
        dfree(out->d_values);
        if (dalloc(&out->d_values, static_cast<size_t>(bytes_needed + 64)))
            return set_err(ctx, PQ_ERR_HIP, "hipMalloc failed (values)");
        out->capacity_bytes = bytes_needed;
    }
    out->num_rows = c->nrows;
    out->type = c->type;
    out->value_width = c->type == PQ_BYTE_ARRAY ? 0 : c->width;
    return 0;
}

static void launch_gather(pq_ctx* ctx, pq_chunk* c, pq_column* out) {
    Timed t(ctx, "ba_gather");
    pqk::launch_ba_gather(ctx->stream, c->d_bytes, c->d_pages, c->d_tiles, c->ntiles, c->d_dicts,
                          c->d_entries, c->d_row_codes, c->d_tile_base, c->nrows, c->d_total,
                          out->capacity_bytes, c->d_flags + 1, out->d_validity, out->d_offsets,
                          out->d_values, !ctx->opt_gather_rows);
}

// Launch parameters of the three-pass dictionary path (dict_pipe.hip); `out`
// may be null when only the codes are wanted (regex page filter).
static pqk::PipeLaunch pipe_launch(pq_ctx* ctx, pq_chunk* c, pq_column* out) {
    pqk::PipeLaunch P{};
    P.bytes = c->d_bytes; P.pages = c->d_pages; P.npages = c->npages; P.tiles = c->d_tiles;
    P.ntiles = c->ntiles; P.page_tile0 = c->d_page_tile0; P.max_def = c->max_def; P.max_rep = c->max_rep;
    P.dicts = c->d_dicts; P.dict_id = c->pipe_dict; P.entries = c->d_entries; P.dict_count = c->d_dict_count;
    P.runs = c->d_runs; P.info = c->d_info; P.flist = c->d_flist; P.tile_nn = c->d_tile_nn; P.codes = c->d_codes;
    if (c->pipe_wide) {
        P.codes32 = reinterpret_cast<uint32_t*>(c->d_codes);
        P.codes = nullptr;
        for (const auto& b : c->hbigd)
            if (b.di == c->pipe_dict) {
                P.lens8 = c->d_bigd + b.lens_off;
                P.lens8_cap = static_cast<uint32_t>(std::min<int64_t>(std::max(b.d.nvals, 0), b.d.size / 4 + 1));
                P.pad16 = reinterpret_cast<const uint4*>(c->d_bigd + b.pad_off);
            }
    }
    P.tile_chars = c->d_tile_chars; P.bsum = c->d_bsum; P.total = c->d_total;
    P.nrows_total = c->nrows; P.overflow = c->d_flags + 1;
    if (out) {
        P.capacity = out->capacity_bytes;
        P.validity = out->d_validity; P.offsets = out->d_offsets; P.chars = out->d_values;
    }
    P.page_err = c->d_page_err; P.err_any = c->d_flags;
    P.dict_chars_bytes = c->pipe_dict_chars_bytes; P.dict_bytes = c->pipe_dict_bytes; P.lds = c->pipe_lds;
    P.grid = c->pipe_grid;
    P.debug = ctx->opt_debug;
    P.dict_entries_cap = c->pipe_ecap;
    P.cus = c->pipe_cus;
    P.has_small = c->pipe_small;
    P.write_waves = c->pipe_wpw;
    return P;
}

// Run tables and per-row codes (k_pipe_runs, k_pipe_big, k_pipe_codes3; the
// exact decoder for pages outside the fast shape).  With dict_on_side the
// dictionary decodes on ctx->side and the codes wait for it (ev_join).
// With dict_in_runs the dictionary pages decode in k_pipe_runs' leading
// workgroups (same launch, main stream: ordered after the previous decode's
// readers of the entry table, no side-stream events).
// k_dict_index for every dictionary page of a BYTE_ARRAY chunk, and the
// multi-workgroup index for pages too large for its LDS.
static void launch_dicts(pq_chunk* c, hipStream_t s, int32_t* err_any) {
    if (c->hbigd.size() < static_cast<size_t>(c->ndicts))  // k_dict_index leaves the large pages alone
        pqk::launch_dict_index(s, c->d_bytes, c->d_dicts, c->ndicts, c->d_entries, c->d_dict_count, c->d_dict_err, err_any,
                           c->max_dict_bytes);
    for (const auto& b : c->hbigd)
        pqk::launch_dict_big(s, c->d_bytes + b.d.off, static_cast<uint32_t>(b.d.size), static_cast<uint32_t>(std::max(b.d.nvals, 0)),
                             c->d_entries + b.d.entry_base, c->d_bigd + b.lens_off,
                             reinterpret_cast<uint4*>(c->d_bigd + b.pad_off), c->d_dict_count + b.di,
                             c->d_dict_err + b.di, err_any, reinterpret_cast<uint32_t*>(c->d_bigd + b.scr_off));
}

static void pipe_front(pq_ctx* ctx, pq_chunk* c, const pqk::PipeLaunch& P, bool dict_on_side, bool dict_in_runs) {
    hipStream_t s = ctx->stream;
    {
        Timed t(ctx, "pipe_runs");
        const pqk::RunDicts rd{c->d_dicts, c->ndicts, c->d_entries, c->d_dict_count, c->d_dict_err, c->d_dflag};
        pqk::launch_pipe_runs(s, c->d_bytes, c->d_pages, c->pipe_small ? c->npages : 0, c->max_def, c->max_rep,
                              c->d_runs, c->d_info, ctx->opt_run_pages, c->d_flist,  // flist[0], bsum: cleared with d_flags
                              ctx->opt_debug, dict_in_runs ? &rd : nullptr, 0u,
                              (c->pipe_small_bytes + 15) / 16 * 16 + 16, c->max_dict_bytes, ctx->cus);
    }
    // the wide pipe's k_pipe_big writes raw indices and needs no dictionary:
    // it runs beside the dictionary's decode, k_wide_chars after both
    if (dict_on_side && c->ndicts && !c->pipe_wide) (void)hipStreamWaitEvent(s, ctx->ev_join, 0);
    if (!c->hbig.empty()) {
        Timed t(ctx, "pipe_big");
        pqk::launch_pipe_big(s, P, c->d_bigp, static_cast<int>(c->hbig.size()), c->big_max_bytes);
    }
    if (c->pipe_wide) {
        if (dict_on_side && c->ndicts) (void)hipStreamWaitEvent(s, ctx->ev_join, 0);
        Timed t(ctx, "wide_chars");
        pqk::launch_wide_chars(s, P);
    }
    if (c->pipe_count) {
        Timed t(ctx, "pipe_count");
        pqk::launch_pipe_codes(s, P, true);
    }
    Timed t(ctx, "pipe_codes");
    pqk::launch_pipe_codes(s, P, false);
}

static int decode_launch(pq_ctx* ctx, pq_chunk* c, pq_column* out);

int pq_decode_async(pq_ctx* ctx, pq_chunk* c, pq_column* out) {
    if (!ctx || !c || !out) return PQ_ERR_ARG;
    DevGuard dg(ctx);
    if (c->type == PQ_BYTE_ARRAY) {
        int64_t cap = std::max<int64_t>(out->capacity_bytes, c->char_estimate);
        if (int rc = ensure_output(ctx, c, out, cap)) return rc;
    } else {
        if (int rc = ensure_output(ctx, c, out, 0)) return rc;
    }
    c->last_out = out;
    return decode_launch(ctx, c, out);
}

static int decode_launch(pq_ctx* ctx, pq_chunk* c, pq_column* out) {
    hipStream_t s = ctx->stream;
    pqk::ColumnParams cp{c->type, c->max_def, c->max_rep, c->width, c->plain_width};
    const bool pipe = c->pipe && ctx->opt_pipe;
    // k_pipe_write stores whole validity words when every tile starts on a
    // 32-row boundary; other paths OR bits into zeroed words
    // OPTIONAL chunks take the PLAIN kernels only in their one-pass form
    const bool plain_go = c->plain && ctx->opt_plain && !(c->plain_spec && c->spec_failed) &&
                          !(c->plain_opt && (c->popt_failed || !ctx->opt_plain_fused));
    const bool pipe_path = pipe && !plain_go;
    if (pipe_path) c->codes_pending = true;
    if (c->ndicts && c->type == PQ_BYTE_ARRAY) c->entries_pending = true;
    if (pipe_path && c->d_zero && ctx->opt_zflip) {
        // flags, bsum and flist[0] of this decode: the other block, which the
        // previous decode's k_pipe_write cleared (else one fill)
        c->zsel ^= 1;
        uint8_t* zb = c->d_zero + static_cast<size_t>(c->zsel) * c->zfull;
        c->d_flags = reinterpret_cast<int32_t*>(zb);
        c->d_bsum = reinterpret_cast<unsigned long long*>(zb + c->z_bsum);
        c->d_flist = reinterpret_cast<int32_t*>(zb + c->z_flist);
        if (!c->next_zeroed) (void)hipMemsetAsync(c->d_flags, 0, c->zero_bytes, s);
        c->next_zeroed = false;
    } else {
        (void)hipMemsetAsync(c->d_flags, 0, c->zero_bytes, s);  // pipe chunks: flags, bsum and flist[0] at once
    }
    if (!(pipe_path && c->tiles_aligned32))
        (void)hipMemsetAsync(out->d_validity, 0, static_cast<size_t>(c->nrows / 32 + 4) * 4, s);
    // dictionary pages small enough for k_pipe_runs' workgroups decode there
    const bool dict_in_runs = pipe && !plain_go && ctx->opt_run_dict && c->ndicts &&
                              c->type == PQ_BYTE_ARRAY && c->d_dflag && c->max_dict_bytes <= pqk::kRunDictMax;
    if (dict_in_runs) {
        // k_pipe_runs decodes the dictionary
    } else if (c->ndicts && c->type == PQ_BYTE_ARRAY && pipe) {
        // the dictionary (one workgroup) decodes on the side stream while the
        // run-table pass runs; k_pipe_codes waits for both (ev_join).  The
        // side stream first waits for everything already on the main stream
        // (ev_fork): the previous decode's k_pipe_write / regex k_pipe_match
        // read the entry table this k_dict_index rewrites.  Its error flag is
        // its own sticky word (d_dflag), not the per-decode flags the main
        // stream clears.
        (void)hipEventRecord(ctx->ev_fork, s);
        (void)hipStreamWaitEvent(ctx->side, ctx->ev_fork, 0);
        {
            Timed t(ctx, "dict_index", ctx->side);
            launch_dicts(c, ctx->side, c->d_dflag);
        }
        (void)hipEventRecord(ctx->ev_join, ctx->side);
    } else if (c->ndicts && c->type == PQ_BYTE_ARRAY) {
        Timed t(ctx, "dict_index");
        launch_dicts(c, s, c->d_flags);
    } else if (c->ndicts) {
        Timed t(ctx, "dict_entries");
        pqk::launch_dict_entries(s, c->d_bytes, c->d_dicts, c->ndicts, c->d_entries, c->d_dict_count,
                                 c->d_dict_err, c->d_flags, c->type, c->plain_width);
    }
    if (plain_go && c->plain_opt) {
        // levels -> value-section pages -> one pass over them -> row offsets;
        // any error or misfit sets d_flags[3] and collect() re-runs the chunk
        // on the general path (which reports the reference's errors)
        int32_t* redo = c->d_flags + 3;
        Timed t(ctx, "plain_opt");
        (void)hipMemsetAsync(c->d_operr, 0, static_cast<size_t>(c->npages) * sizeof(DevErr), s);
        if (c->opt_lane_levels)
            pqk::launch_opt_levels(s, c->d_bytes, c->d_pages, c->npages, c->d_page_tile0, c->max_def, out->d_validity,
                                   c->d_tile_rank, c->d_page_pos, c->d_page_nn, c->d_operr, redo);
        else
            pqk::launch_fixed_levels(s, c->d_bytes, c->d_pages, c->npages, c->d_page_tile0, cp, out->d_validity,
                                     c->d_tile_rank, c->d_page_pos, c->d_page_nn, c->d_operr, redo, ctx->opt_levels_small);
        pqk::OptLaunch O{};
        O.pages = c->d_pages; O.npages = c->npages; O.page_nn = c->d_page_nn; O.page_pos = c->d_page_pos;
        O.lerr = c->d_operr; O.nnv = c->d_onnv; O.chv = c->d_ochv; O.pdense = c->d_opdense; O.pbase = c->d_opbase;
        O.scratch = c->d_scan_scratch; O.tot_nn = c->d_otot; O.tot_ch = c->d_otot + 1; O.vpages = c->d_vpages;
        O.doffs = c->d_doffs; O.redo = redo;
        pqk::launch_opt_pages(s, O);
        pqk::PlainLaunch P{};
        P.bytes = c->d_bytes; P.pages = c->d_vpages; P.wins = c->d_pwins;
        P.nwins = static_cast<int32_t>(c->hpwins.size()); P.rowinfo = c->d_rowinfo; P.wchars = c->d_wchars;
        P.bsum = c->d_pbsum; P.grid = c->plain_grid; P.nrows_total = -1; P.total = c->d_total;
        P.capacity = out->capacity_bytes; P.overflow = c->d_flags + 1; P.validity = nullptr;
        P.offsets = c->d_doffs; P.chars = out->d_values; P.page_err = c->d_operr; P.err_any = redo;
        P.redo = redo; P.gate = c->d_flags + 2;
        P.wmode = pqk::kWinOpt; P.pbase = c->d_opbase; P.pdense = c->d_opdense; P.ppos = c->d_page_pos;
        if (c->plain_spec) {
            pqk::SpecLaunch S{};
            S.bytes = c->d_bytes; S.pages = c->d_pages; S.npages = c->npages; S.chunk_base = c->d_chunk_base;
            S.chunks = c->d_chunks; S.nchunks = static_cast<int32_t>(c->hchunks.size()); S.cand = c->d_cand;
            S.ppages = c->d_ppages; S.page_err = c->d_operr; S.err_any = redo; S.fallback = c->d_flags + 2;
            S.ppos = c->d_page_pos; S.vpages = c->d_vpages;
            pqk::launch_plain_spec(s, S);
            P.pages = c->d_ppages;
            P.wmode = pqk::kWinOptPseudo; P.wpage = c->d_pwpage; P.rpages = c->d_pages;
        }
        pqk::launch_plain_ba(s, P);
        pqk::launch_opt_offsets(s, c->d_pages, c->d_tiles, c->ntiles, c->d_tile_rank, c->d_opdense, out->d_validity,
                                c->d_doffs, out->d_offsets, redo);
        (void)hipMemcpyAsync(c->d_total, c->d_otot + 1, sizeof(int64_t), hipMemcpyDeviceToDevice, s);
        (void)hipMemcpyAsync(out->d_offsets + c->nrows, c->d_otot + 1, sizeof(int64_t), hipMemcpyDeviceToDevice, s);
    } else if (plain_go) {
        pqk::PlainLaunch P{};
        P.bytes = c->d_bytes; P.pages = c->d_pages; P.wins = c->d_pwins;
        P.nwins = static_cast<int32_t>(c->hpwins.size()); P.rowinfo = c->d_rowinfo; P.wchars = c->d_wchars;
        P.bsum = c->d_pbsum; P.grid = c->plain_grid; P.nrows_total = c->nrows; P.total = c->d_total;
        P.capacity = out->capacity_bytes; P.overflow = c->d_flags + 1; P.validity = out->d_validity;
        P.offsets = out->d_offsets; P.chars = out->d_values; P.page_err = c->d_page_err; P.err_any = c->d_flags;
        if (c->nrows == 0) {
            (void)hipMemsetAsync(out->d_offsets, 0, sizeof(int64_t), s);
            (void)hipMemsetAsync(c->d_total, 0, sizeof(int64_t), s);
        }
        if (c->plain_spec) {
            // pseudo pages from speculative chunk chains; a fallback flag
            // (d_flags[2]) skips the two passes and collect() re-runs the
            // chunk on the generic path
            pqk::SpecLaunch S{};
            S.bytes = c->d_bytes; S.pages = c->d_pages; S.npages = c->npages; S.chunk_base = c->d_chunk_base;
            S.chunks = c->d_chunks; S.nchunks = static_cast<int32_t>(c->hchunks.size()); S.cand = c->d_cand;
            S.ppages = c->d_ppages; S.page_err = c->d_page_err; S.err_any = c->d_flags; S.fallback = c->d_flags + 2;
            {
                Timed t(ctx, "plain_spec");
                pqk::launch_plain_spec(s, S);
            }
            P.pages = c->d_ppages;
            P.page_err = c->d_perr;
            P.gate = c->d_flags + 2;
            if (c->d_pwbase && ctx->opt_plain_fused && !c->pfused_failed) {
                P.wbase = c->d_pwbase;
                P.redo = c->d_flags + 3;
                P.wmode = pqk::kWinPseudo;
            }
        } else if (c->d_pwbase && ctx->opt_plain_fused && !c->pfused_failed) {
            P.wbase = c->d_pwbase;
            P.redo = c->d_flags + 3;
        }
        Timed t(ctx, "plain_ba");
        pqk::launch_plain_ba(s, P);
    } else if (pipe) {
        pqk::PipeLaunch P = pipe_launch(ctx, c, out);
        pipe_front(ctx, c, P, !dict_in_runs, dict_in_runs);
        if (c->arm) {  // the page filter in the same pass: match bits per entry, then the writer tests them
            Timed t(ctx, "regex_dict");
            pqre::launch_regex_dict(s, c->d_prog, c->d_bytes, c->d_dicts, c->ndicts, c->d_entries, c->d_dict_count,
                                    c->d_dict_match, c->d_page_flags, c->npages);
            P.match = c->d_dict_match + c->pipe_entry_base;
            P.match_neg = c->arm_neg;
            P.page_flags = c->d_page_flags;
        }
        if (c->ntiles == 0) {
            (void)hipMemsetAsync(out->d_offsets, 0, sizeof(int64_t), s);
            (void)hipMemsetAsync(c->d_total, 0, sizeof(int64_t), s);
        }
        if (c->d_zero) {  // k_pipe_write clears the other block for the next decode
            P.znext = reinterpret_cast<uint32_t*>(c->d_zero + static_cast<size_t>(c->zsel ^ 1) * c->zfull);
            P.znext_words = static_cast<uint32_t>(c->zero_bytes / 4);
        }
        {
            Timed t(ctx, "pipe_write");
            pqk::launch_pipe_write(s, P);
        }
        // the other block is clear only if k_pipe_write ran (it returns early on a chunk without tiles)
        if (c->d_zero) c->next_zeroed = c->ntiles > 0;
    } else if (c->fused) {
        const size_t nr = c->ranges.size();
        (void)hipMemsetAsync(c->d_status, 0, std::max<size_t>(c->npages, 1) * sizeof(uint64_t), s);
        (void)hipMemsetAsync(c->d_tickets, 0, nr * sizeof(int32_t), s);
        (void)hipMemsetAsync(c->d_bases, 0, (nr + 1) * sizeof(int64_t), s);
        for (size_t k = 0; k < nr; k++) {
            const auto& r = c->ranges[k];
            if (r.np == 0) {
                (void)hipMemcpyAsync(c->d_bases + k + 1, c->d_bases + k, sizeof(int64_t), hipMemcpyDeviceToDevice, s);
                continue;
            }
            pqk::FusedLaunch L{};
            L.bytes = c->d_bytes; L.pages = c->d_pages; L.p0 = r.p0; L.np = r.np;
            L.dicts = c->d_dicts; L.dict_id = r.dict_id; L.entries = c->d_entries;
            L.dict_count = c->d_dict_count; L.max_def = c->max_def; L.max_rep = c->max_rep;
            L.rows_cap = r.rows_cap; L.stage_bytes = r.stage_bytes; L.wave_bytes = r.wave_bytes;
            L.dict_bytes = r.dict_bytes; L.dict_chars_bytes = r.dict_chars_bytes;
            L.status = c->d_status + r.p0; L.ticket = c->d_tickets + k;
            L.base_in = c->d_bases + k; L.base_out = c->d_bases + k + 1; L.nrows_total = c->nrows;
            L.validity = out->d_validity; L.offsets = out->d_offsets; L.chars = out->d_values;
            L.capacity = out->capacity_bytes; L.overflow = c->d_flags + 1;
            L.page_err = c->d_page_err; L.err_any = c->d_flags; L.grid = r.grid; L.waves_per_block = r.waves;
            L.debug = ctx->opt_debug;
            L.prof = ctx->d_prof;
            L.claim = ctx->opt_claim;
            Timed t(ctx, "ba_fused");
            pqk::launch_ba_fused(s, L);
        }
        (void)hipMemcpyAsync(c->d_total, c->d_bases + nr, sizeof(int64_t), hipMemcpyDeviceToDevice, s);
        (void)hipMemcpyAsync(out->d_offsets + c->nrows, c->d_bases + nr, sizeof(int64_t), hipMemcpyDeviceToDevice, s);
    } else if (c->type == PQ_BYTE_ARRAY) {
        {
            Timed t(ctx, "ba_rows");
            const uint32_t big = (c->max_def == 0 && c->max_rep == 0 && ctx->opt_plain) ? pqk::ba_rows_stage_bytes() : 0u;
            pqk::launch_ba_rows(s, c->d_bytes, c->d_pages, c->npages, c->d_dicts, c->d_entries,
                                c->d_dict_count, cp, c->d_row_codes, c->d_tile_chars,
                                c->d_page_tile0, c->d_page_err, c->d_flags, big, c->max_page_bytes,
                                ctx->opt_wide_rows && c->ndicts > 0, ctx->d_prof);
            if (big)
                pqk::launch_plain_big_rows(s, c->d_bytes, c->d_pages, c->npages, big, c->d_row_codes,
                                           c->d_tile_chars, c->d_page_tile0, c->d_page_err, c->d_flags);
        }
        {
            Timed t(ctx, "scan");
            pqk::launch_scan_i64(s, c->d_tile_chars, c->d_tile_base, c->ntiles, c->d_total,
                                 c->d_scan_scratch);
        }
        if (c->ntiles == 0) {
            (void)hipMemsetAsync(out->d_offsets, 0, sizeof(int64_t), s);
        }
        launch_gather(ctx, c, out);
    } else if (c->fixed_plain && ctx->opt_fixed_plain) {
        Timed t(ctx, "fixed_plain");
        pqk::launch_fixed_plain(s, c->d_bytes, c->d_pages, c->npages, c->d_tiles, c->ntiles, c->d_page_tile0, cp,
                                out->d_validity, out->d_values, c->d_tile_rank, c->d_page_pos, c->d_page_err,
                                c->d_flags, ctx->opt_fixed_fused, ctx->opt_levels_small);
    } else {
        Timed t(ctx, "fixed");
        pqk::launch_fixed(s, c->d_bytes, c->d_pages, c->npages, c->d_dicts, c->d_dict_count, cp,
                          out->d_validity, out->d_values, c->d_page_err, c->d_flags);
    }
    hipError_t e = hipGetLastError();
    return hip_check(ctx, e, "kernel launch");
}

// Synchronise and turn device error records into the reference's first error.
static int collect(pq_ctx* ctx, pq_chunk* c, pq_column* out) {
    int32_t flags[4] = {0, 0, 0, 0}, dflag = 0;
    if (int rc = hip_check(ctx, hipMemcpyAsync(flags, c->d_flags, sizeof flags, hipMemcpyDeviceToHost, ctx->stream), "flags"))
        return rc;
    if (c->d_dflag)
        if (int rc = hip_check(ctx, hipMemcpyAsync(&dflag, c->d_dflag, sizeof dflag, hipMemcpyDeviceToHost, ctx->stream), "flags"))
            return rc;
    if (int rc = hip_check(ctx, hipStreamSynchronize(ctx->stream), "sync")) return rc;
    flags[0] |= dflag;
    if ((flags[2] || flags[3]) && c->plain && c->plain_opt && !c->popt_failed) {
        if (std::getenv("PQ_DEBUG_SPEC")) {
            std::fprintf(stderr, "plain opt redo: fallback %d flag %d\n", flags[2], flags[3]);
            std::vector<DevErr> e(static_cast<size_t>(c->npages));
            std::vector<int32_t> pp(e.size()), pn(e.size());
            (void)hipMemcpy(e.data(), c->d_operr, e.size() * sizeof(DevErr), hipMemcpyDeviceToHost);
            (void)hipMemcpy(pp.data(), c->d_page_pos, pp.size() * 4, hipMemcpyDeviceToHost);
            (void)hipMemcpy(pn.data(), c->d_page_nn, pn.size() * 4, hipMemcpyDeviceToHost);
            for (size_t i = 0; i < e.size() && i < 8; i++)
                std::fprintf(stderr, "  page %zu: err %d pos %d need %d size %d; values at %d, %d non-null\n", i, e[i].code,
                             e[i].pos, e[i].need, e[i].size, pp[i], pn[i]);
            if (c->plain_spec) {
                std::vector<uint4> cd(std::min<size_t>(c->hchunks.size(), 8) * pqk::kPCand);
                (void)hipMemcpy(cd.data(), c->d_cand, cd.size() * sizeof(uint4), hipMemcpyDeviceToHost);
                for (size_t i = 0; i < cd.size(); i++)
                    if (cd[i].x != 0xFFFFFFFFu)
                        std::fprintf(stderr, "  cand chunk %zu slot %zu: entry %u err %u exit %u cnt %u w %u\n", i / pqk::kPCand,
                                     i % pqk::kPCand, cd[i].x & 0x7FFFFFFFu, cd[i].x >> 31, cd[i].y, cd[i].z, cd[i].w);
            }
        }
        // the OPTIONAL chunk did not fit the PLAIN kernels' form (an error,
        // or value sections their strings do not fill): the general path
        // decodes it from now on and reports any error
        c->popt_failed = true;
        if (c->npages) (void)hipMemsetAsync(c->d_page_err, 0, c->npages * sizeof(DevErr), ctx->stream);
        if (!out) out = c->last_out;
        if (!out) return set_err(ctx, PQ_ERR_ARG, "decode check without an output column");
        if (int rc = pq_decode_async(ctx, c, out)) return rc;
        return collect(ctx, c, out);
    }
    if (flags[3] && c->plain && !c->plain_opt && !c->pfused_failed && !(flags[2] && c->plain_spec)) {
        // a page's strings did not fill it exactly (or its chain failed): the
        // one-pass PLAIN kernel's character placement does not hold; the two
        // passes decode the chunk from now on (and report any error)
        c->pfused_failed = true;
        if (!out) out = c->last_out;
        if (!out) return set_err(ctx, PQ_ERR_ARG, "decode check without an output column");
        if (int rc = pq_decode_async(ctx, c, out)) return rc;
        return collect(ctx, c, out);
    }
    if (flags[2] && c->plain_spec && !c->spec_failed) {
        if (std::getenv("PQ_DEBUG_SPEC"))
        {
            std::fprintf(stderr, "plain spec fallback: flags %d (reason %d, chunk %d)\n", flags[2], flags[2] & 0xFF, flags[2] >> 8);
            std::vector<uint4> cd(std::min<size_t>(c->hchunks.size(), 4) * pqk::kPCand);
            (void)hipMemcpy(cd.data(), c->d_cand, cd.size() * sizeof(uint4), hipMemcpyDeviceToHost);
            for (size_t i = 0; i < cd.size(); i++)
                std::fprintf(stderr, "  cand chunk %zu slot %zu: entry %u err %u exit %u cnt %u w %u\n", i / pqk::kPCand,
                             i % pqk::kPCand, cd[i].x & 0x7FFFFFFFu, cd[i].x >> 31, cd[i].y, cd[i].z, cd[i].w);
        }
        // the speculative chunk chains did not resolve (strings longer than
        // the candidate range or the window): this chunk takes the generic
        // path from now on; decode it again
        c->spec_failed = true;
        if (c->npages) (void)hipMemsetAsync(c->d_page_err, 0, c->npages * sizeof(DevErr), ctx->stream);
        if (!out) out = c->last_out;
        if (!out) return set_err(ctx, PQ_ERR_ARG, "decode check without an output column");
        if (int rc = pq_decode_async(ctx, c, out)) return rc;
        return collect(ctx, c, out);
    }
    int64_t best_seq = c->walk_error ? c->walk_error_seq : INT64_MAX;
    int best_code = c->walk_error;
    std::string best_msg = c->walk_message;
    if (flags[0]) {
        std::vector<DevErr> pe(c->npages), de(c->ndicts);
        if (c->npages) (void)hipMemcpy(pe.data(), c->d_page_err, pe.size() * sizeof(DevErr), hipMemcpyDeviceToHost);
        if (c->ndicts) (void)hipMemcpy(de.data(), c->d_dict_err, de.size() * sizeof(DevErr), hipMemcpyDeviceToHost);
        for (int i = 0; i < c->npages; i++)
            if (pe[i].code && c->page_seq[i] < best_seq) {
                best_seq = c->page_seq[i];
                best_code = pe[i].code;
                best_msg = format_error(pe[i]);
            }
        for (int i = 0; i < c->ndicts; i++)
            if (de[i].code && c->dict_seq[i] < best_seq) {
                best_seq = c->dict_seq[i];
                best_code = de[i].code;
                best_msg = format_error(de[i]);
            }
        // clear records for the next call
        if (c->npages) (void)hipMemsetAsync(c->d_page_err, 0, c->npages * sizeof(DevErr), ctx->stream);
        // (dictionary records of chunks decoded on the side stream stay: the
        // next decode's dictionary pass may already be writing them again)
        if (c->ndicts && !c->d_dflag) (void)hipMemsetAsync(c->d_dict_err, 0, c->ndicts * sizeof(DevErr), ctx->stream);
    }
    if (best_code) {
        c->codes_pending = c->entries_pending = c->rx_index_pending = false;
        return set_err(ctx, best_code, best_msg);
    }
    if (c->codes_pending) c->codes_ok = true;
    if (c->entries_pending) c->entries_ok = true;
    if (c->rx_index_pending) c->rx_index_ok = true;
    c->codes_pending = c->entries_pending = c->rx_index_pending = false;
    if (c->type == PQ_BYTE_ARRAY && out) {
        int64_t total = 0;
        (void)hipMemcpy(&total, c->d_total, sizeof total, hipMemcpyDeviceToHost);
        out->num_bytes = total;
        if (flags[1]) {  // chars overflowed the estimate: grow and run again
            dfree(out->d_values);
            if (dalloc(&out->d_values, static_cast<size_t>(total + 64)))
                return set_err(ctx, PQ_ERR_HIP, "hipMalloc failed (chars)");
            out->capacity_bytes = total;
            if (int rc = pq_decode_async(ctx, c, out)) return rc;  // every path writes the whole column
            return hip_check(ctx, hipStreamSynchronize(ctx->stream), "sync");
        }
    } else if (out) {
        out->num_bytes = c->nrows * c->width;
    }
    return 0;
}

int pq_decode_check(pq_ctx* ctx, pq_chunk* c) {
    if (!ctx || !c) return PQ_ERR_ARG;
    DevGuard dg(ctx);
    // the column of the chunk's last async decode gets its byte count (and
    // grows and decodes again if its characters overflowed the estimate)
    // (the column is the caller's: once collected, no later call touches it)
    const int rc = collect(ctx, c, c->last_out);
    c->last_out = nullptr;
    return rc;
}

int pq_decode(pq_ctx* ctx, pq_chunk* c, pq_column* out) {
    DevGuard dg(ctx);
    if (int rc = pq_decode_async(ctx, c, out)) return rc;
    const int rc = collect(ctx, c, out);
    c->last_out = nullptr;
    return rc;
}

int pq_column_copy_out(pq_ctx* ctx, const pq_column* col, uint32_t* validity, uint8_t* values,
                       int64_t* offsets) {
    if (!ctx || !col) return PQ_ERR_ARG;
    // a column a failed decode left behind (its byte count past its buffer)
    if (col->num_bytes < 0 || col->num_rows < 0 || (col->num_bytes && (!col->d_values || col->num_bytes > col->capacity_bytes)))
        return set_err(ctx, PQ_ERR_ARG, "column bytes past its buffer");
    DevGuard dg(ctx);
    hipStream_t s = ctx->stream;
    int rc = hip_check(ctx, hipStreamSynchronize(s), "copy sync");  // (the decode that made the column)
    // large arrays through the pinned ring (DMA of piece i + k while host
    // threads copy piece i out: pageable destinations would take the
    // runtime's bounce buffer at a fraction of PCIe bandwidth, one thread)
    const int hw = static_cast<int>(std::min(16u, std::max(1u, std::thread::hardware_concurrency())));
    auto get = [&](void* dst, const void* src, size_t n, const char* what) {
        if (!dst || !n || rc) return;
        if (n < (4u << 20)) {
            rc |= hip_check(ctx, hipMemcpy(dst, src, n, hipMemcpyDeviceToHost), what);
            return;
        }
        uint8_t* d = static_cast<uint8_t*>(dst);
        rc |= hip_check(ctx, ctx->stager.download(static_cast<const uint8_t*>(src), n, ctx->copy, hw,
                                                  [&](const uint8_t* b, size_t a, size_t z) { std::memcpy(d + a, b, z - a); }),
                        what);
    };
    if (col->num_rows) get(validity, col->d_validity, static_cast<size_t>((col->num_rows + 31) / 32) * 4, "copy validity");
    if (col->num_bytes) get(values, col->d_values, static_cast<size_t>(col->num_bytes), "copy values");
    if (col->d_offsets) get(offsets, col->d_offsets, static_cast<size_t>(col->num_rows + 1) * 8, "copy offsets");
    return rc ? PQ_ERR_HIP : 0;
}

int pq_chunk_assign(pq_ctx* ctx, const pq_column* col, int64_t chunk_bytes, int64_t* d_tuple_to_chunk,
                    int64_t* h_tuple_to_chunk, int64_t* num_chunks) {
    if (!ctx || !col || !num_chunks || chunk_bytes < 0) return PQ_ERR_ARG;
    DevGuard dg(ctx);
    if (col->type != PQ_BYTE_ARRAY || (col->num_rows > 0 && (!col->d_validity || !col->d_offsets)))
        return set_err(ctx, PQ_ERR_ARG, "pq_chunk_assign: a decoded BYTE_ARRAY column is required");
    (void)hipSetDevice(ctx->device);
    const int64_t n = col->num_rows;
    const size_t out_bytes = d_tuple_to_chunk ? 0 : (static_cast<size_t>(std::max<int64_t>(n, 1)) * 8 + 255) / 256 * 256;
    const size_t need = pqk::chunk_assign_scratch(n) + out_bytes;
    if (ctx->chunker_cap < need) {
        dfree(ctx->d_chunker);
        ctx->chunker_cap = 0;
        if (dalloc(&ctx->d_chunker, need)) return set_err(ctx, PQ_ERR_HIP, "hipMalloc failed (chunker)");
        ctx->chunker_cap = need;
    }
    int64_t* out = d_tuple_to_chunk ? d_tuple_to_chunk : reinterpret_cast<int64_t*>(ctx->d_chunker);
    int rc = pqk::chunk_assign(ctx->stream, col->d_validity, col->d_offsets, n, chunk_bytes, out,
                               ctx->d_chunker + out_bytes, num_chunks);
    if (rc == -2) return set_err(ctx, PQ_ERR_UNSUPPORTED, "pq_chunk_assign: column too large");
    if (rc) return set_err(ctx, PQ_ERR_HIP, "pq_chunk_assign: HIP failure");
    if (h_tuple_to_chunk && n > 0)
        return hip_check(ctx, hipMemcpy(h_tuple_to_chunk, out, static_cast<size_t>(n) * 8, hipMemcpyDeviceToHost),
                         "chunker copy-out");
    return 0;
}

void pq_column_free(pq_ctx* ctx, pq_column* col) {
    DevGuard dg(ctx);
    if (!col) return;
    if (ctx) (void)hipStreamSynchronize(ctx->stream);
    dfree(col->d_validity);
    dfree(col->d_values);
    dfree(col->d_offsets);
    std::memset(col, 0, sizeof *col);
}

void pq_timing_enable(pq_ctx* ctx, int enable) { if (ctx) ctx->timing = enable != 0; }
void pq_timing_reset(pq_ctx* ctx) {
    if (!ctx) return;
    DevGuard dg(ctx);
    resolve_timers(ctx);
    ctx->timers.clear();
}
int pq_timing_get(pq_ctx* ctx, const char* name, double* total_ms, int64_t* launches) {
    if (!ctx || !name) return 0;
    DevGuard dg(ctx);
    resolve_timers(ctx);
    auto it = ctx->timers.find(name);
    if (it == ctx->timers.end()) return 0;
    if (total_ms) *total_ms = it->second.first;
    if (launches) *launches = it->second.second;
    return 1;
}

int pq_fused_prof_read(pq_ctx* ctx, uint64_t* out, int n) {
    if (!ctx || !ctx->d_prof) return 0;
    DevGuard dg(ctx);
    const int k = pqk::fused_prof_slots();
    std::vector<uint64_t> h(static_cast<size_t>(k));
    if (hipStreamSynchronize(ctx->stream) != hipSuccess) return 0;
    if (hipMemcpy(h.data(), ctx->d_prof, k * sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess) return 0;
    (void)hipMemset(ctx->d_prof, 0, k * sizeof(uint64_t));
    for (int i = 0; i < std::min(n, k); i++) out[i] = h[static_cast<size_t>(i)];
    return k;
}

// ── regex page filter ───────────────────────────────────────────────────────
int pq_regex_compile_check(const char* pattern, char* err, size_t errlen) {
    std::string msg;
    int rc = pqre::check(pattern ? pattern : "", &msg);
    if (err && errlen) {
        std::strncpy(err, msg.c_str(), errlen - 1);
        err[errlen - 1] = 0;
    }
    return rc;
}

// The compiled pattern (cached per chunk), page flags and the per-entry
// match buffer of a BYTE_ARRAY chunk.
static int regex_prepare(pq_ctx* ctx, pq_chunk* c, const char* pattern) {
    if (c->type != PQ_BYTE_ARRAY) return set_err(ctx, PQ_ERR_ARG, "regex page filter needs a BYTE_ARRAY column");
    try {
        std::string msg;
        pqre::Program prog;
        int rc = pqre::compile(pattern, &prog, &msg);
        if (rc) return set_err(ctx, PQ_ERR_REGEX, msg);
        if (!c->d_page_flags && dalloc(&c->d_page_flags, static_cast<size_t>(c->npages)))
            return set_err(ctx, PQ_ERR_HIP, "hipMalloc failed (page flags)");
        int64_t dict_cap = std::max<int64_t>(c->nentries, 1);
        if (c->dict_match_cap < dict_cap) {
            dfree(c->d_dict_match);
            if (dalloc(&c->d_dict_match, static_cast<size_t>(dict_cap)))
                return set_err(ctx, PQ_ERR_HIP, "hipMalloc failed (dict match)");
            c->dict_match_cap = dict_cap;
        }
        // compiled programs are cached per chunk by pattern (the bench and the
        // CLI rescan with one pattern)
        const std::string key = std::string(pattern) + (ctx->opt_regex_dfa ? "|dfa" : "|nfa");
        if (!c->d_prog || c->prog_pattern != key) {
            if (c->d_prog) pqre::free_device_program(c->d_prog);
            c->d_prog = pqre::upload_program(prog, ctx->stream);
            if (!c->d_prog) return set_err(ctx, PQ_ERR_HIP, "regex program upload failed");
            std::vector<uint8_t> img;
            dfree(c->d_dfa);
            c->dfa_bytes = 0;
            c->dfa_sink = false;
            if (ctx->opt_regex_dfa && pqre::build_dfa(prog, &img)) {
                if (dalloc(&c->d_dfa, img.size())) return set_err(ctx, PQ_ERR_HIP, "hipMalloc failed (dfa)");
                if (int rc2 = hip_check(ctx, hipMemcpy(c->d_dfa, img.data(), img.size(), hipMemcpyHostToDevice), "dfa upload"))
                    return rc2;
                c->dfa_bytes = static_cast<uint32_t>(img.size());
                c->dfa_full = reinterpret_cast<const pqre::DevDfa*>(img.data())->full != 0;
                c->dfa_sink = c->dfa_full && reinterpret_cast<const pqre::DevDfa*>(img.data())->anchored != 0;
            }
            c->prog_pattern = key;
        }
        return 0;
    } catch (const std::exception& e) {
        return set_err(ctx, PQ_ERR_ALLOC, e.what());
    }
}

int pq_regex_pages_async(pq_ctx* ctx, pq_chunk* c, const char* pattern, int neg) {
    if (!ctx || !c || !pattern) return PQ_ERR_ARG;
    DevGuard dg(ctx);
    if (int rc = regex_prepare(ctx, c, pattern)) return rc;
    try {
        hipStream_t s = ctx->stream;
        pqk::ColumnParams cp{c->type, c->max_def, c->max_rep, c->width, c->plain_width};
        const bool on_codes = c->pipe && (!c->pipe_wide || pqk::pipe_match_wide_ok(c->pipe_ecap)) && ctx->opt_pipe &&
                              ctx->opt_regex_codes;
        const bool reuse = on_codes && ctx->opt_regex_reuse && c->codes_ok;
        // over a checked decode's codes: k_regex_dict clears the status words
        // and sets the page flags itself (no fill kernels)
        const bool fold = reuse && c->ndicts && c->entries_ok && c->zero_bytes % 4 == 0;
        if (!fold) (void)hipMemsetAsync(c->d_flags, 0, c->zero_bytes, s);
        if (c->ndicts) {
            if (!(ctx->opt_regex_reuse && c->entries_ok)) {
                c->entries_pending = true;
                Timed t(ctx, "dict_index");
                launch_dicts(c, s, c->d_flags);
            }
            Timed t(ctx, "regex_dict");
            pqre::launch_regex_dict(s, c->d_prog, c->d_bytes, c->d_dicts, c->ndicts, c->d_entries,
                                    c->d_dict_count, c->d_dict_match, fold ? c->d_page_flags : nullptr,
                                    fold ? c->npages : 0, fold ? reinterpret_cast<uint32_t*>(c->d_flags) : nullptr,
                                    fold ? static_cast<int64_t>(c->zero_bytes / 4) : 0);
        }
        if (on_codes) {
            // dictionary-first on the decode's own codes: the pattern ran on
            // every entry above; the pipe passes give each row its index
            // (or a checked earlier decode already did)
            const pqk::PipeLaunch P = pipe_launch(ctx, c, nullptr);
            if (!reuse) {
                pipe_front(ctx, c, P, false, false);
                c->codes_pending = true;
            }
            Timed t(ctx, "regex_codes");
            pqk::launch_pipe_match(s, P, c->d_dict_match + c->pipe_entry_base, neg, c->d_page_flags, fold);
        } else if (c->d_dfa && ctx->opt_regex_plain && c->ndicts == 0 && pqre::regex_plain_lds_ok() &&
                   plan_regex_windows(ctx, c)) {
            // REQUIRED chunks: the first error-free scan files every string's
            // window offset (row-indexed); later scans read it instead of
            // walking the length chains (same windows: same window size)
            const uint16_t* idx_in = nullptr;
            uint16_t* idx_out = nullptr;
            if (ctx->opt_regex_index && c->max_def == 0 && c->max_rep == 0 && c->nrows > 0 && !ctx->opt_regex_debug) {
                if (c->rx_index_ok && c->rx_index_win == c->rwin_bytes && ctx->opt_regex_index != 2) {
                    idx_in = c->d_rx_index;
                } else {
                    c->rx_index_ok = false;
                    if (c->d_rx_index || !dalloc(&c->d_rx_index, static_cast<size_t>(c->nrows))) {
                        idx_out = c->d_rx_index;
                        c->rx_index_pending = true;
                        c->rx_index_win = c->rwin_bytes;
                    }
                }
            }
            Timed t(ctx, "regex_plain");
            pqre::launch_regex_plain(s, c->d_dfa, c->dfa_bytes, c->rwin_bytes, c->d_bytes, c->d_pages, c->d_rwins,
                                     static_cast<int>(c->hrwins.size()), c->d_rwin_ticket, c->rwin_grid, cp,
                                     (neg ? 1 : 0) | ((ctx->opt_regex_debug & 0xFF) << 8),
                                     c->d_page_flags, c->d_page_err, c->d_flags, idx_in, idx_out, c->dfa_sink);
        } else if (c->d_dfa) {
            Timed t(ctx, "regex_lanes");
            pqre::launch_regex_lanes(s, c->d_dfa, c->dfa_bytes, c->d_bytes, c->d_pages, c->npages, c->d_dicts,
                                     c->d_dict_count, c->d_dict_match, cp, neg, c->d_page_flags,
                                     c->d_page_err, c->d_flags);
        } else {
            Timed t(ctx, "regex_pages");
            pqre::launch_regex_pages(s, c->d_prog, c->d_bytes, c->d_pages, c->npages, c->d_dicts,
                                     c->d_entries, c->d_dict_count, c->d_dict_match, cp, neg,
                                     c->d_page_flags, c->d_page_err, c->d_flags);
        }
        return hip_check(ctx, hipGetLastError(), "regex launch");
    } catch (const std::exception& e) {
        return set_err(ctx, PQ_ERR_ALLOC, e.what());
    }
}

int pq_regex_pages_result(pq_ctx* ctx, pq_chunk* c, uint8_t* page_flags) {
    if (!ctx || !c) return PQ_ERR_ARG;
    DevGuard dg(ctx);
    if (int rc = collect(ctx, c, nullptr)) return rc;
    if (page_flags && c->npages)
        return hip_check(ctx, hipMemcpy(page_flags, c->d_page_flags, static_cast<size_t>(c->npages), hipMemcpyDeviceToHost), "copy page flags");
    return 0;
}

int pq_decode_regex_async(pq_ctx* ctx, pq_chunk* c, pq_column* out, const char* pattern, int neg) {
    if (!ctx || !c || !out || !pattern) return PQ_ERR_ARG;
    DevGuard dg(ctx);
    if (int rc = regex_prepare(ctx, c, pattern)) return rc;
    // one pass when the decode takes the pipe (dictionary pages only, one
    // dictionary of < 32 KiB: the writer keeps each entry's match bit beside
    // its length); else the decode, then the scan over its codes
    const bool plain_go = c->plain && ctx->opt_plain;
    const bool one = c->pipe && !c->pipe_wide && ctx->opt_pipe && ctx->opt_regex_codes && !plain_go && c->ndicts > 0 &&
                     c->pipe_dict_payload < pqk::kArmDictBytes;
    if (!one) {
        // the scan clears d_flags, which still holds this decode's status
        // (err_any, char overflow, the PLAIN redo flags): check the decode
        // first, so its redo / growth / error runs before the scan starts
        if (int rc = pq_decode_async(ctx, c, out)) return rc;
        if (int rc = collect(ctx, c, out)) return rc;
        return pq_regex_pages_async(ctx, c, pattern, neg);
    }
    c->arm = true;
    c->arm_neg = neg ? 1 : 0;
    const int rc = pq_decode_async(ctx, c, out);
    c->arm = false;
    return rc;
}

int pq_regex_pages(pq_ctx* ctx, pq_chunk* c, const char* pattern, int neg, uint8_t* page_flags) {
    DevGuard dg(ctx);
    if (int rc = pq_regex_pages_async(ctx, c, pattern, neg)) return rc;
    return pq_regex_pages_result(ctx, c, page_flags);
}

// ── file helpers ────────────────────────────────────────────────────────────
}  // extern "C"

struct pq_file {
    pqfmt::FileMeta meta;
    std::vector<pqfmt::LeafColumn> cols;
    std::vector<std::array<int64_t, 4>> pidx;
};

extern "C" {

int pq_file_open(const uint8_t* file, size_t file_len, pq_file** out, char* err, size_t errlen) {
    if (!file || !out) return PQ_ERR_ARG;
    *out = nullptr;
    try {
        auto f = std::make_unique<pq_file>();
        f->meta = pqfmt::parse_footer(file, file_len);
        f->cols = pqfmt::leaf_columns(f->meta);
        f->pidx = pqfmt::page_index(file, file_len, f->meta);
        *out = f.release();
        return 0;
    } catch (const pqfmt::Error& e) {
        if (err && errlen) { std::strncpy(err, e.what(), errlen - 1); err[errlen - 1] = 0; }
        return e.code;
    } catch (const std::exception& e) {
        if (err && errlen) { std::strncpy(err, e.what(), errlen - 1); err[errlen - 1] = 0; }
        return PQ_ERR_ALLOC;
    }
}
void pq_file_close(pq_file* f) { delete f; }
int64_t pq_file_num_rows(const pq_file* f) { return f ? f->meta.num_rows : 0; }
int pq_file_num_row_groups(const pq_file* f) { return f ? static_cast<int>(f->meta.row_groups.size()) : 0; }
int pq_file_num_columns(const pq_file* f) { return f ? static_cast<int>(f->cols.size()) : 0; }
int pq_file_column_name(const pq_file* f, int col, char* buf, size_t buflen) {
    if (!f || col < 0 || col >= static_cast<int>(f->cols.size()) || !buf || !buflen) return PQ_ERR_ARG;
    std::strncpy(buf, f->cols[col].name.c_str(), buflen - 1);
    buf[buflen - 1] = 0;
    return 0;
}
int pq_file_find_column(const pq_file* f, const char* name) {  // last match wins (build_column_index)
    if (!f || !name) return -1;
    int found = -1;
    for (size_t i = 0; i < f->cols.size(); i++)
        if (f->cols[i].name == name) found = static_cast<int>(i);
    return found;
}
int pq_file_column_info(const pq_file* f, int col, int32_t* type, int16_t* max_def,
                        int16_t* max_rep, int32_t* repetition, int32_t* converted_type) {
    if (!f || col < 0 || col >= static_cast<int>(f->cols.size())) return PQ_ERR_ARG;
    const auto& c = f->cols[col];
    if (type) *type = c.type;
    if (max_def) *max_def = c.max_def;
    if (max_rep) *max_rep = c.max_rep;
    if (repetition) *repetition = c.repetition.value_or(-1);
    if (converted_type) *converted_type = c.converted_type.value_or(-1);
    return 0;
}

int pq_file_chunk(const pq_file* f, int rg, int col, pq_chunk_desc* out) {
    if (!f || !out || rg < 0 || rg >= static_cast<int>(f->meta.row_groups.size()) || col < 0 ||
        col >= static_cast<int>(f->cols.size()))
        return PQ_ERR_ARG;
    const auto& lc = f->cols[col];
    const auto& r = f->meta.row_groups[rg];
    if (lc.column_index >= static_cast<int>(r.columns.size())) return PQ_ERR_ARG;
    const auto& cc = r.columns[lc.column_index];
    if (!cc.meta) return PQ_ERR_OPTIONAL;  // "ColumnChunk has no metadata"
    std::memset(out, 0, sizeof *out);
    out->num_values = cc.meta->num_values;
    out->data_page_offset = cc.meta->data_page_offset;
    out->has_dictionary_page_offset = cc.meta->dictionary_page_offset.has_value();
    out->dictionary_page_offset = cc.meta->dictionary_page_offset.value_or(0);
    out->codec = cc.meta->codec;
    out->type = lc.type;
    out->max_def_level = lc.max_def;
    out->max_rep_level = lc.max_rep;
    out->total_compressed_size = cc.meta->total_compressed;
    return 0;
}
int64_t pq_file_row_group_rows(const pq_file* f, int rg) {
    if (!f || rg < 0 || rg >= static_cast<int>(f->meta.row_groups.size())) return 0;
    return f->meta.row_groups[rg].num_rows;
}
int64_t pq_file_num_pages(const pq_file* f) { return f ? static_cast<int64_t>(f->pidx.size()) : 0; }
int pq_file_page_index(const pq_file* f, int64_t* entries, int64_t cap) {
    if (!f || !entries) return PQ_ERR_ARG;
    for (int64_t i = 0; i < cap && i < static_cast<int64_t>(f->pidx.size()); i++)
        for (int k = 0; k < 4; k++) entries[4 * i + k] = f->pidx[i][k];
    return 0;
}

}  // extern "C"
