// dict_batch.hip — batched decode of dictionary-encoded BYTE_ARRAY column
// chunks (SURVEY §8a R-RLE / R-LEVELS / R-DICT-EXPAND) on gfx950.
//
// Why a different shape from dict_fused.hip: decoding one page per wavefront
// (hybrid.hpp) spends thousands of VALU/SALU instructions and dozens of
// dependent LDS round trips per page on run-dense streams.  Here the serial
// part — the run-header chains of the def-level and index streams — is
// walked by one lane per page, 64 pages per wavefront at once, with the
// reference state machine (rle_decoder.hpp:6-108) restated as plain scalar
// code: each instruction advances 64 pages.  Its output per page is compact
// (validity mask, list of (count, value | bit offset) runs, non-null count,
// character total), so the wide work — expanding runs to rows, the offsets
// prefix sum and the character copy — happens afterwards with one page per
// wavefront and every lane busy.
//
// Workgroup = 1 producer wave + NW writer waves, all state in LDS:
//   producer  batch ticket -> batch payload (contiguous in the device image)
//             -> LDS; lane-per-page walks; batch char total; decoupled
//             look-back over batches; page records published to a queue.
//             Its only global stores: look-back words and error records.
//   writers   take pages from the queue: runs -> index per non-null rank,
//             rows pass (validity, rank -> dictionary entry, offsets), and
//             the characters through an LDS ring (stores only, no loads, so
//             nothing ever waits on the shared vmcnt for a store).
// Batch buffers are double-buffered: the producer fills one while writers
// drain the other.
#include "kernels/device_common.hpp"
#include "kernels/hybrid.hpp"
#include "kernels/kernels.hpp"
#include "kernels/lane_walk.hpp"
#include "kernels/stream.hpp"
#include "pq_gpu.h"

namespace pqk {
namespace {

using namespace dev;

constexpr uint64_t kAgg = 1ull << 62;
constexpr uint64_t kInc = 2ull << 62;
constexpr uint64_t kValMask = (1ull << 62) - 1;
constexpr uint32_t kRingBytes = 2048;
constexpr uint32_t kRingMaxRow = kRingBytes / 2 - 32;
constexpr uint32_t kLitCap = 16;

// run record: count (13 bits) | literal (1 bit) | payload (18 bits):
// RLE -> dictionary index (0xFFFF = out of range, i.e. NULL); literal ->
// page bit offset of the run's first value.
constexpr uint32_t kRunCountBits = 13;
__device__ __forceinline__ uint32_t run_rec(uint32_t count, uint32_t lit, uint32_t payload) {
    return count | (lit << kRunCountBits) | (payload << (kRunCountBits + 1));
}
__device__ __forceinline__ uint32_t run_count(uint32_t r) { return r & ((1u << kRunCountBits) - 1u); }
__device__ __forceinline__ uint32_t run_lit(uint32_t r) { return (r >> kRunCountBits) & 1u; }
__device__ __forceinline__ uint32_t run_payload(uint32_t r) { return r >> (kRunCountBits + 1); }

enum : uint32_t { REC_ERR = 1, REC_SERIAL = 2 };

struct PageRec {          // producer -> writer, 64 B
    int64_t G0;           // first output byte
    int64_t first_row;
    uint64_t goff;        // payload offset in the device image
    uint32_t n, nn, total, nruns;
    uint32_t pay;         // LDS byte address of the page copy
    uint32_t size;
    uint32_t ipos;        // index stream start (page byte)
    uint32_t bw;          // index bit width
    uint32_t flags;       // REC_*
    uint32_t runs;        // LDS byte address of the run list
};

struct Ctrl {             // queue state, LDS
    uint32_t published;   // pages published so far (queue positions)
    uint32_t next;        // next queue position to hand to a writer
    uint32_t finished;    // producer done: no position >= published will come
    uint32_t qstart[2], count[2], done[2];
    uint32_t ver[2];      // seqlock over (qstart, count) of each buffer
};

struct BArgs {
    const uint8_t* bytes;
    const DevPage* pages;
    const DevBatch* batches;
    int32_t nbatches;
    int32_t last_page;           // the chunk's last data page (absolute index)
    const DevDict* dicts;
    int32_t dict_id;
    const uint64_t* entries;
    const int32_t* dict_count;
    int32_t max_def, max_rep;
    uint32_t rows_cap;
    uint32_t batch_bytes;        // payload bytes per batch buffer (multiple of 16)
    uint32_t max_slot;           // largest page slot (bytes)
    uint32_t dict_bytes, dict_chars_bytes;
    uint64_t* status;            // per batch look-back words (zeroed)
    int32_t* ticket;             // zeroed
    const int64_t* base_in;
    int64_t* base_out;
    int64_t nrows_total;
    uint32_t* validity;
    int64_t* offsets;
    uint8_t* chars;
    int64_t capacity;
    int32_t* overflow;
    DevErr* page_err;
    int32_t* err_any;
    int32_t debug;
    uint64_t* prof;
};

// LDS layout (shared with the host through batch_lds_layout).
struct BLayout {
    uint32_t mask_words;                             // per page
    uint32_t ctrl;                                   // offsets from the dict region end
    uint32_t b_pay, b_runs, b_mask, b_recs, buf;     // within one batch buffer
    uint32_t bufs;                                   // first buffer
    uint32_t w_ix, w_off, w_rsrc, w_ring, w_starts, w_lits, writer;  // within one writer region
    uint32_t writers;                                // first writer region
    uint32_t fixed;                                  // everything but the writers
};
__host__ __device__ inline uint32_t bal16(uint32_t x) { return (x + 15u) & ~15u; }
__host__ __device__ inline BLayout batch_layout(uint32_t rows_cap, uint32_t batch_bytes, uint32_t max_slot) {
    BLayout L;
    L.mask_words = rows_cap / 32;
    L.ctrl = 0;
    uint32_t o = bal16(static_cast<uint32_t>(sizeof(Ctrl)));
    L.b_pay = 0;
    L.b_runs = batch_bytes;
    L.b_mask = 2 * batch_bytes;
    L.b_recs = L.b_mask + bal16(4 * 64 * L.mask_words);
    L.buf = L.b_recs + 64 * static_cast<uint32_t>(sizeof(PageRec));
    L.bufs = o;
    o += 2 * L.buf;
    L.writers = o;
    uint32_t w = 0;
    L.w_ix = w; w += bal16(2 * rows_cap);
    L.w_off = w; w += bal16(4 * (rows_cap + 1));
    L.w_rsrc = w; w += bal16(2 * rows_cap);
    L.w_ring = w; w += kRingBytes;
    L.w_starts = w; w += bal16(2 * (max_slot / 4 + 1));
    L.w_lits = w; w += bal16(static_cast<uint32_t>(sizeof(LitRun)) * kLitCap);
    L.writer = w;
    L.fixed = o;
    return L;
}

__device__ __forceinline__ uint32_t lds_u32a(const uint32_t* words, uint32_t a) {
    uint32_t w0 = words[a >> 2], w1 = words[(a >> 2) + 1];
    return __builtin_amdgcn_alignbyte(w1, w0, a & 3);
}

__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, kWave);
    return v;
}

__device__ uint64_t look_back(uint64_t* status, int32_t t, uint64_t total) {
    if (t == 0) {
        if (lane() == 0) __hip_atomic_store(&status[0], kInc | total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return 0;
    }
    if (lane() == 0) __hip_atomic_store(&status[t], kAgg | total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint64_t prefix = 0;
    int32_t q = t - 1;
    uint32_t nap = 1;
    for (;;) {
        const int32_t i = q - static_cast<int32_t>(lane());
        const uint64_t s = i >= 0 ? __hip_atomic_load(&status[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kInc;
        const uint64_t incm = __ballot((s >> 62) == 2);
        const uint64_t notready = __ballot((s >> 62) == 0);
        const uint32_t first_inc = incm ? static_cast<uint32_t>(__builtin_ctzll(incm)) : 64u;
        const uint64_t upto = first_inc >= 63 ? ~0ull : ((2ull << first_inc) - 1ull);
        if (notready & upto) {
            for (uint32_t k = 0; k < nap; k++) __builtin_amdgcn_s_sleep(8);
            nap = nap < 8 ? 2 * nap : 8;
            continue;
        }
        const uint64_t c = lane() <= first_inc ? (s & kValMask) : 0ull;
        prefix += wave_sum64(c);
        if (first_inc < 64) break;
        q -= 64;
    }
    if (lane() == 0)
        __hip_atomic_store(&status[t], kInc | (prefix + total), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return prefix;
}

// LDS queue words: relaxed workgroup-scope atomics; a wave's LDS operations
// execute in order, and the asm barriers keep the compiler from moving LDS
// accesses across them.
__device__ __forceinline__ uint32_t ld_u32(const uint32_t* p) {
    __asm__ __volatile__("" ::: "memory");
    const uint32_t v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __asm__ __volatile__("" ::: "memory");
    return __builtin_amdgcn_readfirstlane(v);
}
__device__ __forceinline__ void st_u32(uint32_t* p, uint32_t v) {
    __asm__ __volatile__("" ::: "memory");
    if (lane() == 0) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __asm__ __volatile__("" ::: "memory");
}

__device__ __forceinline__ uint64_t clk() { return __builtin_amdgcn_s_memtime(); }

enum { BP_WAITBUF = 0, BP_STAGE, BP_WALK, BP_LOOKBACK, BP_BATCHES, BW_WAIT, BW_RUNS, BW_ROWS, BW_CHARS, BW_PAGES,
       BP_DEFWALK, kBProfSlots };

template <bool kProf>
struct BProf {
    uint64_t ph[kBProfSlots];
    uint64_t tk;
    __device__ void start() {
        if (kProf) {
            for (int i = 0; i < kBProfSlots; i++) ph[i] = 0;
            tk = clk();
        }
    }
    __device__ void mark(int s) {
        if (kProf) {
            const uint64_t now = clk();
            ph[s] += now - tk;
            tk = now;
        }
    }
    __device__ void count(int s) {
        if (kProf) ph[s]++;
    }
    __device__ void flush(uint64_t* out) {
        if (kProf && lane() == 0)
            for (int i = 0; i < kBProfSlots; i++)
                if (ph[i]) atomicAdd(reinterpret_cast<unsigned long long*>(&out[i]), ph[i]);
    }
};


// ── lean per-lane walks (the common case) ───────────────────────────────────
// One run header per step: an 8-byte window read, a branch-free varint parse
// and a few selects.  Mask bits are accumulated in registers and written a
// word at a time; index runs are only recorded (their character totals are
// summed afterwards, off the header chain).  Anything unusual — a zero-count
// run, a varint longer than 4 bytes or cut by the stream end, an RLE value cut
// by the stream end, bit width > 32 — returns false and the exact state
// machine (lane_walk.hpp) redoes the stream.
struct Hdr {
    uint32_t lit, count, hl, ok;
};
__device__ __forceinline__ Hdr parse_hdr(uint64_t x, uint32_t avail) {
    Hdr h;
    const uint64_t am = avail >= 8 ? ~0ull : ((1ull << (8 * avail)) - 1ull);
    const uint32_t stops = static_cast<uint32_t>(~x & 0x80808080ull & am);
    h.hl = stops ? (static_cast<uint32_t>(__builtin_ctz(stops)) >> 3) + 1 : 0u;
    uint32_t v = static_cast<uint32_t>((x & 0x7full) | ((x >> 1) & 0x3f80ull) | ((x >> 2) & 0x1fc000ull) |
                                       ((x >> 3) & 0xfe00000ull));
    v &= h.hl >= 4 ? 0x0FFFFFFFu : ((1u << (7 * h.hl)) - 1u);
    h.lit = v & 1u;
    h.count = h.lit ? (v >> 1) * 8u : (v >> 1);
    h.ok = stops != 0 && (v >> 1) != 0;
    return h;
}

// def levels, bit width <= 8: validity mask (word w of this lane's page at
// mask[64 w]) and the non-null count.  Returns false: use the exact walk.
__device__ bool fast_def(const uint32_t* pw, uint32_t psize, uint32_t base, uint32_t size, uint32_t bw,
                         uint32_t md, uint32_t n, uint32_t* mask, uint32_t& nn, bool& above) {
    uint32_t pos = 0, row = 0, acc = 0, fill = 0, wi = 0;
    nn = 0;
    above = false;
    bool ok = true;
    while (row < n) {
        if (pos >= size) break;  // exhausted: remaining levels are 0 (NULL)
        const uint64_t x = lds_u64(pw, base + pos);
        const Hdr h = parse_hdr(x, size - pos);
        if (!h.ok || h.count == 0) { ok = false; break; }
        const uint32_t k = min(h.count, n - row);
        uint32_t bits, nbits = k;
        uint32_t lbit = 0;
        if (!h.lit) {
            if (h.hl >= size - pos) { ok = false; break; }  // value byte cut by the stream end
            const uint32_t v = static_cast<uint32_t>(x >> (8 * h.hl)) & 0xFFu & ((1u << (8 * ((bw + 7) / 8))) - 1u);
            above |= v > md;
            bits = v == md ? 0xFFFFFFFFu : 0u;
            pos += h.hl + (bw + 7) / 8;
        } else {
            if (bw != 1 || md != 1) { ok = false; break; }  // general widths: exact walk
            lbit = (base + pos + h.hl) * 8u;
            bits = 0;
            pos += h.hl + (h.count * bw + 7) / 8;
        }
        // append nbits bits (RLE: repeated pattern; literal: the level bits)
        uint32_t done = 0;
        while (done < nbits) {
            const uint32_t take = min(32u - fill, nbits - done);
            uint32_t chunk = h.lit ? lds_bits(pw, psize, static_cast<uint64_t>(lbit) + done, take) : bits;
            chunk &= take == 32 ? 0xFFFFFFFFu : ((1u << take) - 1u);
            nn += __popc(chunk);
            acc |= chunk << fill;
            fill += take;
            done += take;
            if (fill == 32) {
                mask[64 * wi] = acc;
                wi++;
                acc = 0;
                fill = 0;
            }
        }
        row += k;
    }
    if (fill) mask[64 * wi] = acc;
    return ok;
}

// dictionary index stream, bit width <= 32: run records (count | literal |
// index or bit offset).  Returns false: use the exact walk.
__device__ bool fast_idx(const uint32_t* pw, uint32_t base, uint32_t size, uint32_t bw, uint32_t need,
                         uint32_t dict_n, uint32_t* runs, uint32_t run_cap, uint32_t& nruns) {
    if (bw > 32) return false;
    const uint32_t nb = (bw + 7) / 8;
    uint32_t pos = 0, done = 0;
    nruns = 0;
    while (done < need) {
        if (pos >= size) {  // exhausted: zeros
            if (nruns < run_cap) runs[nruns] = run_rec(need - done, 0u, 0u < dict_n ? 0u : 0xFFFFu);
            nruns++;
            break;
        }
        const uint64_t x = lds_u64(pw, base + pos);
        const Hdr h = parse_hdr(x, size - pos);
        if (!h.ok || h.count == 0) return false;
        const uint32_t k = min(h.count, need - done);
        uint32_t rec;
        if (!h.lit) {
            if (h.hl + nb > size - pos || h.hl + nb > 8) return false;  // value cut by the stream end
            const uint32_t v = nb ? static_cast<uint32_t>(x >> (8 * h.hl)) & (nb >= 4 ? 0xFFFFFFFFu : ((1u << (8 * nb)) - 1u))
                                  : 0u;
            rec = run_rec(k, 0u, static_cast<int32_t>(v) >= 0 && v < dict_n ? v : 0xFFFFu);
            pos += h.hl + nb;
        } else {
            rec = run_rec(k, 1u, (base + pos + h.hl) * 8u);
            pos += h.hl + (h.count * bw + 7) / 8;
        }
        if (nruns < run_cap) runs[nruns] = rec;
        nruns++;
        done += k;
    }
    return true;
}

// character total of a page from its run list (dictionary lengths)
__device__ uint64_t runs_total(const uint32_t* pw, uint32_t psize, const uint32_t* runs, uint32_t nruns, uint32_t bw,
                               uint32_t dict_n, const uint32_t* dtab) {
    uint64_t total = 0;
    for (uint32_t r = 0; r < nruns; r++) {
        const uint32_t rec = runs[r];
        const uint32_t k = run_count(rec), pl = run_payload(rec);
        if (!run_lit(rec)) {
            if (pl != 0xFFFFu) total += static_cast<uint64_t>(k) * (dtab[pl] >> 16);
        } else {
            uint32_t i = 0;
            for (; i + 4 <= k; i += 4) {
                uint32_t v[4];
#pragma unroll
                for (uint32_t u = 0; u < 4; u++)
                    v[u] = lds_bits(pw, psize, static_cast<uint64_t>(pl) + static_cast<uint64_t>(i + u) * bw, bw);
#pragma unroll
                for (uint32_t u = 0; u < 4; u++)
                    if (static_cast<int32_t>(v[u]) >= 0 && v[u] < dict_n) total += dtab[v[u]] >> 16;
            }
            for (; i < k; i++) {
                const uint32_t v = lds_bits(pw, psize, static_cast<uint64_t>(pl) + static_cast<uint64_t>(i) * bw, bw);
                if (static_cast<int32_t>(v) >= 0 && v < dict_n) total += dtab[v] >> 16;
            }
        }
    }
    return total;
}

// ── producer ────────────────────────────────────────────────────────────────
template <bool kProf>
__device__ void batch_produce(const BArgs& a, const BLayout& L, uint8_t* base, Ctrl* ctrl, const uint32_t* dtab,
                              uint32_t dict_n) {
    BProf<kProf> P;
    P.start();
    const uint32_t bw_def = level_bw(a.max_def);
    uint32_t seq = 0;     // batches produced by this workgroup
    uint32_t qnext = 0;   // queue position of the next page
    for (;;) {
        int32_t bt = 0;
        if (lane() == 0) bt = atomicAdd(a.ticket, 1);
        bt = static_cast<int32_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(bt)));
        if (bt >= a.nbatches) break;
        const uint32_t bi = seq & 1u;
        // wait until writers drained this buffer's previous batch
        while (ld_u32(&ctrl->done[bi]) != ld_u32(&ctrl->count[bi])) __builtin_amdgcn_s_sleep(2);
        P.mark(BP_WAITBUF);
        P.count(BP_BATCHES);
        uint8_t* buf = base + L.bufs + bi * L.buf;
        const DevBatch B = a.batches[bt];
        {  // payload of the batch's pages, one contiguous image range
            const uint4* src = reinterpret_cast<const uint4*>(a.bytes + B.img_lo);
            uint4* dst = reinterpret_cast<uint4*>(buf + L.b_pay);
            copy_blocks(dst, src, B.img_bytes / 16, lane(), kWave);
        }
        __builtin_amdgcn_wave_barrier();
        P.mark(BP_STAGE);

        // ── lane-per-page walk ──
        const bool act = lane() < static_cast<uint32_t>(B.np);
        const int32_t pidx = B.p0 + static_cast<int32_t>(lane());
        DevPage pg{};
        if (act) pg = a.pages[pidx];
        const uint32_t pay = static_cast<uint32_t>(pg.off - B.img_lo);  // page copy, batch-relative
        const uint32_t* pw = reinterpret_cast<const uint32_t*>(buf + L.b_pay + pay);
        const uint32_t size = static_cast<uint32_t>(pg.size);
        const uint32_t n = act ? static_cast<uint32_t>(pg.nvals) : 0u;
        uint32_t* mask = reinterpret_cast<uint32_t*>(buf + L.b_mask) + lane();  // word w at mask[64 * w]
        uint32_t* runs = reinterpret_cast<uint32_t*>(buf + L.b_runs + pay);
        const uint32_t run_cap = (static_cast<uint32_t>(pg.size) + 15) / 16 * 4 + 4;  // slot bytes / 4
        auto rd8 = [&](uint32_t a) { return lds_u64(pw, a); };
        int code = 0;
        uint32_t epos = 0, eneed = 0;
        uint32_t nn = 0, nruns = 0, flags = 0, ipos = 0, ibw = 0;
        uint64_t total = 0;
        for (uint32_t w = 0; w < L.mask_words; w++) mask[64 * w] = 0u;
        uint32_t pos = 0, def_base = 0, dl = 0;
        if (act) {
            if (a.max_def > 0) {  // column_reader.cpp:146-170
                if (pos + 4 > size) { code = PQ_ERR_BUFFER; epos = pos; eneed = 4; }
                else {
                    dl = lds_u32a(pw, pos);
                    pos += 4;
                    if (static_cast<uint64_t>(pos) + dl > size) { code = PQ_ERR_BUFFER; epos = pos; eneed = dl; }
                    else { def_base = pos; pos += dl; }
                }
            }
            if (!code && a.max_rep > 0) {
                if (pos + 4 > size) { code = PQ_ERR_BUFFER; epos = pos; eneed = 4; }
                else {
                    const uint32_t rl = lds_u32a(pw, pos);
                    pos += 4;
                    if (static_cast<uint64_t>(pos) + rl > size) { code = PQ_ERR_BUFFER; epos = pos; eneed = rl; }
                    else pos += rl;
                }
            }
            if (!code) {
                if (a.max_def == 0) {
                    for (uint32_t w = 0; w * 32 < n; w++)
                        mask[64 * w] = n - w * 32 >= 32 ? 0xFFFFFFFFu : ((1u << (n - w * 32)) - 1u);
                    nn = n;
                } else {
                    // def levels: rows with level == max_def are non-null
                    const uint32_t md = static_cast<uint32_t>(a.max_def);
                    bool above = false;
                    if (!fast_def(pw, size, def_base, dl, bw_def, md, n, mask, nn, above)) {
                        for (uint32_t w = 0; w < L.mask_words; w++) mask[64 * w] = 0u;
                        nn = 0;
                        above = false;
                        LRle r{def_base, dl, 0, bw_def, 0, 0, 0, 0, 0, 0};
                        uint32_t row = 0;
                        code = lane_rle(r, rd8, n, [&](uint32_t kind, uint32_t k, uint32_t arg) {
                            if (kind == 0) {
                                if (arg > md) above = true;
                                if (arg == md && k) {
                                    nn += k;
                                    uint32_t r0 = row;
                                    const uint32_t r1 = row + k;
                                    while (r0 < r1) {
                                        const uint32_t w = r0 >> 5, b = r0 & 31;
                                        const uint32_t cnt = min(32u - b, r1 - r0);
                                        const uint32_t m = cnt == 32 ? 0xFFFFFFFFu : (((1u << cnt) - 1u) << b);
                                        mask[64 * w] |= m;
                                        r0 += cnt;
                                    }
                                }
                            } else {
                                for (uint32_t i = 0; i < k; i++) {
                                    const uint32_t v = lds_bits(pw, size, static_cast<uint64_t>(arg) + i * bw_def, bw_def);
                                    if (v > md) above = true;
                                    if (v == md) {
                                        nn++;
                                        mask[64 * ((row + i) >> 5)] |= 1u << ((row + i) & 31);
                                    }
                                }
                            }
                            row += k;
                        });
                    }
                    if (!code && above) code = PQ_ERR_UNSUPPORTED;
                }
            }
        }
        P.mark(BP_DEFWALK);
        if (act) {
            if (!code) {  // dictionary indices (column_reader.cpp:196-214)
                if (pos + 1 > size) { code = PQ_ERR_BUFFER; epos = pos; eneed = 1; }
                else {
                    ibw = lds_u32a(pw, pos) & 0xFFu;
                    pos += 1;
                    ipos = pos;
                    if (!fast_idx(pw, pos, size - pos, ibw, nn, dict_n, runs, run_cap, nruns)) {
                        nruns = 0;
                        LRle r{pos, size - pos, 0, ibw, 0, 0, 0, 0, 0, 0};
                        code = lane_rle(r, rd8, nn, [&](uint32_t kind, uint32_t k, uint32_t arg) {
                            if (kind == 0) {
                                const uint32_t idx = static_cast<int32_t>(arg) >= 0 && arg < dict_n ? arg : 0xFFFFu;
                                if (nruns < run_cap) runs[nruns] = run_rec(k, 0u, idx);
                            } else {
                                if (nruns < run_cap) runs[nruns] = run_rec(k, 1u, arg);
                            }
                            nruns++;
                        });
                    }
                    if (!code && nruns <= run_cap) total = runs_total(pw, size, runs, nruns, ibw, dict_n, dtab);
                    if (!code && nruns > run_cap) {  // total from the exact walk, values not kept
                        LRle r{pos, size - pos, 0, ibw, 0, 0, 0, 0, 0, 0};
                        total = 0;
                        (void)lane_rle(r, rd8, nn, [&](uint32_t kind, uint32_t k, uint32_t arg) {
                            if (kind == 0) {
                                if (static_cast<int32_t>(arg) >= 0 && arg < dict_n) total += static_cast<uint64_t>(k) * (dtab[arg] >> 16);
                            } else {
                                for (uint32_t i = 0; i < k; i++) {
                                    const uint32_t v = lds_bits(pw, size, static_cast<uint64_t>(arg) + i * ibw, ibw);
                                    if (static_cast<int32_t>(v) >= 0 && v < dict_n) total += dtab[v] >> 16;
                                }
                            }
                        });
                    }
                    if (nruns > run_cap) flags |= REC_SERIAL;
                }
            }
        }
        if (code) {
            flags = REC_ERR;
            total = 0;
            DevErr* err = a.page_err + pidx;
            err->code = code;
            err->pos = static_cast<int32_t>(epos);
            err->need = static_cast<int32_t>(eneed);
            err->size = static_cast<int32_t>(size);
            atomicOr(a.err_any, 1);
        }
        P.mark(BP_WALK);
        // ── batch prefix and look-back ──
        uint64_t incl = total;
#pragma unroll
        for (int d = 1; d < kWave; d <<= 1) {
            const uint64_t t = __shfl_up(incl, d, kWave);
            if (lane() >= static_cast<uint32_t>(d)) incl += t;
        }
        const uint64_t btotal = __shfl(incl, kWave - 1, kWave);
        const int64_t BG0 = (a.debug & 1) ? static_cast<int64_t>(bt) * 64 * 24 * 512
                                          : *a.base_in + static_cast<int64_t>(look_back(a.status, bt, btotal));
        const int64_t G0 = BG0 + static_cast<int64_t>(incl - total);
        if (act && pidx == a.last_page) {
            *a.base_out = G0 + static_cast<int64_t>(total);
            if (pg.first_row + n == a.nrows_total) a.offsets[a.nrows_total] = G0 + static_cast<int64_t>(total);
        }
        P.mark(BP_LOOKBACK);
        if (act) {
            PageRec* rec = reinterpret_cast<PageRec*>(buf + L.b_recs) + lane();
            rec->G0 = G0;
            rec->first_row = pg.first_row;
            rec->goff = pg.off;
            rec->n = n;
            rec->nn = nn;
            rec->total = static_cast<uint32_t>(total);
            rec->nruns = nruns;
            rec->pay = static_cast<uint32_t>(buf + L.b_pay + pay - base);
            rec->size = size;
            rec->ipos = ipos;
            rec->bw = ibw;
            rec->flags = flags;
            rec->runs = static_cast<uint32_t>(reinterpret_cast<uint8_t*>(runs) - base);
        }
        // publish (the seqlock lets writers read (qstart, count) consistently)
        st_u32(&ctrl->ver[bi], 2 * seq + 1);
        st_u32(&ctrl->qstart[bi], qnext);
        st_u32(&ctrl->done[bi], 0u);
        st_u32(&ctrl->count[bi], static_cast<uint32_t>(B.np));
        st_u32(&ctrl->ver[bi], 2 * seq + 2);
        qnext += static_cast<uint32_t>(B.np);
        st_u32(&ctrl->published, qnext);
        seq++;
    }
    st_u32(&ctrl->finished, 1u);
    P.flush(a.prof);
}

// ── writer ──────────────────────────────────────────────────────────────────
__device__ __forceinline__ void store_block(uint8_t* chars, int64_t blk, uint32_t lo, uint32_t hi, uint4 v) {
    if (lo == 0 && hi == 16) {
        *reinterpret_cast<uint4*>(chars + blk) = v;
    } else {
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
        for (uint32_t bb = lo; bb < hi; bb++) chars[blk + bb] = static_cast<uint8_t>(w[bb >> 2] >> (8 * (bb & 3)));
    }
}

// Characters of one page through the LDS ring (see dict_fused.hip).
__device__ void ring_copy(const BArgs& a, const uint32_t* off, const uint16_t* rsrc, uint32_t* ring,
                          const uint32_t* srcw, uint32_t srcw_last, uint32_t n, int64_t G0, int64_t G1) {
    constexpr uint32_t kRingMask = kRingBytes / 4 - 1;
    int64_t fb = G0 >> 4;
    uint32_t r0 = 0;
    while (r0 < n) {
        const uint32_t r = r0 + lane();
        const uint32_t e = r < n ? off[r + 1] : 0xFFFFFFFFu;
        const int64_t limit = fb * 16 + kRingBytes - 16;
        const uint64_t fit = __ballot(r < n && G0 + static_cast<int64_t>(e) <= limit);
        const uint32_t k = fit == ~0ull ? kWave : static_cast<uint32_t>(__builtin_ctzll(~fit));
        const uint32_t cnt = k ? k : 1u;
        if (lane() < cnt) {
            // all source dwords of a 64-byte segment are read before any
            // destination dword is written (one LDS round trip per segment)
            const uint32_t s0 = off[r];
            const uint32_t len = e - s0;
            const uint32_t src = rsrc[r];
            const int64_t d = G0 + s0;
            const uint32_t lo0 = static_cast<uint32_t>(d & 3);
            const uint32_t nd = (lo0 + len + 3) >> 2;
            const uint32_t a0 = src - lo0;  // >= 1: every value follows a 4-byte length prefix
            const uint32_t sh = a0 & 3, i0 = a0 >> 2;
            const uint32_t lastb = (lo0 + len - 1) & 3;
            const uint32_t dw0 = static_cast<uint32_t>(d >> 2);
            for (uint32_t j0 = 0; j0 < nd && len; j0 += 16) {
                uint32_t x[17];
#pragma unroll
                for (uint32_t k = 0; k < 17; k++) x[k] = srcw[min(i0 + j0 + k, srcw_last)];
#pragma unroll
                for (uint32_t k = 0; k < 16; k++) {
                    const uint32_t j = j0 + k;
                    uint32_t v = __builtin_amdgcn_alignbyte(x[k + 1], x[k], sh);
                    if (j == 0) v &= 0xFFFFFFFFu << (8 * lo0);
                    if (j == nd - 1) v &= 0xFFFFFFFFu >> (8 * (3 - lastb));
                    if (j < nd) atomicOr(&ring[(dw0 + j) & kRingMask], v);
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
        const uint32_t r1 = r0 + cnt;
        const int64_t end = G0 + static_cast<int64_t>(off[r1]);
        const int64_t lb = r1 >= n ? ((end + 15) >> 4) : (end >> 4);
        for (int64_t b = fb + lane(); b < lb; b += kWave) {
            uint4* rb = reinterpret_cast<uint4*>(ring + ((static_cast<uint32_t>(b) * 4) & kRingMask));
            const uint4 v = *rb;
            *rb = make_uint4(0, 0, 0, 0);
            const int64_t blk = b << 4;
            const uint32_t lo = blk < G0 ? static_cast<uint32_t>(G0 - blk) : 0u;
            const uint32_t hi = blk + 16 > G1 ? static_cast<uint32_t>(G1 - blk) : 16u;
            store_block(a.chars, blk, lo, hi, v);
        }
        __builtin_amdgcn_wave_barrier();
        fb = lb;
        r0 = r1;
    }
}

// Byte-wise fallback for pages with a row longer than the ring allows.
__device__ void slow_copy(const BArgs& a, const uint32_t* off, const uint16_t* rsrc, const uint32_t* srcw, uint32_t n,
                          int64_t G0) {
    for (uint32_t r = 0; r < n; r++) {
        const uint32_t s0 = off[r], len = off[r + 1] - s0, src = rsrc[r];
        for (uint32_t q = lane(); q < len; q += kWave)
            a.chars[G0 + s0 + q] = static_cast<uint8_t>((srcw[(src + q) >> 2] >> (8 * ((src + q) & 3))) & 0xFFu);
    }
}

template <bool kProf>
__device__ void batch_write(const BArgs& a, const BLayout& L, uint8_t* base, Ctrl* ctrl, uint8_t* wmem,
                            const uint32_t* dwords, const uint32_t* dtab, uint32_t dict_n) {
    uint16_t* ix = reinterpret_cast<uint16_t*>(wmem + L.w_ix);
    uint32_t* off = reinterpret_cast<uint32_t*>(wmem + L.w_off);
    uint16_t* R = reinterpret_cast<uint16_t*>(wmem + L.w_off);  // rank -> run marks (before off is built)
    uint16_t* rsrc = reinterpret_cast<uint16_t*>(wmem + L.w_rsrc);
    uint32_t* ring = reinterpret_cast<uint32_t*>(wmem + L.w_ring);
    uint16_t* starts = reinterpret_cast<uint16_t*>(wmem + L.w_starts);
    LitRun* lits = reinterpret_cast<LitRun*>(wmem + L.w_lits);
    for (uint32_t i = lane(); i < kRingBytes / 16; i += kWave) reinterpret_cast<uint4*>(ring)[i] = make_uint4(0, 0, 0, 0);
    __builtin_amdgcn_wave_barrier();
    BProf<kProf> P;
    P.start();
    for (;;) {
        uint32_t q = 0;
        if (lane() == 0) q = atomicAdd(&ctrl->next, 1u);
        q = __builtin_amdgcn_readfirstlane(q);
        bool quit = false;
        for (;;) {
            if (q < ld_u32(&ctrl->published)) break;
            if (ld_u32(&ctrl->finished) && q >= ld_u32(&ctrl->published)) { quit = true; break; }
            __builtin_amdgcn_s_sleep(2);
        }
        if (quit) break;
        P.mark(BW_WAIT);
        P.count(BW_PAGES);
        // buffer holding queue position q (stable until its pages are done)
        uint32_t bi = 1, slot = 0;
        for (uint32_t b = 0; b < 2; b++) {
            uint32_t v1, qs, c, v2;
            do {
                v1 = ld_u32(&ctrl->ver[b]);
                qs = ld_u32(&ctrl->qstart[b]);
                c = ld_u32(&ctrl->count[b]);
                v2 = ld_u32(&ctrl->ver[b]);
            } while (v1 != v2 || (v1 & 1u));
            if (q - qs < c) { bi = b; slot = q - qs; break; }
        }
        uint8_t* buf = base + L.bufs + bi * L.buf;
        const PageRec* rec = reinterpret_cast<const PageRec*>(buf + L.b_recs) + slot;
        const uint32_t flags = __builtin_amdgcn_readfirstlane(rec->flags);
        const uint32_t n = __builtin_amdgcn_readfirstlane(rec->n);
        const uint32_t nn = __builtin_amdgcn_readfirstlane(rec->nn);
        const uint32_t nruns = __builtin_amdgcn_readfirstlane(rec->nruns);
        const uint32_t size = __builtin_amdgcn_readfirstlane(rec->size);
        const uint32_t bw = __builtin_amdgcn_readfirstlane(rec->bw);
        const uint32_t* pw = reinterpret_cast<const uint32_t*>(base + __builtin_amdgcn_readfirstlane(rec->pay));
        const uint32_t* runs = reinterpret_cast<const uint32_t*>(base + __builtin_amdgcn_readfirstlane(rec->runs));
        const int64_t G0 = rec->G0;
        const int64_t first_row = rec->first_row;
        const uint32_t* mask = reinterpret_cast<const uint32_t*>(buf + L.b_mask) + slot;  // word w at mask[64 w]
        if (!(flags & REC_ERR) && n) {
            // 1. index of every non-null rank
            if (flags & REC_SERIAL) {
                SRle r;
                srle_init(r, __builtin_amdgcn_readfirstlane(rec->ipos), size - __builtin_amdgcn_readfirstlane(rec->ipos), bw);
                uint32_t nl = 0;
                const uint64_t go = rec->goff;
                const uint8_t* gpage = a.bytes + ((static_cast<uint64_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(go >> 32))) << 32) |
                                                  __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(go)));
                auto put = [&](uint32_t j, uint32_t v) {
                    ix[j] = static_cast<uint16_t>(static_cast<int32_t>(v) >= 0 && v < dict_n ? v : 0xFFFFu);
                };
                (void)srle_walk(r, gpage, nn, put, lits, nl, kLitCap,
                                [&]() { expand_lits(lits, nl, pw, size, bw, put); });
                expand_lits(lits, nl, pw, size, bw, put);
            } else {
                for (uint32_t j = lane(); j < nn; j += kWave) R[j] = 0;
                __builtin_amdgcn_wave_barrier();
                uint32_t carry = 0;
                for (uint32_t k0 = 0; k0 < nruns; k0 += kWave) {
                    const uint32_t k = k0 + lane();
                    const uint32_t rr = k < nruns ? runs[k] : 0u;
                    const uint32_t c = k < nruns ? run_count(rr) : 0u;
                    const uint32_t inc = wave_incl_scan(c);
                    const uint32_t st = carry + inc - c;
                    if (k < nruns && st < nn) {
                        starts[k] = static_cast<uint16_t>(st);
                        R[st] = static_cast<uint16_t>(k);
                    }
                    carry += bcast_last(inc);
                }
                __builtin_amdgcn_wave_barrier();
                uint32_t rmax = 0;
                for (uint32_t j0 = 0; j0 < nn; j0 += 2 * kWave) {
                    const uint32_t ja = j0 + lane(), jb = ja + kWave;
                    uint32_t ra = ja < nn ? R[ja] : 0u;
                    uint32_t rb = jb < nn ? R[jb] : 0u;
                    ra = max(wave_incl_max(ra), rmax);
                    rmax = bcast_last(ra);
                    rb = max(wave_incl_max(rb), rmax);
                    rmax = bcast_last(rb);
                    const uint32_t xa = runs[ra], xb = runs[rb];
                    const uint32_t sa = starts[ra], sb = starts[rb];
                    uint32_t va = run_payload(xa), vb = run_payload(xb);
                    if (run_lit(xa) && ja < nn) {
                        const uint32_t v = lds_bits(pw, size, static_cast<uint64_t>(va) + static_cast<uint64_t>(ja - sa) * bw, bw);
                        va = static_cast<int32_t>(v) >= 0 && v < dict_n ? v : 0xFFFFu;
                    }
                    if (run_lit(xb) && jb < nn) {
                        const uint32_t v = lds_bits(pw, size, static_cast<uint64_t>(vb) + static_cast<uint64_t>(jb - sb) * bw, bw);
                        vb = static_cast<int32_t>(v) >= 0 && v < dict_n ? v : 0xFFFFu;
                    }
                    if (ja < nn) ix[ja] = static_cast<uint16_t>(va);
                    if (jb < nn) ix[jb] = static_cast<uint16_t>(vb);
                }
            }
            __builtin_amdgcn_wave_barrier();
            P.mark(BW_RUNS);
            // 2. rows: validity, rank -> dictionary entry, offsets
            uint32_t rank = 0, run = 0, maxlen = 0;
            for (uint32_t j0 = 0; j0 < n; j0 += kWave) {
                const uint32_t j = j0 + lane();
                const bool in = j < n;
                const uint32_t mw = in ? mask[64 * (j >> 5)] : 0u;
                const bool dv = in && ((mw >> (j & 31)) & 1u);
                const uint64_t m = __ballot(dv);
                const uint32_t k = rank + popc_below(m);
                rank += __popcll(m);
                uint32_t len = 0, src = 0;
                bool valid = false;
                if (dv) {
                    const uint32_t idx = ix[k];
                    if (idx != 0xFFFFu) {
                        const uint32_t e = dtab[idx];
                        src = e & 0xFFFFu;
                        len = e >> 16;
                        valid = true;
                    }
                }
                const uint32_t inc = wave_incl_scan(len);
                const uint32_t ex = run + inc - len;
                maxlen = max(maxlen, len);
                if (in) {
                    off[j] = ex;
                    rsrc[j] = static_cast<uint16_t>(src);
                    if (!(a.debug & 4)) a.offsets[first_row + j] = G0 + ex;
                }
                run += bcast_last(inc);
                // validity bits of rows [first_row + j0, +64)
                const uint64_t vm = __ballot(valid);
                const int64_t Rw = first_row + j0;
                const uint32_t wi = static_cast<uint32_t>(Rw >> 5), sh = static_cast<uint32_t>(Rw & 31);
                const uint32_t cnt = min(64u, n - j0);
                if (lane() < 3) {
                    const uint32_t part = lane() == 0 ? static_cast<uint32_t>(vm << sh)
                                        : lane() == 1 ? static_cast<uint32_t>(sh ? (vm >> (32 - sh)) : (vm >> 32))
                                                      : (sh ? static_cast<uint32_t>(vm >> (64 - sh)) : 0u);
                    const int64_t wlo = static_cast<int64_t>(wi + lane()) * 32;
                    const int64_t rlo = Rw, rhi = Rw + cnt;
                    const bool full = wlo >= first_row && wlo + 32 <= first_row + static_cast<int64_t>(n) &&
                                      wlo >= rlo && wlo + 32 <= rhi;
                    if (wlo < rhi && wlo + 32 > rlo) {
                        if (full) a.validity[wi + lane()] = part;
                        else if (part) atomicOr(&a.validity[wi + lane()], part);
                    }
                }
            }
            if (lane() == 0) off[n] = run;
            __builtin_amdgcn_wave_barrier();
            P.mark(BW_ROWS);
            // 3. characters
            const int64_t G1 = G0 + static_cast<int64_t>(run);
            if (run && !(a.debug & 2)) {
                if (G1 > a.capacity) {
                    if (lane() == 0) atomicOr(a.overflow, 1);
                } else if (bcast_last(wave_incl_max(maxlen)) <= kRingMaxRow) {
                    ring_copy(a, off, rsrc, ring, dwords, a.dict_chars_bytes / 4 - 1, n, G0, G1);
                } else {
                    slow_copy(a, off, rsrc, dwords, n, G0);
                }
            }
            P.mark(BW_CHARS);
        }
        __asm__ __volatile__("" ::: "memory");
        if (lane() == 0) atomicAdd(&ctrl->done[bi], 1u);
        __asm__ __volatile__("" ::: "memory");
    }
    P.flush(a.prof);
}

template <bool kProf>
__global__ void __launch_bounds__(1024) k_ba_batch(BArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t wv = threadIdx.x / kWave;
    const BLayout L = batch_layout(a.rows_cap, a.batch_bytes, a.max_slot);
    uint32_t* dwords = reinterpret_cast<uint32_t*>(smem);
    uint32_t* dtab = reinterpret_cast<uint32_t*>(smem + a.dict_chars_bytes);
    uint32_t dict_n = 0;
    {
        const DevDict d = a.dicts[a.dict_id];
        dict_n = static_cast<uint32_t>(a.dict_count[a.dict_id]);
        const uint4* src = reinterpret_cast<const uint4*>(a.bytes + d.off);
        uint4* dst = reinterpret_cast<uint4*>(dwords);
        copy_blocks(dst, src, a.dict_chars_bytes / 16, threadIdx.x, blockDim.x);
        copy_map(dtab, a.entries + d.entry_base, dict_n, threadIdx.x, blockDim.x, [](uint64_t e) {
            return static_cast<uint32_t>(e & 0xFFFFu) | (static_cast<uint32_t>(e >> 32) << 16);
        });
    }
    uint8_t* base = smem + a.dict_bytes;
    Ctrl* ctrl = reinterpret_cast<Ctrl*>(base + L.ctrl);
    if (threadIdx.x == 0) {
        ctrl->published = 0;
        ctrl->next = 0;
        ctrl->finished = 0;
        for (int i = 0; i < 2; i++) { ctrl->qstart[i] = 0; ctrl->count[i] = 0; ctrl->done[i] = 0; ctrl->ver[i] = 0; }
    }
    __syncthreads();
    if (wv == 0) batch_produce<kProf>(a, L, base, ctrl, dtab, dict_n);
    else batch_write<kProf>(a, L, base, ctrl, base + L.writers + (wv - 1) * L.writer, dwords, dtab, dict_n);
}

void set_batch_attrs() {
    static bool attr = false;
    if (attr) return;
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_ba_batch<false>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_ba_batch<true>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
}

}  // namespace

BatchPlan plan_batch_lds(uint32_t rows_cap, uint32_t batch_bytes, uint32_t max_slot, uint32_t dict_bytes) {
    const BLayout L = batch_layout(rows_cap, batch_bytes, max_slot);
    BatchPlan p{};
    const uint32_t kLds = 160 * 1024;
    const uint32_t fixed = dict_bytes + L.fixed;
    if (fixed + L.writer > kLds) return p;
    p.writers = static_cast<int>(std::min<uint32_t>(15, (kLds - fixed) / L.writer));
    p.lds = fixed + static_cast<uint32_t>(p.writers) * L.writer;
    return p;
}

int batch_occupancy(uint32_t lds_bytes, int waves) {
    int blocks = 0;
    set_batch_attrs();
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, k_ba_batch<false>, waves * kWave, lds_bytes) != hipSuccess)
        return 0;
    return blocks;
}

void launch_ba_batch(hipStream_t s, const BatchLaunch& B) {
    BArgs a;
    a.bytes = B.bytes; a.pages = B.pages; a.batches = B.batches; a.nbatches = B.nbatches;
    a.last_page = B.last_page; a.dicts = B.dicts; a.dict_id = B.dict_id; a.entries = B.entries;
    a.dict_count = B.dict_count; a.max_def = B.max_def; a.max_rep = B.max_rep; a.rows_cap = B.rows_cap;
    a.batch_bytes = B.batch_bytes; a.max_slot = B.max_slot; a.dict_bytes = B.dict_bytes;
    a.dict_chars_bytes = B.dict_chars_bytes; a.status = B.status; a.ticket = B.ticket; a.base_in = B.base_in;
    a.base_out = B.base_out; a.nrows_total = B.nrows_total; a.validity = B.validity; a.offsets = B.offsets;
    a.chars = B.chars; a.capacity = B.capacity; a.overflow = B.overflow; a.page_err = B.page_err;
    a.err_any = B.err_any; a.debug = B.debug; a.prof = B.prof;
    set_batch_attrs();
    const dim3 block((1 + B.writers) * kWave);
    if (a.prof)
        hipLaunchKernelGGL(k_ba_batch<true>, dim3(B.grid), block, B.lds, s, a);
    else
        hipLaunchKernelGGL(k_ba_batch<false>, dim3(B.grid), block, B.lds, s, a);
}

int batch_prof_slots() { return kBProfSlots; }

}  // namespace pqk
