// dict_fused.hip — fast path for BYTE_ARRAY column chunks (SURVEY §8a
// R-DICT-EXPAND / R-PLAIN / R-LEVELS / R-RLE) on gfx950.
//
// k_dict_index   dictionary page -> entry table (column_reader.cpp:128-138,
//                249-253): one wavefront walks the u32 length chain with a
//                register window (window.hpp), ~1 readlane chain per entry.
// k_ba_fused     one launch per column chunk; persistent workgroups, one page
//                per wavefront at a time (ticket queue, pages in file order):
//                  1 page payload -> LDS (16-byte loads)
//                  2 def-level and index streams decoded (rle_decoder.hpp
//                    state machine; run headers via register window, runs
//                    expanded 64 values per step)
//                  3 per-row (source, length) + page-local prefix sum
//                  4 decoupled look-back over page totals -> the page's
//                    first output byte (no separate scan pass)
//                  5 int64 offsets, validity words, and the characters as
//                    16-byte aligned, fully coalesced stores assembled from
//                    the dictionary (or the page) held in LDS.
// The chunk's dictionary sits in LDS once per workgroup.
#include "kernels/device_common.hpp"
#include "kernels/kernels.hpp"
#include "kernels/window.hpp"
#include "pq_gpu.h"

namespace pqk {
namespace {

using namespace dev;

constexpr uint64_t kAgg = 1ull << 62;
constexpr uint64_t kInc = 2ull << 62;
constexpr uint64_t kValMask = (1ull << 62) - 1;
constexpr uint32_t kGatherWin = 512;  // 16-byte blocks per gather window

// ── dictionary entry table ─────────────────────────────────────────────────
// The serial walk keeps its results in LDS and flushes them once: a global
// store inside the loop would make every later window read wait for the
// store to retire (loads and stores share vmcnt).
constexpr int kDictBatch = 4096;  // entries buffered in LDS between flushes

__global__ void __launch_bounds__(64) k_dict_index(const uint8_t* __restrict__ bytes,
                                                   const DevDict* __restrict__ dicts,
                                                   uint64_t* __restrict__ entries,
                                                   int32_t* __restrict__ dict_count,
                                                   DevErr* __restrict__ dict_err,
                                                   int32_t* __restrict__ err_any) {
    __shared__ uint64_t buf[kDictBatch];
    const DevDict d = dicts[blockIdx.x];
    const uint32_t size = static_cast<uint32_t>(d.size);
    DevErr* err = dict_err + blockIdx.x;
    Win w;
    win_init(w, reinterpret_cast<const uint32_t*>(bytes + d.off), (size + 3) / 4);
    uint32_t pos = 0;
    int32_t k = 0, flushed = 0;
    const int32_t n = d.nvals;
    auto flush = [&]() {
        __builtin_amdgcn_wave_barrier();
        for (int32_t i = flushed + static_cast<int32_t>(lane()); i < k; i += kWave)
            entries[d.entry_base + i] = buf[i - flushed];
        __builtin_amdgcn_wave_barrier();
        flushed = k;
    };
    for (; k < n; k++) {
        if (pos + 4 > size) { set_err(err, err_any, PQ_ERR_BUFFER, pos, 4, size); break; }
        uint32_t len = uni(win_u32(w, pos));
        pos += 4;
        if (static_cast<uint64_t>(pos) + len > size) {
            set_err(err, err_any, PQ_ERR_BUFFER, pos, len, size);
            break;
        }
        if (lane() == 0) buf[k - flushed] = (static_cast<uint64_t>(len) << 32) | pos;
        pos += len;
        if (k + 1 - flushed == kDictBatch) { k++; flush(); k--; }
    }
    flush();
    if (lane() == 0) dict_count[blockIdx.x] = k;
}

// ── hybrid stream decode: headers from the register window, literals from LDS
template <class F>
__device__ int rlew_decode(Rle& r, Win& w, const Src& s, uint32_t n, F&& out) {
    uint32_t done = 0;
    while (done < n) {
        if (r.repeat == 0 && r.literal == 0) {
            if (r.pos >= r.size) {  // exhausted: zero-fill (rle_decoder.hpp:20-23)
                for (uint32_t j = done + lane(); j < n; j += kWave) out(j, 0u);
                return 0;
            }
            // varint header (76-86), bounded by the stream size
            uint32_t ind = 0, shift = 0;
            for (;;) {
                uint64_t x = win_u64(w, r.base + r.pos);
                uint32_t avail = min(8u, r.size - r.pos);
                uint32_t i = 0;
                bool end = false;
                for (; i < avail; i++) {
                    uint32_t b = static_cast<uint32_t>(x >> (8 * i)) & 0xFFu;
                    if (shift < 32) ind |= (b & 0x7Fu) << shift;
                    if (!(b & 0x80u)) { end = true; i++; break; }
                    shift += 7;
                }
                r.pos += i;
                if (end || r.pos >= r.size) break;
            }
            ind = uni(ind);
            if (ind & 1u) {
                r.literal = (ind >> 1) * 8u;
                r.lit_start = r.pos;
                r.lit_valid = 1;
                r.lit_bit = 0;
            } else {
                r.repeat = ind >> 1;
                uint32_t nb = min((r.bw + 7) / 8, r.size - r.pos);
                uint64_t x = win_u64(w, r.base + r.pos);
                uint32_t keep = min(nb, 4u);
                r.value = uni(keep == 0 ? 0u : keep >= 4 ? static_cast<uint32_t>(x)
                                                         : static_cast<uint32_t>(x) & ((1u << (8 * keep)) - 1u));
                r.pos += nb;
            }
        }
        if (r.bw > 64) return PQ_ERR_UNSUPPORTED;
        if (r.repeat > 0) {
            uint32_t k = min(r.repeat, n - done);
            for (uint32_t j = lane(); j < k; j += kWave) out(done + j, r.value);
            r.repeat -= k;
            done += k;
        } else {
            if (r.bw > 0 && !r.lit_valid) return PQ_ERR_UNSUPPORTED;
            bool wrapped = r.literal == 0;
            uint32_t k = wrapped ? n - done : min(r.literal, n - done);
            uint64_t bit0 = static_cast<uint64_t>(r.base + r.lit_start) * 8u + r.lit_bit;
            for (uint32_t j = lane(); j < k; j += kWave)
                out(done + j, r.bw ? src_bits(s, bit0 + static_cast<uint64_t>(j) * r.bw, r.bw) : 0u);
            bool finishes = !wrapped && k == r.literal;
            r.lit_bit += k * r.bw;
            r.literal -= k;
            if (finishes && r.bw > 0) r.pos = r.lit_start + (r.lit_bit + 7) / 8;
            done += k;
        }
    }
    return 0;
}

// ── fused page decode + gather ──────────────────────────────────────────────
struct FusedArgs {
    const uint8_t* bytes;
    const DevPage* pages;
    int32_t p0, np;              // this chunk's data pages
    const DevDict* dicts;
    int32_t dict_id;             // dictionary in force for DICT pages (or -1)
    const uint64_t* entries;
    const int32_t* dict_count;
    int32_t max_def, max_rep;
    uint32_t rows_cap;           // max rows of a page (multiple of 64)
    uint32_t stage_bytes;        // max payload bytes (multiple of 16)
    uint32_t wave_bytes;         // LDS bytes per wavefront
    uint32_t dict_bytes;         // LDS bytes of the dictionary region
    uint32_t dict_chars_bytes;   // payload bytes region (multiple of 16)
    uint64_t* status;            // np look-back words (zeroed)
    int32_t* ticket;             // zeroed
    const int64_t* base_in;      // characters before this chunk
    int64_t* base_out;           // characters through this chunk
    int64_t nrows_total;
    uint32_t* validity;
    int64_t* offsets;
    uint8_t* chars;
    int64_t capacity;
    int32_t* overflow;
    DevErr* page_err;
    int32_t* err_any;
    int32_t debug;               // ablation switches (timing only; output invalid)
};

struct WaveMem {
    uint32_t* stage;    // stage_bytes
    uint8_t* lv;        // rows_cap
    uint16_t* ix;       // rows_cap: dict index / plain chars position per rank
    uint16_t* il;       // rows_cap: plain length per rank
    uint16_t* rsrc;     // rows_cap: source position per row
    uint32_t* off;      // rows_cap + 1: page-local char offsets per row
    uint16_t* brow;     // kGatherWin: first row of each 16-byte block
};

__device__ __forceinline__ WaveMem carve(uint8_t* base, const FusedArgs& a) {
    WaveMem m;
    uint8_t* p = base;
    m.stage = reinterpret_cast<uint32_t*>(p); p += a.stage_bytes;
    m.off = reinterpret_cast<uint32_t*>(p); p += 4 * (a.rows_cap + 16);
    m.lv = p; p += a.rows_cap;
    m.ix = reinterpret_cast<uint16_t*>(p); p += 2 * a.rows_cap;
    m.il = reinterpret_cast<uint16_t*>(p); p += 2 * a.rows_cap;
    m.rsrc = reinterpret_cast<uint16_t*>(p); p += 2 * a.rows_cap;
    m.brow = reinterpret_cast<uint16_t*>(p);
    return m;
}

__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, kWave);
    return v;
}

// Decoupled look-back (status[t]: kAgg|aggregate or kInc|inclusive).
__device__ uint64_t look_back(uint64_t* status, int32_t t, uint64_t total) {
    if (t == 0) {
        if (lane() == 0) __hip_atomic_store(&status[0], kInc | total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return 0;
    }
    if (lane() == 0) __hip_atomic_store(&status[t], kAgg | total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint64_t prefix = 0;
    int32_t q = t - 1;
    for (;;) {
        int32_t i = q - static_cast<int32_t>(lane());
        uint64_t s = i >= 0 ? __hip_atomic_load(&status[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kInc;
        uint64_t incm = __ballot((s >> 62) == 2);
        uint64_t notready = __ballot((s >> 62) == 0);
        uint32_t first_inc = incm ? static_cast<uint32_t>(__builtin_ctzll(incm)) : 64u;
        uint64_t upto = first_inc >= 63 ? ~0ull : ((2ull << first_inc) - 1ull);
        if (notready & upto) {
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        uint64_t c = lane() <= first_inc ? (s & kValMask) : 0ull;
        prefix += wave_sum64(c);
        if (first_inc < 64) break;
        q -= 64;
    }
    if (lane() == 0)
        __hip_atomic_store(&status[t], kInc | (prefix + total), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return prefix;
}

// Unaligned dword at LDS byte address a (zero-extended reads stay in bounds).
__device__ __forceinline__ uint32_t lds_u32(const uint32_t* words, uint32_t a) {
    uint32_t w0 = words[a >> 2], w1 = words[(a >> 2) + 1];
    return __builtin_amdgcn_alignbyte(w1, w0, a & 3);
}
__device__ __forceinline__ uint32_t lds_u8(const uint32_t* words, uint32_t a) {
    return (words[a >> 2] >> (8 * (a & 3))) & 0xFFu;
}

__global__ void __launch_bounds__(1024) k_ba_fused(FusedArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t wv = threadIdx.x / kWave;

    // dictionary -> LDS: raw payload words, then (pos | len << 16) per entry
    uint32_t* dwords = reinterpret_cast<uint32_t*>(smem);
    uint32_t* dtab = reinterpret_cast<uint32_t*>(smem + a.dict_chars_bytes);
    uint32_t dict_n = 0;
    if (a.dict_id >= 0) {
        const DevDict d = a.dicts[a.dict_id];
        dict_n = static_cast<uint32_t>(a.dict_count[a.dict_id]);
        const uint4* src = reinterpret_cast<const uint4*>(a.bytes + d.off);
        uint4* dst = reinterpret_cast<uint4*>(dwords);
        for (uint32_t i = threadIdx.x; i < a.dict_chars_bytes / 16; i += blockDim.x) dst[i] = src[i];
        for (uint32_t k = threadIdx.x; k < dict_n; k += blockDim.x) {
            uint64_t e = a.entries[d.entry_base + k];
            dtab[k] = static_cast<uint32_t>(e & 0xFFFFu) | (static_cast<uint32_t>(e >> 32) << 16);
        }
    }
    __syncthreads();
    WaveMem M = carve(smem + a.dict_bytes + wv * a.wave_bytes, a);
    const uint32_t bw_def = level_bw(a.max_def);

    for (;;) {
        int32_t t = 0;
        if (lane() == 0) t = atomicAdd(a.ticket, 1);
        t = __shfl(t, 0, kWave);
        if (t >= a.np) break;
        const int32_t p = a.p0 + t;
        const DevPage pg = a.pages[p];
        DevErr* err = a.page_err + p;
        const uint32_t size = static_cast<uint32_t>(pg.size);
        const uint32_t n = static_cast<uint32_t>(pg.nvals);
        // 1. payload -> LDS (16-byte aligned in the device image)
        {
            const uint4* src = reinterpret_cast<const uint4*>(a.bytes + pg.off);
            uint4* dst = reinterpret_cast<uint4*>(M.stage);
            const uint32_t n16 = (size + 15) / 16;
            for (uint32_t i = lane(); i < n16; i += kWave) dst[i] = src[i];
        }
        __builtin_amdgcn_wave_barrier();
        const Src s{M.stage, nullptr, size};
        Win w;
        win_init(w, M.stage, (size + 3) / 4);
        int code = 0;
        uint32_t epos = 0, eneed = 0;
        // 2. levels (column_reader.cpp:146-170)
        uint32_t pos = 0;
        Rle def, ix;
        if (a.max_def > 0) {
            if (pos + 4 > size) { code = PQ_ERR_BUFFER; epos = pos; eneed = 4; }
            else {
                uint32_t dl = uni(win_u32(w, pos));
                pos += 4;
                if (static_cast<uint64_t>(pos) + dl > size) { code = PQ_ERR_BUFFER; epos = pos; eneed = dl; }
                else { rle_init(def, pos, dl, bw_def); pos += dl; }
            }
        }
        if (!code && a.max_rep > 0) {
            if (pos + 4 > size) { code = PQ_ERR_BUFFER; epos = pos; eneed = 4; }
            else {
                uint32_t rl2 = uni(win_u32(w, pos));
                pos += 4;
                if (static_cast<uint64_t>(pos) + rl2 > size) { code = PQ_ERR_BUFFER; epos = pos; eneed = rl2; }
                else pos += rl2;
            }
        }
        if (!code) {
            if (a.max_def > 0) {
                code = rlew_decode(def, w, s, n, [&](uint32_t j, uint32_t v) { M.lv[j] = static_cast<uint8_t>(v > 255 ? 255 : v); });
            } else {
                for (uint32_t j = lane(); j < n; j += kWave) M.lv[j] = 0;
            }
        }
        __builtin_amdgcn_wave_barrier();
        const bool dict = pg.mode == MODE_DICT;
        uint32_t nn = 0;
        if (!code) {
            uint32_t above = 0;
            for (uint32_t j0 = 0; j0 < n; j0 += kWave) {
                uint32_t j = j0 + lane();
                uint32_t d = j < n ? M.lv[j] : 0u;
                bool isnn = j < n && (dict ? d == static_cast<uint32_t>(a.max_def) : d >= static_cast<uint32_t>(a.max_def));
                nn += __popcll(__ballot(isnn));
                above |= __ballot(j < n && d > static_cast<uint32_t>(a.max_def)) != 0;
            }
            if (dict && above) code = PQ_ERR_UNSUPPORTED;
        }
        // values: dictionary indices or the PLAIN length chain
        if (!code && dict) {
            if (pos + 1 > size) { code = PQ_ERR_BUFFER; epos = pos; eneed = 1; }
            else {
                uint32_t bw = uni(win_u32(w, pos) & 0xFFu);
                pos += 1;
                rle_init(ix, pos, size - pos, bw);
                code = rlew_decode(ix, w, s, nn, [&](uint32_t j, uint32_t v) {
                    M.ix[j] = static_cast<uint16_t>(static_cast<int32_t>(v) >= 0 && v < dict_n ? v : 0xFFFFu);
                });
            }
        } else if (!code) {
            for (uint32_t k = 0; k < nn; k++) {  // column_reader.cpp:249-253
                if (static_cast<uint64_t>(pos) + 4 > size) { code = PQ_ERR_BUFFER; epos = pos; eneed = 4; break; }
                uint32_t len = uni(win_u32(w, pos));
                pos += 4;
                if (static_cast<uint64_t>(pos) + len > size) { code = PQ_ERR_BUFFER; epos = pos; eneed = len; break; }
                if (lane() == 0) { M.ix[k] = static_cast<uint16_t>(pos); M.il[k] = static_cast<uint16_t>(len); }
                pos += len;
            }
        }
        __builtin_amdgcn_wave_barrier();
        // 3. per-row source/length, page-local offsets
        uint64_t total = 0;
        if (!code) {
            uint32_t rank = 0, run = 0;
            for (uint32_t j0 = 0; j0 < n; j0 += kWave) {
                uint32_t j = j0 + lane();
                bool in = j < n;
                uint32_t d = in ? M.lv[j] : 0u;
                bool isnn = in && (dict ? d == static_cast<uint32_t>(a.max_def) : d >= static_cast<uint32_t>(a.max_def));
                uint64_t mask = __ballot(isnn);
                uint32_t k = rank + popc_below(mask);
                rank += __popcll(mask);
                uint32_t len = 0, src = 0;
                bool valid = false;
                if (isnn) {
                    if (dict) {
                        uint32_t idx = M.ix[k];
                        if (idx != 0xFFFFu) {
                            uint32_t e = dtab[idx];
                            src = e & 0xFFFFu;
                            len = e >> 16;
                            valid = true;
                        }
                    } else {
                        src = M.ix[k];
                        len = M.il[k];
                        valid = true;
                    }
                }
                uint32_t inc = wave_incl_scan(len);
                if (in) {
                    M.off[j] = run + inc - len;
                    M.rsrc[j] = static_cast<uint16_t>(src);
                }
                run += bcast_last(inc);
                // validity bits of rows [first_row + j0, +64)
                uint64_t vm = __ballot(valid);
                const int64_t R = pg.first_row + j0;
                const uint32_t wi = static_cast<uint32_t>(R >> 5), sh = static_cast<uint32_t>(R & 31);
                const uint32_t cnt = min(64u, n - j0);
                if (lane() < 3) {
                    uint32_t part = lane() == 0 ? static_cast<uint32_t>(vm << sh)
                                  : lane() == 1 ? static_cast<uint32_t>(sh ? (vm >> (32 - sh)) : (vm >> 32))
                                                : (sh ? static_cast<uint32_t>(vm >> (64 - sh)) : 0u);
                    // bit range of this word covered by the page's rows
                    int64_t wlo = static_cast<int64_t>(wi + lane()) * 32;
                    int64_t rlo = R, rhi = R + cnt;
                    bool full = wlo >= pg.first_row && wlo + 32 <= pg.first_row + static_cast<int64_t>(n) &&
                                wlo >= rlo && wlo + 32 <= rhi;
                    if (wlo < rhi && wlo + 32 > rlo) {
                        if (full) a.validity[wi + lane()] = part;
                        else if (part) atomicOr(&a.validity[wi + lane()], part);
                    }
                }
            }
            if (lane() == 0) M.off[n] = run;
            total = run;
        }
        if (code) {
            if (lane() == 0) {
                err->code = code;
                err->pos = static_cast<int32_t>(epos);
                err->need = static_cast<int32_t>(eneed);
                err->size = static_cast<int32_t>(size);
                atomicOr(a.err_any, 1);
            }
            total = 0;
        }
        __builtin_amdgcn_wave_barrier();
        // 4. page start in the output
        const int64_t G0 = (a.debug & 1) ? static_cast<int64_t>(t) * 24 * n
                                         : *a.base_in + static_cast<int64_t>(look_back(a.status, t, total));
        if (t == a.np - 1 && lane() == 0) {
            *a.base_out = G0 + static_cast<int64_t>(total);
            if (pg.first_row + n == a.nrows_total) a.offsets[a.nrows_total] = G0 + total;
        }
        if (code) continue;
        // 5a. offsets
        if (!(a.debug & 4))
            for (uint32_t j = lane(); j < n; j += kWave) a.offsets[pg.first_row + j] = G0 + M.off[j];
        if (total == 0 || (a.debug & 2)) continue;
        const int64_t G1 = G0 + static_cast<int64_t>(total);
        if (G1 > a.capacity) {
            if (lane() == 0) atomicOr(a.overflow, 1);
            continue;
        }
        // 5b. characters: 16-byte blocks of the global char stream
        const uint32_t* srcw = dict ? dwords : M.stage;
        const int64_t B0 = G0 >> 4;
        const int64_t nb = ((G1 - 1) >> 4) - B0 + 1;
        for (int64_t w0 = 0; w0 < nb; w0 += kGatherWin) {
            const int64_t w1 = min(nb, w0 + static_cast<int64_t>(kGatherWin));
            for (uint32_t r = lane(); r < n; r += kWave) {
                uint32_t s0 = M.off[r], e0 = M.off[r + 1];
                if (e0 <= s0) continue;
                int64_t blo = s0 == 0 ? 0 : ((s0 + G0 + 15) >> 4) - B0;
                int64_t bhi = ((e0 + G0 + 15) >> 4) - B0 - 1;
                blo = max(blo, w0);
                bhi = min(bhi, w1 - 1);
                for (int64_t b = blo; b <= bhi; b++) M.brow[b - w0] = static_cast<uint16_t>(r);
            }
            __builtin_amdgcn_wave_barrier();
            for (int64_t b = w0 + lane(); b < w1; b += kWave) {
                const int64_t blk = (B0 + b) << 4;
                const int64_t gs = max(blk, G0), ge = min(blk + 16, G1);
                uint32_t r = M.brow[b - w0];
                uint32_t q = static_cast<uint32_t>(gs - G0);  // page-local output byte
                uint32_t o = static_cast<uint32_t>(gs - blk);
                const uint32_t oe = static_cast<uint32_t>(ge - blk);
                uint32_t rend = M.off[r + 1];
                uint32_t out[4] = {0, 0, 0, 0};
                // output dword k covers block bytes [4k, 4k+4)
#pragma unroll
                for (uint32_t k = 0; k < 4; k++) {
                    uint32_t lo = max(4 * k, o), hi = min(4 * k + 4, oe);
                    if (lo >= hi) continue;
                    uint32_t ql = q + (lo - o);  // page-local byte of block byte lo
                    while (ql >= rend && r + 1 < n) { r++; rend = M.off[r + 1]; }
                    if (ql + (hi - lo) <= rend) {
                        // whole piece from one row: one unaligned dword read
                        uint32_t sa = M.rsrc[r] + (ql - M.off[r]);
                        uint32_t x = lds_u32(srcw, sa - (lo - 4 * k));
                        uint32_t m = (hi - lo == 4) ? 0xFFFFFFFFu : (((1u << (8 * (hi - lo))) - 1u) << (8 * (lo - 4 * k)));
                        out[k] |= x & m;
                    } else {
                        for (uint32_t bb = lo; bb < hi; bb++) {
                            uint32_t qb = q + (bb - o);
                            while (qb >= rend && r + 1 < n) { r++; rend = M.off[r + 1]; }
                            uint32_t sa = M.rsrc[r] + (qb - M.off[r]);
                            out[k] |= lds_u8(srcw, sa) << (8 * (bb & 3));
                        }
                    }
                }
                if (o == 0 && oe == 16) {
                    *reinterpret_cast<uint4*>(a.chars + blk) = make_uint4(out[0], out[1], out[2], out[3]);
                } else {
                    for (uint32_t bb = o; bb < oe; bb++)
                        a.chars[blk + bb] = static_cast<uint8_t>(out[bb >> 2] >> (8 * (bb & 3)));
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
}

}  // namespace

void launch_dict_index(hipStream_t s, const uint8_t* bytes, const DevDict* dicts, int ndicts,
                       uint64_t* entries, int32_t* dict_count, DevErr* dict_err, int32_t* err_any) {
    if (ndicts <= 0) return;
    hipLaunchKernelGGL(k_dict_index, dim3(ndicts), dim3(64), 0, s, bytes, dicts, entries, dict_count,
                       dict_err, err_any);
}

int fused_occupancy_waves(uint32_t lds_bytes_per_block, int waves_per_block) {
    int blocks = 0;
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_ba_fused),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, k_ba_fused, waves_per_block * kWave,
                                                     lds_bytes_per_block) != hipSuccess)
        return 0;
    return blocks;
}

void launch_ba_fused(hipStream_t s, const FusedLaunch& L) {
    FusedArgs a;
    a.bytes = L.bytes; a.pages = L.pages; a.p0 = L.p0; a.np = L.np; a.dicts = L.dicts;
    a.dict_id = L.dict_id; a.entries = L.entries; a.dict_count = L.dict_count;
    a.max_def = L.max_def; a.max_rep = L.max_rep; a.rows_cap = L.rows_cap;
    a.stage_bytes = L.stage_bytes; a.wave_bytes = L.wave_bytes; a.dict_bytes = L.dict_bytes;
    a.dict_chars_bytes = L.dict_chars_bytes; a.status = L.status; a.ticket = L.ticket;
    a.base_in = L.base_in; a.base_out = L.base_out; a.nrows_total = L.nrows_total;
    a.validity = L.validity; a.offsets = L.offsets; a.chars = L.chars; a.capacity = L.capacity;
    a.overflow = L.overflow; a.page_err = L.page_err; a.err_any = L.err_any; a.debug = L.debug;
    const uint32_t lds = L.dict_bytes + L.waves_per_block * L.wave_bytes;
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_ba_fused),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr = true;
    }
    hipLaunchKernelGGL(k_ba_fused, dim3(L.grid), dim3(L.waves_per_block * kWave), lds, s, a);
}

uint32_t fused_wave_bytes(uint32_t rows_cap, uint32_t stage_bytes) {
    uint32_t b = stage_bytes + 4 * (rows_cap + 16) + rows_cap + 2 * rows_cap * 3 + 2 * kGatherWin;
    return (b + 15) / 16 * 16;
}

}  // namespace pqk
