// dict_pipe.hip — dictionary BYTE_ARRAY decode as three data-parallel passes
// (SURVEY §8a R-DICT-EXPAND, R-RLE, R-LEVELS) for chunks whose data pages all
// use one dictionary that fits in LDS.
//
//   k_pipe_runs   one lane per (page, stream): the def-level stream and the
//                 dictionary-index stream of 32 pages per wavefront, staged
//                 into LDS, have their run headers parsed (rle_decoder.hpp:
//                 36-95) into a run table: (first value, count, RLE value or
//                 literal bit offset).  Streams outside the fast path's shape
//                 (zero-count runs, truncated headers, bit widths > 16, more
//                 than kPipeRunCap runs, a prologue error) mark the page for
//                 the exact serial decoder instead.
//   k_pipe_codes  one wavefront per 512-row tile: run table -> def levels ->
//                 non-null ranks -> dictionary indices (column_reader.cpp:
//                 174-196; out-of-range index -> NULL), as a u16 code per row
//                 (0xFFFF = NULL), plus the tile's character count.  Marked
//                 pages are decoded here by the exact state machine
//                 (stream.hpp), one wavefront per page.
//   (scan)        exclusive scan of the tile character counts (decode.hip).
//   k_pipe_write  persistent workgroups with the dictionary in LDS: int64
//                 offsets, validity words and the characters, every 16-byte
//                 output block assembled in registers from the LDS dictionary
//                 and stored once.
// Only pages of more than 512 rows with def levels need tile_nn, the
// non-null counts of the earlier tiles of their page (k_pipe_codes<true>).
#include "kernels/device_common.hpp"
#include "kernels/kernels.hpp"
#include "kernels/lane_walk.hpp"
#include "kernels/stream.hpp"
#include "pq_gpu.h"

namespace pqk {
namespace {

using namespace dev;

constexpr int kRunWaves = 4;
constexpr int kRunPages = 32;                 // pages per wavefront (2 streams each)
constexpr uint32_t kRunStage = 16384;         // staged payload bytes per wavefront
constexpr uint32_t kFallback = 1u << 31;      // info flag: exact serial decode
constexpr int kCodeWaves = 4;
constexpr uint16_t kNull = 0xFFFFu;
constexpr int kWriteWaves = 8;
constexpr uint32_t kWin = 512;                // 16-byte output blocks per window
constexpr uint32_t kFront = 16;               // zero bytes before the LDS dictionary
constexpr uint32_t kLitCapP = 16;

// run record: x = first value | count << 16, y = literal << 31 | payload
// (RLE value, or the page bit offset of the literal run's first value)
__device__ __forceinline__ uint32_t rr_start(uint2 r) { return r.x & 0xFFFFu; }
__device__ __forceinline__ uint32_t rr_lit(uint2 r) { return r.y >> 31; }
__device__ __forceinline__ uint32_t rr_pay(uint2 r) { return r.y & 0x7FFFFFFFu; }


__global__ void __launch_bounds__(kRunWaves * 64) k_pipe_runs(const uint8_t* __restrict__ bytes,
                                                              const DevPage* __restrict__ pages, int npages,
                                                              int32_t max_def, int32_t max_rep,
                                                              uint2* __restrict__ runs,
                                                              uint32_t* __restrict__ info) {
    __shared__ __attribute__((aligned(16))) uint32_t stage_all[kRunWaves][kRunStage / 4 + 8];
    const uint32_t wv = threadIdx.x / kWave;
    const int g0 = (blockIdx.x * kRunWaves + static_cast<int>(wv)) * kRunPages;
    if (g0 >= npages) return;
    const int g1 = min(npages, g0 + kRunPages);
    uint32_t* stage = stage_all[wv];
    const uint64_t wlo = pages[g0].off;
    const DevPage lastp = pages[g1 - 1];
    const uint64_t whi = lastp.off + static_cast<uint32_t>(max(lastp.size, 0));
    bool staged = whi >= wlo && whi - wlo <= kRunStage;
    if (staged) {  // every page of the group inside the window (image order)
        bool inside = true;
        for (int q = g0 + static_cast<int>(lane()); q < g1; q += kWave) {
            const DevPage pq = pages[q];
            inside &= pq.off >= wlo && pq.off + static_cast<uint32_t>(max(pq.size, 0)) <= whi;
        }
        staged = __ballot(!inside) == 0;
    }
    if (staged) {  // payload slots are 16-byte aligned with >= 16 zero bytes after each
        const uint4* src = reinterpret_cast<const uint4*>(bytes + wlo);
        uint4* dst = reinterpret_cast<uint4*>(stage);
        const uint32_t nb = static_cast<uint32_t>((whi - wlo + 15) / 16) + 1;
        for (uint32_t i = lane(); i < nb; i += kWave) dst[i] = src[i];
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    const uint32_t s = lane() & 1;
    const int p = g0 + static_cast<int>(lane() >> 1);
    const bool act = p < g1;
    uint32_t flag = 0, nrec = 0, bwi = 0;
    if (act) {
        const DevPage pg = pages[p];
        const uint32_t size = static_cast<uint32_t>(max(pg.size, 0));
        const uint32_t n = static_cast<uint32_t>(max(pg.nvals, 0));
        const uint32_t sbase = static_cast<uint32_t>(pg.off - wlo);
        const uint8_t* gp = bytes + pg.off;
        auto rd = [&](uint32_t a) -> uint64_t { return staged ? lds_u64(stage, sbase + a) : gld8(gp, a); };
        // prologue (column_reader.cpp:146-182); any error -> exact decoder
        uint32_t pos = 0, dbase = 0, dlen = 0;
        if (n > 65535u) flag = 1;
        if (!flag && max_def > 0) {
            if (size < 4) flag = 1;
            else {
                dlen = static_cast<uint32_t>(rd(0));
                pos = 4;
                if (static_cast<uint64_t>(pos) + dlen > size) flag = 1;
                else { dbase = 4; pos += dlen; }
            }
        }
        if (!flag && max_rep > 0) {
            if (pos + 4 > size) flag = 1;
            else {
                const uint32_t rl = static_cast<uint32_t>(rd(pos));
                pos += 4;
                if (static_cast<uint64_t>(pos) + rl > size) flag = 1;
                else pos += rl;
            }
        }
        if (!flag) {
            if (pos + 1 > size) flag = 1;
            else { bwi = static_cast<uint32_t>(rd(pos)) & 0xFFu; pos += 1; }
        }
        if (!flag && bwi > 16) flag = 1;
        if (!flag && (s == 1 || max_def > 0)) {
            const uint32_t base = s ? pos : dbase;
            const uint32_t end = s ? size : dbase + dlen;
            const uint32_t bw = s ? bwi : level_bw(max_def);
            const uint32_t nbv = (bw + 7) / 8;
            uint2* out = runs + (static_cast<size_t>(p) * 2 + s) * kPipeRunCap;
            uint32_t cnt = 0, q = base;
            while (cnt < n) {
                if (nrec == kPipeRunCap) { flag = 1; break; }
                if (q >= end) {  // exhausted: the rest of the batch is 0 (rle_decoder.hpp:20-23)
                    out[nrec++] = make_uint2(cnt | ((n - cnt) << 16), 0u);
                    break;
                }
                const uint64_t x = rd(q);
                // varint header (76-86), at most 5 bytes, inside the stream
                const uint64_t stop = ~x & 0x8080808080ull;
                if (!stop) { flag = 1; break; }
                const uint32_t hl = static_cast<uint32_t>(__builtin_ctzll(stop)) / 8 + 1;
                if (q + hl > end) { flag = 1; break; }
                const uint64_t xm = hl >= 8 ? x : (x & ((1ull << (8 * hl)) - 1));
                const uint32_t ind = static_cast<uint32_t>((xm & 0x7Full) | ((xm >> 1) & 0x3F80ull) |
                                                           ((xm >> 2) & 0x1FC000ull) | ((xm >> 3) & 0xFE00000ull) |
                                                           ((xm >> 4) & 0xF0000000ull));
                q += hl;
                const uint32_t left = n - cnt;
                if (ind & 1u) {  // literal run: (ind >> 1) groups of 8 (41-46)
                    const uint32_t g = ind >> 1;
                    if (g == 0) { flag = 1; break; }  // zero-group run: counter wraps
                    const uint64_t c8 = static_cast<uint64_t>(g) * 8;
                    const uint32_t c = c8 < left ? static_cast<uint32_t>(c8) : left;
                    out[nrec++] = bw ? make_uint2(cnt | (c << 16), 0x80000000u | (q * 8))
                                     : make_uint2(cnt | (c << 16), 0u);
                    cnt += c;
                    const uint64_t nq = static_cast<uint64_t>(q) + static_cast<uint64_t>(g) * bw;
                    q = nq > end ? end : static_cast<uint32_t>(nq);
                } else {  // repeated run (48-50, 88-95)
                    const uint32_t rep = ind >> 1;
                    if (rep == 0) { flag = 1; break; }  // zero-count run: stale literal cursor
                    if (q + nbv > end) { flag = 1; break; }
                    const uint32_t v = nbv ? static_cast<uint32_t>(x >> (8 * hl)) & ((1u << (8 * nbv)) - 1u) : 0u;
                    const uint32_t c = rep < left ? rep : left;
                    out[nrec++] = make_uint2(cnt | (c << 16), v);
                    cnt += c;
                    q += nbv;
                }
            }
        }
    }
    const uint32_t oflag = static_cast<uint32_t>(__shfl_xor(static_cast<int>(flag), 1));
    const uint32_t orec = static_cast<uint32_t>(__shfl_xor(static_cast<int>(nrec), 1));
    if (act && s == 0)
        info[p] = ((flag | oflag) ? kFallback : 0u) | nrec | (orec << 8) | (bwi << 16);
}

// ── per-tile codes ─────────────────────────────────────────────────────────
struct CodeLds {
    uint2 recd[kPipeRunCap];
    uint2 reci[kPipeRunCap];
    uint8_t mark[kTileRows];
    uint8_t mark2[kTileRows];
    uint64_t vm[kTileRows / 64];
};

struct CodeArgs {
    const uint8_t* bytes;
    const DevPage* pages;
    const DevTile* tiles;
    int ntiles;
    const int32_t* page_tile0;
    int32_t max_def, max_rep;
    const DevDict* dicts;
    int32_t dict_id;
    const uint64_t* entries;
    const int32_t* dict_count;
    const uint2* runs;
    const uint32_t* info;
    int32_t* tile_nn;
    uint16_t* codes;
    int64_t* tile_chars;
    DevErr* page_err;
    int32_t* err_any;
};

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) { return bcast_last(wave_incl_scan(v)); }

// Rows of a page the decode failed on: NULL codes, no characters.
__device__ void fail_page(const CodeArgs& a, const DevPage& pg, int32_t t0, uint32_t n) {
    for (uint32_t j = lane(); j < n; j += kWave) a.codes[pg.first_row + j] = kNull;
    for (uint32_t t = lane(); t * kTileRows < n; t += kWave) a.tile_chars[t0 + t] = 0;
}

// Exact decoder for a marked page: the reference state machine (stream.hpp)
// over the page in HBM, tile by tile; same error order as k_ba_fused.
__device__ void exact_page(const CodeArgs& a, CodeLds& L, int p, uint32_t dict_n, uint32_t ebase) {
    const DevPage pg = a.pages[p];
    const uint8_t* page = a.bytes + pg.off;
    const uint32_t size = static_cast<uint32_t>(max(pg.size, 0));
    const uint32_t n = static_cast<uint32_t>(max(pg.nvals, 0));
    const int32_t t0 = a.page_tile0[p];
    DevErr* err = a.page_err + p;
    uint8_t* lv = L.mark;
    uint16_t* ix = reinterpret_cast<uint16_t*>(L.recd);
    LitRun* lits = reinterpret_cast<LitRun*>(L.reci);
    const uint32_t md = static_cast<uint32_t>(a.max_def);
    uint32_t pos = 0, dbase = 0, dlen = 0;
    auto fail = [&](int code, uint32_t ep, uint32_t need) {
        set_err(err, a.err_any, code, ep, need, size);
        fail_page(a, pg, t0, n);
    };
    if (a.max_def > 0) {
        if (pos + 4 > size) return fail(PQ_ERR_BUFFER, pos, 4);
        dlen = suni(sload_u32(page, pos));
        pos += 4;
        if (static_cast<uint64_t>(pos) + dlen > size) return fail(PQ_ERR_BUFFER, pos, dlen);
        dbase = pos;
        pos += dlen;
    }
    if (a.max_rep > 0) {
        if (pos + 4 > size) return fail(PQ_ERR_BUFFER, pos, 4);
        const uint32_t rl = suni(sload_u32(page, pos));
        pos += 4;
        if (static_cast<uint64_t>(pos) + rl > size) return fail(PQ_ERR_BUFFER, pos, rl);
        pos += rl;
    }
    const uint32_t bwd = level_bw(a.max_def);
    uint32_t nl = 0;
    auto put_lv = [&](uint32_t j, uint32_t v) { lv[j] = static_cast<uint8_t>(v > 255 ? 255 : v); };
    auto expand = [&](const SRle& r, auto&& put) {
        __builtin_amdgcn_wave_barrier();
        for (uint32_t k = 0; k < nl; k++) {
            const LitRun R = lits[k];
            const uint64_t b0 = (static_cast<uint64_t>(R.bit0_hi) << 32) | R.bit0_lo;
            for (uint32_t j = lane(); j < R.count; j += kWave)
                put(R.start + j, gbits(page, size, b0 + static_cast<uint64_t>(j) * r.bw, r.bw));
        }
        nl = 0;
        __builtin_amdgcn_wave_barrier();
    };
    // pass 1: every def level (column_reader.cpp:146-154), then the levels check
    if (a.max_def > 0) {
        SRle def;
        srle_init(def, dbase, dlen, bwd);
        for (uint32_t r0 = 0; r0 < n; r0 += kTileRows) {
            const uint32_t m = min(n - r0, static_cast<uint32_t>(kTileRows));
            const int rc = srle_walk(def, page, m, put_lv, lits, nl, kLitCapP, [&]() { expand(def, put_lv); });
            if (rc) return fail(rc, 0, 0);
            expand(def, put_lv);
            bool above = false;
            for (uint32_t j = lane(); j < m; j += kWave) above |= lv[j] > md;
            if (__ballot(above)) return fail(PQ_ERR_UNSUPPORTED, 0, 0);
        }
    }
    // dictionary index stream (179-182)
    if (pos + 1 > size) return fail(PQ_ERR_BUFFER, pos, 1);
    const uint32_t bwi = suni(sload_u32(page, pos) & 0xFFu);
    pos += 1;
    SRle def, idx;
    srle_init(def, dbase, dlen, bwd);
    srle_init(idx, pos, size - pos, bwi);
    auto put_ix = [&](uint32_t k, uint32_t v) {
        ix[k] = static_cast<uint16_t>(static_cast<int32_t>(v) >= 0 && v < dict_n ? v : kNull);
    };
    for (uint32_t r0 = 0, ti = 0; r0 < n; r0 += kTileRows, ti++) {
        const uint32_t m = min(n - r0, static_cast<uint32_t>(kTileRows));
        if (a.max_def > 0) {
            const int rc = srle_walk(def, page, m, put_lv, lits, nl, kLitCapP, [&]() { expand(def, put_lv); });
            if (rc) return fail(rc, 0, 0);
            expand(def, put_lv);
        } else {
            for (uint32_t j = lane(); j < m; j += kWave) lv[j] = 0;
            __builtin_amdgcn_wave_barrier();
        }
        uint32_t nn = 0;
        for (uint32_t j0 = 0; j0 < m; j0 += kWave) {
            const uint32_t j = j0 + lane();
            const uint64_t vm = __ballot(j < m && lv[j] == md);
            if (lane() == 0) L.vm[j0 / kWave] = vm;
            nn += __popcll(vm);
        }
        const int rc = srle_walk(idx, page, nn, put_ix, lits, nl, kLitCapP, [&]() { expand(idx, put_ix); });
        if (rc) return fail(rc, 0, 0);
        expand(idx, put_ix);
        uint32_t chars = 0, rank = 0;
        for (uint32_t j0 = 0; j0 < m; j0 += kWave) {
            const uint32_t j = j0 + lane();
            const uint64_t vm = L.vm[j0 / kWave];
            const bool nnul = (vm >> lane()) & 1ull;
            const uint32_t k = rank + popc_below(vm);
            rank += __popcll(vm);
            uint16_t code = kNull;
            if (nnul) {
                code = ix[k];
                if (code != kNull) chars += static_cast<uint32_t>(a.entries[ebase + code] >> 32);
            }
            if (j < m) a.codes[pg.first_row + r0 + j] = code;
        }
        chars = wave_sum(chars);
        if (lane() == 0) a.tile_chars[t0 + ti] = chars;
        __builtin_amdgcn_wave_barrier();
    }
}

// The run covering value `v` among `nr` records held two per lane in LDS:
// (number of starts <= v) - 1.
__device__ __forceinline__ uint32_t run_at(const uint2* rec, uint32_t nr, uint32_t v) {
    const bool a0 = lane() < nr && rr_start(rec[lane()]) <= v;
    const bool a1 = lane() + kWave < nr && rr_start(rec[lane() + kWave]) <= v;
    return static_cast<uint32_t>(__popcll(__ballot(a0)) + __popcll(__ballot(a1))) - 1u;
}

template <bool kCount>
__global__ void __launch_bounds__(kCodeWaves * 64) k_pipe_codes(CodeArgs a) {
    __shared__ CodeLds lds_all[kCodeWaves];
    const int wv = static_cast<int>(threadIdx.x / kWave);
    const int t = blockIdx.x * kCodeWaves + wv;
    if (t >= a.ntiles) return;
    CodeLds& L = lds_all[wv];
    const DevTile T = a.tiles[t];
    const int p = T.page;
    const uint32_t inf = a.info[p];
    const uint32_t dict_n = static_cast<uint32_t>(a.dict_count[a.dict_id]);
    const uint32_t ebase = static_cast<uint32_t>(a.dicts[a.dict_id].entry_base);
    if (inf & kFallback) {
        if (!kCount && T.row0 == 0) exact_page(a, L, p, dict_n, ebase);
        return;
    }
    const DevPage pg = a.pages[p];
    const uint8_t* page = a.bytes + pg.off;
    const uint32_t size = static_cast<uint32_t>(max(pg.size, 0));
    const uint32_t nd = inf & 0xFFu, ni = (inf >> 8) & 0xFFu, bwi = (inf >> 16) & 0xFFu;
    const uint32_t r0 = static_cast<uint32_t>(T.row0), m = static_cast<uint32_t>(T.nrows);
    const uint32_t md = static_cast<uint32_t>(a.max_def), bwd = level_bw(a.max_def);
    const uint2* rd_ = a.runs + static_cast<size_t>(p) * 2 * kPipeRunCap;

    // def levels of rows [r0, r0 + m)
    uint32_t nn = 0;
    if (a.max_def > 0) {
        for (uint32_t k = lane(); k < nd; k += kWave) L.recd[k] = rd_[k];
        for (uint32_t j = lane(); j < m; j += kWave) L.mark[j] = 0;
        __builtin_amdgcn_wave_barrier();
        const uint32_t rd0 = run_at(L.recd, nd, r0);
        for (uint32_t k = lane(); k < nd; k += kWave) {
            const uint32_t st = rr_start(L.recd[k]);
            if (k > rd0 && st < r0 + m) L.mark[st - r0] = static_cast<uint8_t>(k - rd0);
        }
        __builtin_amdgcn_wave_barrier();
        uint32_t carry = 0;
        bool above = false;
        for (uint32_t j0 = 0; j0 < m; j0 += kWave) {
            const uint32_t j = j0 + lane();
            const bool in = j < m;
            const uint32_t mx = max(wave_incl_max(in ? L.mark[j] : 0u), carry);
            carry = bcast_last(mx);
            const uint2 R = L.recd[rd0 + mx];
            uint32_t lvl = rr_pay(R);
            if (rr_lit(R)) lvl = gbits(page, size, rr_pay(R) + static_cast<uint64_t>(r0 + j - rr_start(R)) * bwd, bwd);
            const uint64_t vm = __ballot(in && lvl == md);
            above |= in && lvl > md;
            if (lane() == 0) L.vm[j0 / kWave] = vm;
            nn += __popcll(vm);
        }
        if (__ballot(above)) {  // levels above max_def: outside the supported format
            set_err(a.page_err + p, a.err_any, PQ_ERR_UNSUPPORTED, 0, 0, size);
            if (!kCount) {
                for (uint32_t j = lane(); j < m; j += kWave) a.codes[pg.first_row + r0 + j] = kNull;
                if (lane() == 0) a.tile_chars[t] = 0;
            }
            return;
        }
    } else {
        nn = m;
        for (uint32_t j0 = 0; j0 < m; j0 += kWave) {
            const uint64_t vm = __ballot(j0 + lane() < m);
            if (lane() == 0) L.vm[j0 / kWave] = vm;
        }
    }
    if (kCount) {
        if (lane() == 0) a.tile_nn[t] = static_cast<int32_t>(nn);
        return;
    }
    // first rank of the tile
    uint32_t k0 = 0;
    if (a.max_def == 0) k0 = r0;
    else {
        const int32_t tp = a.page_tile0[p];
        uint32_t sum = 0;
        for (int32_t q = tp + static_cast<int32_t>(lane()); q < t; q += kWave) sum += static_cast<uint32_t>(a.tile_nn[q]);
        k0 = wave_sum(sum);
    }
    // dictionary indices of ranks [k0, k0 + nn)
    const uint2* ri_ = rd_ + kPipeRunCap;
    for (uint32_t k = lane(); k < ni; k += kWave) L.reci[k] = ri_[k];
    for (uint32_t q = lane(); q < nn; q += kWave) L.mark2[q] = 0;
    __builtin_amdgcn_wave_barrier();
    uint32_t ri0 = 0;
    if (nn) {
        ri0 = run_at(L.reci, ni, k0);
        for (uint32_t k = lane(); k < ni; k += kWave) {
            const uint32_t st = rr_start(L.reci[k]);
            if (k > ri0 && st < k0 + nn) L.mark2[st - k0] = static_cast<uint8_t>(k - ri0);
        }
        __builtin_amdgcn_wave_barrier();
        uint32_t carry = 0;
        for (uint32_t q0 = 0; q0 < nn; q0 += kWave) {
            const uint32_t q = q0 + lane();
            const uint32_t mx = max(wave_incl_max(q < nn ? L.mark2[q] : 0u), carry);
            carry = bcast_last(mx);
            if (q < nn) L.mark2[q] = static_cast<uint8_t>(mx);
        }
        __builtin_amdgcn_wave_barrier();
    }
    uint32_t chars = 0, rank = 0;
    for (uint32_t j0 = 0; j0 < m; j0 += kWave) {
        const uint32_t j = j0 + lane();
        const uint64_t vm = L.vm[j0 / kWave];
        const bool nnul = (vm >> lane()) & 1ull;
        const uint32_t k = rank + popc_below(vm);
        rank += __popcll(vm);
        uint16_t code = kNull;
        if (nnul) {
            const uint2 R = L.reci[ri0 + L.mark2[k]];
            uint32_t v = rr_pay(R);
            if (rr_lit(R)) v = gbits(page, size, rr_pay(R) + static_cast<uint64_t>(k0 + k - rr_start(R)) * bwi, bwi);
            if (v < dict_n) {
                code = static_cast<uint16_t>(v);
                chars += static_cast<uint32_t>(a.entries[ebase + v] >> 32);
            }
        }
        if (j < m) a.codes[pg.first_row + r0 + j] = code;
    }
    chars = wave_sum(chars);
    if (lane() == 0) a.tile_chars[t] = chars;
}

// ── offsets, validity, characters ──────────────────────────────────────────
struct WriteLds {
    uint2 ri[kTileRows + 1];  // (tile-relative first byte, dictionary byte) per row
    uint16_t brow[kWin];      // row holding each block's first byte
    uint32_t pad[2];
};

struct WriteArgs {
    const uint8_t* bytes;
    const DevPage* pages;
    const DevTile* tiles;
    int ntiles;
    const DevDict* dicts;
    int32_t dict_id;
    const uint64_t* entries;
    const int32_t* dict_count;
    const uint16_t* codes;
    const int64_t* tile_base;
    int64_t nrows_total;
    const int64_t* total;
    int64_t capacity;
    int32_t* overflow;
    uint32_t* validity;
    int64_t* offsets;
    uint8_t* chars;
    uint32_t dict_chars_bytes, dict_bytes;
    int debug;  // ablation: 2 = no characters, 4 = no offsets/validity stores
};

// bits [R, R + cnt) of the validity bitmap from a 64-row ballot; words wholly
// inside [lo, hi) and [R, R + cnt) are stored, the others ORed.
__device__ __forceinline__ void put_valid(uint32_t* validity, int64_t R, uint32_t cnt, uint64_t vm, int64_t lo,
                                          int64_t hi) {
    const uint32_t sh = static_cast<uint32_t>(R & 31);
    const int64_t w0 = R >> 5;
    if (lane() < 3) {
        const uint32_t part = lane() == 0 ? static_cast<uint32_t>(vm << sh)
                            : lane() == 1 ? static_cast<uint32_t>(sh ? (vm >> (32 - sh)) : (vm >> 32))
                                          : (sh ? static_cast<uint32_t>(vm >> (64 - sh)) : 0u);
        const int64_t wlo = (w0 + lane()) * 32;
        const int64_t rhi = R + cnt;
        if (wlo < rhi && wlo + 32 > R) {
            if (wlo >= lo && wlo + 32 <= hi && wlo >= R && wlo + 32 <= rhi) validity[w0 + lane()] = part;
            else if (part) atomicOr(&validity[w0 + lane()], part);
        }
    }
}

__global__ void __launch_bounds__(kWriteWaves * 64) k_pipe_write(WriteArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    // [kFront zero bytes][dictionary payload][entry table][per-wave scratch]
    uint32_t* dwa = reinterpret_cast<uint32_t*>(smem);
    uint32_t* dw = reinterpret_cast<uint32_t*>(smem + kFront);
    uint32_t* dtab = reinterpret_cast<uint32_t*>(smem + kFront + a.dict_chars_bytes);
    const uint32_t wv = threadIdx.x / kWave;
    WriteLds& S = reinterpret_cast<WriteLds*>(smem + a.dict_bytes)[wv];
    const DevDict d = a.dicts[a.dict_id];
    const uint32_t dict_n = static_cast<uint32_t>(a.dict_count[a.dict_id]);
    {
        const uint4* src = reinterpret_cast<const uint4*>(a.bytes + d.off);
        uint4* dst = reinterpret_cast<uint4*>(dw);
        for (uint32_t i = threadIdx.x; i < a.dict_chars_bytes / 16; i += blockDim.x) dst[i] = src[i];
        for (uint32_t k = threadIdx.x; k < dict_n; k += blockDim.x) {
            const uint64_t e = a.entries[d.entry_base + k];
            dtab[k] = static_cast<uint32_t>(e & 0xFFFFu) | (static_cast<uint32_t>(e >> 32) << 16);
        }
    }
    __syncthreads();
    // each wavefront owns a contiguous run of tiles (consecutive rows): the
    // descriptors of up to 64 tiles are loaded at once, one per lane, and the
    // next tile's codes are loaded before this tile's stores are issued
    const int nw = static_cast<int>(gridDim.x) * kWriteWaves;
    const int per = (a.ntiles + nw - 1) / nw;
    const int ta = static_cast<int>(blockIdx.x * kWriteWaves + wv) * per;
    const int tb = min(a.ntiles, ta + per);
    for (int c0 = ta; c0 < tb; c0 += kWave) {
        const int cn = min(kWave, tb - c0);
        int64_t myR0 = 0, myG0 = 0;
        uint32_t mym = 0;
        if (static_cast<int>(lane()) < cn) {
            const DevTile T = a.tiles[c0 + lane()];
            myR0 = a.pages[T.page].first_row + T.row0;
            mym = static_cast<uint32_t>(T.nrows);
            myG0 = a.tile_base[c0 + lane()];
        }
        auto rl64 = [](int64_t v, int i) -> int64_t {
            const uint32_t lo = __builtin_amdgcn_readlane(static_cast<uint32_t>(v), i);
            const uint32_t hi = __builtin_amdgcn_readlane(static_cast<uint32_t>(static_cast<uint64_t>(v) >> 32), i);
            return static_cast<int64_t>((static_cast<uint64_t>(hi) << 32) | lo);
        };
        uint32_t cd[kTileRows / kWave];
        auto load_codes = [&](int i) {
            const int64_t R = rl64(myR0, i);
            const uint32_t mm = __builtin_amdgcn_readlane(mym, i);
#pragma unroll
            for (int k = 0; k < kTileRows / kWave; k++) {
                const uint32_t j = k * kWave + lane();
                cd[k] = j < mm ? a.codes[R + j] : kNull;
            }
        };
        load_codes(0);
        for (int i = 0; i < cn; i++) {
            const int64_t R0 = rl64(myR0, i);
            const int64_t G0 = rl64(myG0, i);
            const uint32_t m = __builtin_amdgcn_readlane(mym, i);
            uint32_t cur[kTileRows / kWave];
#pragma unroll
            for (int k = 0; k < kTileRows / kWave; k++) cur[k] = cd[k];
            if (i + 1 < cn) load_codes(i + 1);
            uint32_t run = 0;
#pragma unroll
            for (int k = 0; k < kTileRows / kWave; k++) {
                const uint32_t j0 = k * kWave;
                if (j0 >= m) break;
                const uint32_t j = j0 + lane();
                const bool in = j < m;
                const uint32_t code = cur[k];
                const bool valid = code < dict_n;
                const uint32_t e = valid ? dtab[code] : 0u;
                const uint32_t len = e >> 16;
                const uint32_t inc = wave_incl_scan(len);
                const uint32_t ex = run + inc - len;
                if (in) {
                    S.ri[j] = make_uint2(ex, e & 0xFFFFu);
                    if (!(a.debug & 4)) a.offsets[R0 + j] = G0 + ex;
                }
                run += bcast_last(inc);
                const uint64_t vmask = __ballot(valid);
                if (!(a.debug & 4)) put_valid(a.validity, R0 + j0, min(64u, m - j0), vmask, R0, R0 + m);
            }
            if (lane() == 0) S.ri[m] = make_uint2(run, 0u);
            if (R0 + m == a.nrows_total && lane() == 0) a.offsets[a.nrows_total] = *a.total;
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            const uint32_t total = run;
            if (total == 0 || (a.debug & 2)) continue;
            if (G0 + total > a.capacity) {  // output too small: the host grows it and re-runs
                if (lane() == 0) atomicOr(a.overflow, 1);
                continue;
            }
            const int64_t G1 = G0 + total;
            const int64_t B0 = G0 >> 4;
            const uint32_t nb = static_cast<uint32_t>(((G1 - 1) >> 4) - B0 + 1);
            const uint32_t mis = static_cast<uint32_t>(G0 & 15);
            for (uint32_t w0 = 0; w0 < nb; w0 += kWin) {
                const uint32_t w1 = min(nb, w0 + kWin);
                // row r owns the blocks whose first in-tile byte lies in it
                for (uint32_t r = lane(); r < m; r += kWave) {
                    const uint32_t s = S.ri[r].x, e = S.ri[r + 1].x;
                    if (e <= s) continue;
                    uint32_t blo = s == 0 ? 0u : (s + mis + 15) / 16;
                    uint32_t bhi = (e + mis + 15) / 16 - 1;
                    blo = max(blo, w0);
                    bhi = min(bhi, w1 - 1);
                    for (uint32_t b = blo; b <= bhi; b++) S.brow[b - w0] = static_cast<uint16_t>(r);
                }
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                for (uint32_t b = w0 + lane(); b < w1; b += kWave) {
                    // tile-relative byte of the block start (negative before G0);
                    // each overlapping row contributes one masked 16-byte segment
                    const int32_t a0 = static_cast<int32_t>(b * 16) - static_cast<int32_t>(mis);
                    uint32_t r = S.brow[b - w0];
                    uint2 cur = S.ri[r], nxt = S.ri[r + 1];
                    uint32_t o0 = 0, o1 = 0, o2 = 0, o3 = 0;
                    for (;;) {
                        const int32_t lo = max(static_cast<int32_t>(cur.x) - a0, 0);
                        const int32_t hi = min(static_cast<int32_t>(nxt.x) - a0, 16);
                        if (hi > lo) {
                            const uint32_t base = cur.y + kFront + static_cast<uint32_t>(a0 - static_cast<int32_t>(cur.x));
                            const uint32_t wi = base >> 2, sh = base & 3;
                            const uint32_t s0 = dwa[wi], s1 = dwa[wi + 1], s2 = dwa[wi + 2], s3 = dwa[wi + 3],
                                           s4 = dwa[wi + 4];
                            auto fmask = [](int32_t x, uint64_t& ml, uint64_t& mh) {
                                ml = x >= 8 ? ~0ull : ((1ull << (8 * x)) - 1);
                                mh = x <= 8 ? 0ull : (x >= 16 ? ~0ull : ((1ull << (8 * (x - 8))) - 1));
                            };
                            uint64_t hl, hh, ll, lh;
                            fmask(hi, hl, hh);
                            fmask(lo, ll, lh);
                            const uint64_t ml = hl & ~ll, mh = hh & ~lh;
                            o0 |= __builtin_amdgcn_alignbyte(s1, s0, sh) & static_cast<uint32_t>(ml);
                            o1 |= __builtin_amdgcn_alignbyte(s2, s1, sh) & static_cast<uint32_t>(ml >> 32);
                            o2 |= __builtin_amdgcn_alignbyte(s3, s2, sh) & static_cast<uint32_t>(mh);
                            o3 |= __builtin_amdgcn_alignbyte(s4, s3, sh) & static_cast<uint32_t>(mh >> 32);
                        }
                        if (static_cast<int32_t>(nxt.x) >= a0 + 16 || r + 1 >= m) break;
                        r++;
                        cur = nxt;
                        nxt = S.ri[r + 1];
                    }
                    const uint32_t ow[4] = {o0, o1, o2, o3};
                    const int64_t blk = (B0 + b) << 4;
                    if (blk >= G0 && blk + 16 <= G1) {
                        *reinterpret_cast<uint4*>(a.chars + blk) = make_uint4(ow[0], ow[1], ow[2], ow[3]);
                    } else {
                        const int64_t gs = max(blk, G0), ge = min(blk + 16, G1);
                        for (int64_t x = gs; x < ge; x++) {
                            const uint32_t at = static_cast<uint32_t>(x - blk);
                            a.chars[x] = static_cast<uint8_t>(ow[at >> 2] >> (8 * (at & 3)));
                        }
                    }
                }
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            }
        }
    }
}

}  // namespace

PipePlan plan_pipe_lds(uint32_t dict_bytes) {
    PipePlan pl{};
    pl.lds = dict_bytes + kWriteWaves * static_cast<uint32_t>(sizeof(WriteLds));
    pl.blocks_per_cu = pl.lds <= 160u * 1024 ? static_cast<int>((160u * 1024) / pl.lds) : 0;
    if (pl.blocks_per_cu > 4) pl.blocks_per_cu = 4;
    return pl;
}

void launch_pipe_runs(hipStream_t s, const uint8_t* bytes, const DevPage* pages, int npages, int32_t max_def,
                      int32_t max_rep, uint2* runs, uint32_t* info) {
    if (npages <= 0) return;
    const int per = kRunWaves * kRunPages;
    hipLaunchKernelGGL(k_pipe_runs, dim3((npages + per - 1) / per), dim3(kRunWaves * kWave), 0, s, bytes, pages,
                       npages, max_def, max_rep, runs, info);
}

void launch_pipe_codes(hipStream_t s, const PipeLaunch& P, bool count_pass) {
    if (P.ntiles <= 0) return;
    CodeArgs a{P.bytes, P.pages, P.tiles, P.ntiles, P.page_tile0, P.max_def, P.max_rep, P.dicts, P.dict_id,
               P.entries, P.dict_count, P.runs, P.info, P.tile_nn, P.codes, P.tile_chars, P.page_err, P.err_any};
    const dim3 grid((P.ntiles + kCodeWaves - 1) / kCodeWaves);
    if (count_pass) hipLaunchKernelGGL(k_pipe_codes<true>, grid, dim3(kCodeWaves * kWave), 0, s, a);
    else hipLaunchKernelGGL(k_pipe_codes<false>, grid, dim3(kCodeWaves * kWave), 0, s, a);
}

void launch_pipe_write(hipStream_t s, const PipeLaunch& P) {
    if (P.ntiles <= 0) return;
    static uint32_t attr = 0;
    if (P.lds > attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_pipe_write),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(P.lds));
        attr = P.lds;
    }
    WriteArgs a{P.bytes, P.pages, P.tiles, P.ntiles, P.dicts, P.dict_id, P.entries, P.dict_count, P.codes,
                P.tile_base, P.nrows_total, P.total, P.capacity, P.overflow, P.validity, P.offsets, P.chars,
                P.dict_chars_bytes, P.dict_bytes, P.debug};
    const int need = (P.ntiles + kWriteWaves - 1) / kWriteWaves;
    const int grid = max(1, min(need, P.grid));
    hipLaunchKernelGGL(k_pipe_write, dim3(grid), dim3(kWriteWaves * kWave), P.lds, s, a);
}

}  // namespace pqk
