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
//                 offsets, validity words and the characters, each row copied
//                 from the LDS dictionary to HBM with unaligned 16-byte moves.
// Only pages of more than 512 rows with def levels need tile_nn, the
// non-null counts of the earlier tiles of their page (k_pipe_codes<true>).
#include <cstddef>
#include <type_traits>
#include "kernels/device_common.hpp"
#include "kernels/dict_index.hpp"
#include "kernels/kernels.hpp"
#include "kernels/lane_walk.hpp"
#include "kernels/run_walk.hpp"
#include "kernels/run_spec.hpp"
#include "kernels/stream.hpp"
#include "pq_gpu.h"

namespace pqk {
namespace {

using namespace dev;

constexpr int kRunWaves = 4;
constexpr int kRunPages = 32;                 // max pages per wavefront (2 streams each)
constexpr uint32_t kRunStage = 16384;         // staged payload bytes per wavefront
constexpr uint32_t kFallback = 1u << 31;      // info flag: exact serial decode
constexpr uint32_t kBig = 1u << 30;           // info flag: k_pipe_big wrote the page's codes
constexpr uint32_t kSkip = kFallback | kBig;  // k_pipe_codes3 leaves the page alone
constexpr int kCodeWaves = 4;
constexpr uint16_t kNull = 0xFFFFu;
constexpr int kWriteMax = 16;                // writer waves per k_pipe_write workgroup: runtime wpw <= this
constexpr uint32_t kFront = 16;               // zero bytes before the LDS dictionary
constexpr uint32_t kLitCapP = 16;

struct __attribute__((packed, aligned(1))) U16B { uint32_t x, y, z, w; };
struct __attribute__((packed, aligned(1))) U8B { uint32_t x, y; };
struct __attribute__((packed, aligned(1))) U4B { uint32_t x; };
struct __attribute__((packed, aligned(1))) U2B { uint16_t x; };

// Codes of rows 8l .. 8l + 7 (lane l) to codes[R0 + 8l ..]: one 16-byte
// store when all eight rows are in the tile, else one store per row.
__device__ __forceinline__ void store_codes8(uint16_t* codes, int64_t R0, uint32_t l8, uint32_t m, const uint32_t c[8]) {
    if (l8 + 8 <= m) {
        *reinterpret_cast<U16B*>(codes + R0 + l8) =
            U16B{c[0] | (c[1] << 16), c[2] | (c[3] << 16), c[4] | (c[5] << 16), c[6] | (c[7] << 16)};
    } else {
#pragma unroll
        for (int k = 0; k < 8; k++)
            if (l8 + k < m) codes[R0 + l8 + k] = static_cast<uint16_t>(c[k]);
    }
}

// 32-bit codes (dictionaries of more than 65,535 entries or beyond the
// writer's LDS: k_pipe_big<true> -> k_pipe_wwide); 0xFFFFFFFF = NULL
constexpr uint32_t kNull32 = 0xFFFFFFFFu;
__device__ __forceinline__ void store_codes8w(uint32_t* codes, int64_t R0, uint32_t l8, uint32_t m, const uint32_t c[8]) {
    if (l8 + 8 <= m) {
        U16B* d = reinterpret_cast<U16B*>(codes + R0 + l8);
        d[0] = U16B{c[0], c[1], c[2], c[3]};
        d[1] = U16B{c[4], c[5], c[6], c[7]};
    } else {
#pragma unroll
        for (int k = 0; k < 8; k++)
            if (l8 + k < m) codes[R0 + l8 + k] = c[k];
    }
}

// run record: x = first value | count << 16, y = literal << 31 | payload
// (RLE value, or the page bit offset of the literal run's first value)
__device__ __forceinline__ uint32_t rr_start(uint2 r) { return r.x & 0xFFFFu; }
__device__ __forceinline__ uint32_t rr_lit(uint2 r) { return r.y >> 31; }
__device__ __forceinline__ uint32_t rr_pay(uint2 r) { return r.y & 0x7FFFFFFFu; }


// Dictionary pages decoded by k_pipe_runs' leading workgroups (ndicts = 0:
// none; the dictionary then decodes in its own k_dict_index launch).
struct RunDictArgs {
    const DevDict* dicts;
    int ndicts;
    uint64_t* entries;
    int32_t* dict_count;
    DevErr* dict_err;
    int32_t* err_any;
};

__global__ void __launch_bounds__(kRunWaves * 64) k_pipe_runs(const uint8_t* __restrict__ bytes,
                                                              const DevPage* __restrict__ pages, int npages,
                                                              int32_t max_def, int32_t max_rep,
                                                              uint2* __restrict__ runs,
                                                              uint32_t* __restrict__ info, int ppw,
                                                              int32_t* __restrict__ flist, uint32_t stage_max,
                                                              RunDictArgs d, int debug, uint32_t wstage) {
    // dynamic LDS: kRunWaves windows of wstage + 32 bytes each (wstage: the
    // group's pages fit when it is at least ppw page slots), or the leading
    // workgroups' dictionary page
    extern __shared__ __attribute__((aligned(16))) uint32_t stage_dyn[];
    const uint32_t wwords = wstage / 4 + 8;
    if (static_cast<int>(blockIdx.x) < d.ndicts) {
        // leading workgroups: the chunk's dictionary pages (dict_index.hpp),
        // the page staged over this workgroup's payload windows
        dict_index_block<kRunWaves>(bytes, d.dicts, static_cast<int>(blockIdx.x), d.entries, d.dict_count,
                                    d.dict_err, d.err_any, kRunWaves * wwords * 4, stage_dyn);
        return;
    }
    const uint32_t wv = threadIdx.x / kWave;
    const int g0 = ((static_cast<int>(blockIdx.x) - d.ndicts) * kRunWaves + static_cast<int>(wv)) * ppw;
    if (g0 >= npages) return;
    const int g1 = min(npages, g0 + ppw);
    uint32_t* stage = stage_dyn + wv * wwords;
    // one load of the group's page records (lane 2i, 2i + 1: page g0 + i;
    // lanes past the group re-read its last page): the window bounds and the
    // inside test come from it, and so does each lane's own page below
    const uint32_t gl = static_cast<uint32_t>(g1 - 1 - g0);
    const DevPage mine = pages[g0 + static_cast<int>(min(lane() >> 1, gl))];
    auto rl64 = [](uint64_t v, uint32_t i) -> uint64_t {
        return (static_cast<uint64_t>(__builtin_amdgcn_readlane(static_cast<uint32_t>(v >> 32), i)) << 32) |
               __builtin_amdgcn_readlane(static_cast<uint32_t>(v), i);
    };
    const uint64_t wlo = rl64(mine.off, 0);
    const uint64_t whi = rl64(mine.off, 2 * gl) +
                         static_cast<uint32_t>(max(static_cast<int32_t>(__builtin_amdgcn_readlane(
                                                       static_cast<uint32_t>(mine.size), 2 * gl)), 0));
    bool staged = whi >= wlo && whi - wlo <= wstage;
    if (staged) {  // every page of the group inside the window (image order)
        const bool inside = mine.off >= wlo && mine.off + static_cast<uint32_t>(max(mine.size, 0)) <= whi;
        staged = __ballot(!inside) == 0;
    }
    if (staged) {  // payload slots are 16-byte aligned with >= 16 zero bytes after each
        const uint4* src = reinterpret_cast<const uint4*>(bytes + wlo);
        uint4* dst = reinterpret_cast<uint4*>(stage);
        const uint32_t nb = static_cast<uint32_t>((whi - wlo + 15) / 16) + 1;
        copy_blocks(dst, src, nb, lane(), kWave);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (probe(debug, 1 << 26)) return;  // timing ablation: staging only (outputs invalid)

    const uint32_t s = lane() & 1;
    const int p = g0 + static_cast<int>(lane() >> 1);
    const bool act = p < g1 && static_cast<int>(lane() >> 1) < ppw && mine.nvals <= kPipeSmallRows;
    uint32_t flag = 0, nrec = 0, bwi = 0;
    RunWalk W{};
    if (act) {
        const DevPage pg = mine;
        const uint32_t size = static_cast<uint32_t>(max(pg.size, 0));
        const uint32_t n = static_cast<uint32_t>(max(pg.nvals, 0));
        const uint32_t sbase = static_cast<uint32_t>(pg.off - wlo);
        const uint8_t* gp = bytes + pg.off;
        auto rd = [&](uint32_t a) -> uint32_t {
            return staged ? static_cast<uint32_t>(lds_u64(stage, sbase + a)) : static_cast<uint32_t>(gld8(gp, a));
        };
        // prologue (column_reader.cpp:146-182); any error -> exact decoder
        uint32_t pos = 0, dbase = 0, dlen = 0;
        if (n > 65535u || size > stage_max) flag = 1;  // stage_max: k_pipe_codes3's payload stage
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
            W.alive = true;
            W.q = s ? pos : dbase;
            W.end = s ? size : dbase + dlen;
            W.bw = s ? bwi : level_bw(max_def);
            W.n = n;
            W.out = runs + (static_cast<size_t>(p) * 2 + s) * kPipeRunCap;
            W.cap = kPipeRunCap;
            W.sbase = sbase;
            W.gp = gp;
        }
    }
    // (the run table's per-stream rows are kPipeRunCap * 8 = 1 KiB apart:
    // 16-byte aligned, records stored in pairs)
    static_assert((kPipeRunCap * sizeof(uint2)) % 16 == 0, "record rows 16-byte aligned");
    if (staged && probe(debug, 1 << 24)) {  // timing probe: position-only walk of 1-byte headers (outputs invalid)
        uint32_t q = W.q, cnt = 0, nr = 0;
        bool alive = W.alive && W.n > 0;
        const uint32_t nbv = (W.bw + 7) / 8;
        const uint8_t* st8 = reinterpret_cast<const uint8_t*>(stage);
        while (__ballot(alive)) {
            const uint32_t b = st8[W.sbase + min(q, W.end)];
            const uint32_t lit = b & 1u, g = (b >> 1) & 0x3Fu;
            cnt += lit ? g * 8u : g;
            q += 1u + (lit ? g * W.bw : nbv);
            nr++;
            alive = alive && (b & 0x80u) == 0 && g != 0 && cnt < W.n && q < W.end && nr < W.cap;
        }
        if (nr == 0xFFFFFFu) info[0] = q;  // keeps the loop
        return;
    }
    if (staged) walk_runs<true, true>(W, stage, flag, nrec, probe(debug, 1 << 25));  // bit 25: no record stores (timing)
    else walk_runs<false, true>(W, stage, flag, nrec);
    const uint32_t oflag = static_cast<uint32_t>(__shfl_xor(static_cast<int>(flag), 1));
    const uint32_t orec = static_cast<uint32_t>(__shfl_xor(static_cast<int>(nrec), 1));
    if (act && s == 0)
        info[p] = ((flag | oflag) ? kFallback : 0u) | nrec | (orec << 8) | (bwi << 16);
    if (act && s == 0 && (flag | oflag)) flist[1 + atomicAdd(flist, 1)] = p;  // for k_pipe_codes3's exact decoder
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
    unsigned long long* bsum;  // characters per k_pipe_write workgroup (its tiles)
    int per;                   // tiles per k_pipe_write wavefront
    int debug;                 // 256: skip the exact decoder (timing only)
    int wpw;                   // k_pipe_write's writer waves per workgroup (bsum index)
    uint32_t* codes32 = nullptr;  // wide chunks: 32-bit codes here instead of `codes` (k_pipe_big<true>)
    const uint8_t* lens8 = nullptr;  // wide chunks: entry lengths as bytes (255: 255 or more), or null
};

// Characters of tile t also go to the k_pipe_write workgroup that writes it.
__device__ __forceinline__ void tile_done(const CodeArgs& a, int t, uint32_t chars) {
    if (lane() == 0) {
        a.tile_chars[t] = chars;
        if (chars && a.bsum) atomicAdd(&a.bsum[(t / a.per) / a.wpw], static_cast<unsigned long long>(chars));
    }
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) { return bcast_last(wave_incl_scan(v)); }

// Rows of a page the decode failed on: NULL codes, no characters.
__device__ void fail_page(const CodeArgs& a, const DevPage& pg, int32_t t0, uint32_t n) {
    for (uint32_t j = lane(); j < n; j += kWave) {
        if (a.codes32) a.codes32[pg.first_row + j] = kNull32;
        else a.codes[pg.first_row + j] = kNull;
    }
    for (uint32_t t = lane(); t * kTileRows < n; t += kWave) a.tile_chars[t0 + t] = 0;
}

// Exact decoder for a marked page: the reference state machine (stream.hpp)
// over the page in HBM, tile by tile; same error order as k_ba_fused.
// (always inlined: a call would pass the LDS scratch as a generic pointer and
// spill CodeArgs to scratch memory)
template <bool kWide = false>
__device__ __forceinline__ void exact_page_body(const CodeArgs& a, CodeLds& L, int p, uint32_t dict_n, uint32_t ebase) {
    using CodeT = typename std::conditional<kWide, uint32_t, uint16_t>::type;
    constexpr CodeT kNullT = kWide ? static_cast<CodeT>(kNull32) : static_cast<CodeT>(kNull);
    const DevPage pg = a.pages[p];
    const uint8_t* page = a.bytes + pg.off;
    const uint32_t size = static_cast<uint32_t>(max(pg.size, 0));
    const uint32_t n = static_cast<uint32_t>(max(pg.nvals, 0));
    const int32_t t0 = a.page_tile0[p];
    DevErr* err = a.page_err + p;
    uint8_t* lv = L.mark;
    // a tile's indices: u16 in recd; u32 over recd and reci (the literal
    // runs then go to mark2, unused here)
    static_assert(sizeof(L.recd) + sizeof(L.reci) >= kTileRows * 4 && sizeof(L.mark2) >= kLitCapP * sizeof(LitRun) &&
                      offsetof(CodeLds, reci) == sizeof(L.recd), "exact decoder scratch");
    CodeT* ix = reinterpret_cast<CodeT*>(L.recd);
    LitRun* lits = kWide ? reinterpret_cast<LitRun*>(L.mark2) : reinterpret_cast<LitRun*>(L.reci);
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
    // (kWide: the raw index; k_wide_chars and the writer test it against the
    // dictionary, which may still be decoding while this runs)
    auto put_ix = [&](uint32_t k, uint32_t v) {
        if constexpr (kWide) ix[k] = v;
        else ix[k] = static_cast<CodeT>(static_cast<int32_t>(v) >= 0 && v < dict_n ? v : static_cast<uint32_t>(kNullT));
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
            CodeT code = kNullT;
            if (nnul) {
                code = ix[k];
                if (!kWide && code != kNullT) chars += static_cast<uint32_t>(a.entries[ebase + code] >> 32);
            }
            if (j < m) {
                if (kWide) a.codes32[pg.first_row + r0 + j] = code;
                else a.codes[pg.first_row + r0 + j] = static_cast<uint16_t>(code);
            }
        }
        if (!kWide) {  // (kWide: k_wide_chars sums the tiles' characters)
            chars = wave_sum(chars);
            tile_done(a, t0 + static_cast<int>(ti), chars);
        }
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
    if (inf & kBig) return;
    if (inf & kFallback) {
        if (!kCount && T.row0 == 0) exact_page_body(a, L, p, dict_n, ebase);
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
    tile_done(a, t, chars);
}

__device__ __forceinline__ uint32_t wave_shr1(uint32_t v) {  // lane i <- lane i - 1, lane 0 <- 0
    return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x138, 0xf, 0xf, true));
}

// ── per-tile codes, lean form ──────────────────────────────────────────────
// k_pipe_codes3: per-tile codes with the dictionary's entry lengths in LDS,
// each wavefront's rows 8l .. 8l + 7 contiguous (one wave scan per quantity),
// and three properties that keep it lean:
//  * no global loads inside a tile.  On gfx9 loads and stores share vmcnt, so
//    a load in the tile waits for the previous tile's code stores; here the
//    tile's descriptors, run records, payload and earlier-tile non-null counts
//    all arrive in the prefetch, and a tile's stores are issued at the top of
//    the next tile, before that tile's prefetch (one wait per tile, for
//    operations issued a whole tile earlier);
//  * bit fields come from the staged payload without branches: two clamped
//    dword reads and a funnel shift (the slot's zero padding, capi.hip
//    `slot`, stands for the bytes past the page end);
//  * every row takes the same instructions (selects, not branches).
// Pages whose payload does not fit the stage (> kStage3 - 16 bytes), and every
// page when the dictionary has more entries than the LDS length table, take
// the exact decoder (exact_page).
constexpr int kCodeWaves3 = 4;                // 3 waves per SIMD fit its registers: 3 workgroups per CU
constexpr uint32_t kStage3 = 5120;            // staged payload bytes per tile (5 x 16 B per lane)
constexpr uint32_t kStage3Blocks = kStage3 / 16;
static_assert(kStage3Blocks == 5 * kWave, "prefetch registers");

struct CodeLds3 {  // leading fields as CodeLds (exact_page reuses them)
    uint2 recd[kPipeRunCap];
    uint2 reci[kPipeRunCap];
    uint8_t mark[kTileRows];
    uint8_t mark2[kTileRows];
    uint32_t stage[kStage3 / 4];
};
static_assert(sizeof(CodeLds3) >= sizeof(CodeLds) && offsetof(CodeLds3, mark2) == offsetof(CodeLds, mark2), "layout");

// bw-bit field (mask = 2^bw - 1, bw <= 16) at page bit b of the staged
// payload; word indices past `zw` (a zero word of the slot's padding) clamp.
__device__ __forceinline__ uint32_t sbits3(const uint32_t* st, uint32_t b, uint32_t zw, uint32_t mask) {
    const uint32_t wi = b >> 5;
    const uint32_t w0 = st[min(wi, zw)], w1 = st[min(wi + 1, zw)];
    return __builtin_amdgcn_alignbit(w1, w0, b & 31u) & mask;
}

// Codes of rows 8l .. 8l + 7 packed two per word.
__device__ __forceinline__ void store_packed8(uint16_t* codes, int64_t R0, uint32_t l8, uint32_t m, const uint32_t w[4]) {
    if (l8 + 8 <= m) {
        *reinterpret_cast<U16B*>(codes + R0 + l8) = U16B{w[0], w[1], w[2], w[3]};
    } else {
#pragma unroll
        for (int k = 0; k < 8; k++)
            if (l8 + k < m) codes[R0 + l8 + k] = static_cast<uint16_t>(w[k >> 1] >> (16 * (k & 1)));
    }
}

// (number of records among rec[lane], rec[lane + 64] with start <= v) - 1
__device__ __forceinline__ uint32_t run_at_reg(uint2 r0, uint2 r1, uint32_t nr, uint32_t v) {
    const bool a0 = lane() < nr && rr_start(r0) <= v;
    const bool a1 = lane() + kWave < nr && rr_start(r1) <= v;
    return static_cast<uint32_t>(__popcll(__ballot(a0)) + __popcll(__ballot(a1))) - 1u;
}

__global__ void __launch_bounds__(kCodeWaves3 * 64) k_pipe_codes3(CodeArgs a, uint32_t lt_n, const int32_t* __restrict__ flist) {
    extern __shared__ __attribute__((aligned(16))) uint16_t lens[];
    __shared__ CodeLds3 lds_all[kCodeWaves3];
    const int wv = static_cast<int>(threadIdx.x / kWave);
    CodeLds3& L = lds_all[wv];
    CodeLds& LX = *reinterpret_cast<CodeLds*>(&L);  // exact_page scratch (same leading fields)
    const uint32_t dict_n = static_cast<uint32_t>(a.dict_count[a.dict_id]);
    const uint32_t ebase = static_cast<uint32_t>(a.dicts[a.dict_id].entry_base);
    const uint32_t nl = min(dict_n, lt_n);
    const bool lean = dict_n <= lt_n;  // every entry length in LDS
    copy_map(lens, a.entries + ebase, nl, threadIdx.x, blockDim.x,
             [](uint64_t e) { return static_cast<uint16_t>(e >> 32); });
    __syncthreads();
    const uint32_t md = static_cast<uint32_t>(a.max_def), bwd = level_bw(a.max_def);
    const uint32_t maskd = (1u << bwd) - 1u;
    const int nw = static_cast<int>(gridDim.x) * kCodeWaves3;
    const int per = (a.ntiles + nw - 1) / nw;
    const int ta = min(a.ntiles, (static_cast<int>(blockIdx.x) * kCodeWaves3 + wv) * per);
    const int tb = min(a.ntiles, ta + per);
    const uint32_t l8 = lane() * 8;
    auto rl64 = [](uint64_t v, int i) -> uint64_t {
        const uint32_t lo = __builtin_amdgcn_readlane(static_cast<uint32_t>(v), i);
        const uint32_t hi = __builtin_amdgcn_readlane(static_cast<uint32_t>(v >> 32), i);
        return (static_cast<uint64_t>(hi) << 32) | lo;
    };
    // the previous tile's codes and characters, stored at the top of the next
    bool pend = false;
    int64_t pR0 = 0;
    uint32_t pm = 0, pch = 0;
    int pt = 0;
    uint32_t pw[4] = {0u, 0u, 0u, 0u};
    for (int c0 = ta; c0 < tb; c0 += kWave) {
        const int cn = min(kWave, tb - c0);
        uint32_t myp = 0, myrow0 = 0, mym = 0, myinf = kFallback, mysize = 0, mytp = 0;
        uint64_t myoff = 0, myfirst = 0;
        {  // (loads from clamped in-bounds indices, selected after: a load under a
           // lane condition compiles to a flat load from a select with a stack
           // address, and flat loads also count in lgkmcnt, so every LDS wait of
           // the tile would wait for the prefetch too)
            const bool in = static_cast<int>(lane()) < cn;
            const DevTile T = a.tiles[c0 + min(static_cast<int>(lane()), cn - 1)];
            const DevPage pg = a.pages[T.page];
            const uint32_t inf = a.info[T.page];
            const uint32_t tp = static_cast<uint32_t>(a.page_tile0[T.page]);
            myp = in ? static_cast<uint32_t>(T.page) : 0u;
            myrow0 = in ? static_cast<uint32_t>(T.row0) : 0u;
            mym = in ? static_cast<uint32_t>(T.nrows) : 0u;
            myinf = in ? inf : kFallback;
            mytp = in ? tp : 0u;
            mysize = in ? static_cast<uint32_t>(max(pg.size, 0)) : 0u;
            myoff = in ? pg.off : 0ull;
            myfirst = in ? static_cast<uint64_t>(pg.first_row) : 0ull;
        }
        uint2 rq0, rq1, rq2, rq3;
        uint4 sq0, sq1, sq2, sq3, sq4;
        uint32_t tnn = 0;
        auto prefetch = [&](int i) {
            const uint32_t inf = __builtin_amdgcn_readlane(myinf, i);
            const uint32_t pp = __builtin_amdgcn_readlane(myp, i);
            const uint32_t sz = __builtin_amdgcn_readlane(mysize, i);
            const uint32_t tp = __builtin_amdgcn_readlane(mytp, i);
            const uint64_t off = rl64(myoff, i);
            const bool skip = (inf & kSkip) || !lean;  // k_pipe_runs marks pages past the stage
            const uint32_t nd = skip ? 0u : (inf & 0xFFu), ni = skip ? 0u : ((inf >> 8) & 0xFFu);
            // every load from an in-bounds index (the page's 2 x kPipeRunCap
            // record block; blocks of its payload slot), selected after
            // (indices clamped to the page's record counts: lanes past them read
            // the last record's line again, not the block's unwritten slots, so
            // a page costs its records' lines, not 2 x kPipeRunCap x 8 bytes)
            const uint2* rd_ = a.runs + static_cast<size_t>(pp) * 2 * kPipeRunCap;
            const uint2 z = make_uint2(0u, 0u);
            const uint32_t nd1 = nd ? nd - 1 : 0u, ni1 = ni ? ni - 1 : 0u;
            const uint2 r0 = rd_[min(lane(), nd1)], r1 = rd_[min(lane() + kWave, nd1)];
            const uint2 r2 = rd_[kPipeRunCap + min(lane(), ni1)], r3 = rd_[kPipeRunCap + min(lane() + kWave, ni1)];
            rq0 = lane() < nd ? r0 : z;
            rq1 = lane() + kWave < nd ? r1 : z;
            rq2 = lane() < ni ? r2 : z;
            rq3 = lane() + kWave < ni ? r3 : z;
            const uint32_t nb = skip ? 0u : (sz + 15) / 16 + 1;
            const uint32_t nbl = nb ? nb - 1 : 0u;  // last block of the slot (block 0 always exists)
            const uint4* src = reinterpret_cast<const uint4*>(a.bytes + off);
            const uint4 z4 = make_uint4(0u, 0u, 0u, 0u);
            const uint4 b0 = src[min(lane(), nbl)], b1 = src[min(lane() + kWave, nbl)],
                        b2 = src[min(lane() + 2 * kWave, nbl)], b3 = src[min(lane() + 3 * kWave, nbl)],
                        b4 = src[min(lane() + 4 * kWave, nbl)];
            sq0 = lane() < nb ? b0 : z4;
            sq1 = lane() + kWave < nb ? b1 : z4;
            sq2 = lane() + 2 * kWave < nb ? b2 : z4;
            sq3 = lane() + 3 * kWave < nb ? b3 : z4;
            sq4 = lane() + 4 * kWave < nb ? b4 : z4;
            // non-null counts of the page's earlier tiles (pages of <= 2048 rows: <= 3)
            const uint32_t t = static_cast<uint32_t>(c0 + i);
            const uint32_t tn = static_cast<uint32_t>(a.tile_nn[min(tp + lane(), static_cast<uint32_t>(a.ntiles - 1))]);
            tnn = (md > 0 && !skip && tp + lane() < t) ? tn : 0u;
        };
        prefetch(0);
        for (int i = 0; i < cn; i++) {
            const int t = c0 + i;
            const uint32_t inf = __builtin_amdgcn_readlane(myinf, i);
            const int p = static_cast<int>(__builtin_amdgcn_readlane(myp, i));
            const uint32_t r0 = __builtin_amdgcn_readlane(myrow0, i), m = __builtin_amdgcn_readlane(mym, i);
            const uint32_t size = __builtin_amdgcn_readlane(mysize, i);
            const int64_t first_row = static_cast<int64_t>(rl64(myfirst, i));
            const bool skip = (inf & kSkip) || !lean;
            // this tile's records and payload -> LDS
            const uint2 d0 = rq0, d1 = rq1, x0 = rq2, x1 = rq3;
            const uint32_t k0n = tnn;
            L.recd[lane()] = rq0;
            L.recd[lane() + kWave] = rq1;
            L.reci[lane()] = rq2;
            L.reci[lane() + kWave] = rq3;
            uint4* st4 = reinterpret_cast<uint4*>(L.stage);
            st4[lane()] = sq0;
            st4[lane() + kWave] = sq1;
            st4[lane() + 2 * kWave] = sq2;
            st4[lane() + 3 * kWave] = sq3;
            st4[lane() + 4 * kWave] = sq4;
            // the previous tile's stores, then the next tile's loads
            if (pend) {
                store_packed8(a.codes, pR0, l8, pm, pw);
                tile_done(a, pt, pch);
                pend = false;
            }
            if (i + 1 < cn) prefetch(i + 1);
            if (skip) continue;  // marked pages: the exact decoder after the loop (flist)
            const uint32_t zw = ((size + 15) / 16 + 1) * 4 - 1;  // last word of the slot: zero
            const uint32_t nd = inf & 0xFFu, ni = (inf >> 8) & 0xFFu, bwi = (inf >> 16) & 0xFFu;
            const uint32_t maski = (1u << bwi) - 1u;
            *reinterpret_cast<uint2*>(L.mark + l8) = make_uint2(0u, 0u);
            *reinterpret_cast<uint2*>(L.mark2 + l8) = make_uint2(0u, 0u);
            // def levels of rows r0 + 8l .. r0 + 8l + 7
            uint32_t vb;
            if (md > 0) {
                const uint32_t rd0 = run_at_reg(d0, d1, nd, r0);
                __builtin_amdgcn_wave_barrier();
                {
                    const uint32_t k = lane(), st = rr_start(d0);
                    if (k < nd && k > rd0 && st < r0 + m) L.mark[st - r0] = static_cast<uint8_t>(k - rd0);
                    const uint32_t k1 = lane() + kWave, st1 = rr_start(d1);
                    if (k1 < nd && k1 > rd0 && st1 < r0 + m) L.mark[st1 - r0] = static_cast<uint8_t>(k1 - rd0);
                }
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                const uint2 mk = *reinterpret_cast<const uint2*>(L.mark + l8);
                uint32_t rm[8], run = 0;
#pragma unroll
                for (int k = 0; k < 8; k++) {
                    run = max(run, ((k < 4 ? mk.x : mk.y) >> (8 * (k & 3))) & 0xFFu);
                    rm[k] = run;
                }
                const uint32_t ex = wave_shr1(wave_incl_max(run));
                vb = 0;
                bool above = false;
#pragma unroll
                for (int k = 0; k < 8; k++) {
                    const uint32_t j = l8 + k;
                    const uint2 R = L.recd[(rd0 + max(ex, rm[k])) & (kPipeRunCap - 1)];
                    const uint32_t pay = rr_pay(R);
                    const uint32_t lb = sbits3(L.stage, pay + (r0 + j - rr_start(R)) * bwd, zw, maskd);
                    const uint32_t lvl = rr_lit(R) ? lb : pay;
                    const bool in = j < m;
                    vb |= (in && lvl == md ? 1u : 0u) << k;
                    above |= in && lvl > md;
                }
                if (__ballot(above)) {  // levels above max_def: outside the supported format
                    set_err(a.page_err + p, a.err_any, PQ_ERR_UNSUPPORTED, 0, 0, size);
                    for (uint32_t j = lane(); j < m; j += kWave) a.codes[first_row + r0 + j] = kNull;
                    if (lane() == 0) a.tile_chars[t] = 0;
                    __builtin_amdgcn_wave_barrier();
                    continue;
                }
            } else {
                vb = l8 >= m ? 0u : (m - l8 >= 8 ? 0xFFu : ((1u << (m - l8)) - 1u));
            }
            const uint32_t nnl = __popc(vb);
            const uint32_t nincl = wave_incl_scan(nnl);
            const uint32_t rbase = nincl - nnl, nn = bcast_last(nincl);
            const uint32_t k0 = md > 0 ? wave_sum(k0n) : r0;
            // dictionary index runs over ranks [k0, k0 + nn): run of each rank -> mark2
            const uint32_t ri0 = run_at_reg(x0, x1, ni, k0);
            if (nn) {
                __builtin_amdgcn_wave_barrier();
                {
                    const uint32_t k = lane(), st = rr_start(x0);
                    if (k < ni && k > ri0 && st < k0 + nn) L.mark2[st - k0] = static_cast<uint8_t>(k - ri0);
                    const uint32_t k1 = lane() + kWave, st1 = rr_start(x1);
                    if (k1 < ni && k1 > ri0 && st1 < k0 + nn) L.mark2[st1 - k0] = static_cast<uint8_t>(k1 - ri0);
                }
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                const uint2 mk = *reinterpret_cast<const uint2*>(L.mark2 + l8);
                uint32_t rm[8], run = 0;
#pragma unroll
                for (int k = 0; k < 8; k++) {
                    run = max(run, ((k < 4 ? mk.x : mk.y) >> (8 * (k & 3))) & 0xFFu);
                    rm[k] = run;
                }
                const uint32_t ex = wave_shr1(wave_incl_max(run));
                uint32_t w0 = 0, w1 = 0;
#pragma unroll
                for (int k = 0; k < 8; k++) {
                    const uint32_t v = max(ex, rm[k]);
                    if (k < 4) w0 |= v << (8 * k);
                    else w1 |= v << (8 * (k - 4));
                }
                __builtin_amdgcn_wave_barrier();
                *reinterpret_cast<uint2*>(L.mark2 + l8) = make_uint2(w0, w1);
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
            uint32_t chars = 0;
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const uint32_t rk = min(rbase + __popc(vb & ((1u << k) - 1u)), static_cast<uint32_t>(kTileRows - 1));
                const uint2 R = L.reci[(ri0 + L.mark2[rk]) & (kPipeRunCap - 1)];
                const uint32_t pay = rr_pay(R);
                const uint32_t lb = sbits3(L.stage, pay + (k0 + rk - rr_start(R)) * bwi, zw, maski);
                const uint32_t v = rr_lit(R) ? lb : pay;
                const bool ok = ((vb >> k) & 1u) && v < dict_n;
                const uint32_t len = lens[ok ? v : 0u];
                chars += ok ? len : 0u;
                const uint32_t code = ok ? v : static_cast<uint32_t>(kNull);
                if (k & 1) pw[k >> 1] |= code << 16;
                else pw[k >> 1] = code;
            }
            pch = wave_sum(chars);
            pend = true;
            pR0 = first_row + r0;
            pm = m;
            pt = t;
        }
    }
    if (pend) {
        store_packed8(a.codes, pR0, l8, pm, pw);
        tile_done(a, pt, pch);
    }
    // pages k_pipe_runs / k_pipe_big marked (complete before this launch):
    // the exact serial decoder, one wave per page
    const int nf = flist[0];
    for (int i = static_cast<int>(blockIdx.x) * kCodeWaves3 + wv; i < nf; i += nw) {
        exact_page_body(a, LX, flist[1 + i], dict_n, ebase);
        __builtin_amdgcn_wave_barrier();
    }
    // a dictionary longer than the length table (not planned: lt_n covers
    // every entry the page can hold): every unmarked page exactly
    if (!lean) {
        for (int t = ta; t < tb; t++) {
            const DevTile T = a.tiles[t];
            if (T.row0 == 0 && !(a.info[T.page] & kSkip)) exact_page_body(a, LX, T.page, dict_n, ebase);
            __builtin_amdgcn_wave_barrier();
        }
    }
}

// ── offsets, validity, characters ──────────────────────────────────────────
constexpr int kRowsPerLane = kTileRows / kWave;

constexpr int kWBatch = 4;          // tiles whose codes k_pipe_write loads at once
constexpr uint32_t kLongRow = 128;  // longer rows are copied by the whole wave

struct __attribute__((aligned(16))) WriteLds {  // 16-byte aligned: each lane stores its rows as b128
    uint32_t off[kTileRows + 4];  // tile-relative first byte per row (+ the end at [m])
    uint16_t src[kTileRows];      // dictionary byte per row
    uint8_t vb[kWave];            // validity bits of rows 8l .. 8l + 7
};
static_assert(sizeof(WriteLds) % 16 == 0, "per-wave scratch alignment");


__device__ __forceinline__ uint32_t dword_of(const uint4& v, uint32_t i) {  // register select, no scratch
    return i == 0 ? v.x : (i == 1 ? v.y : (i == 2 ? v.z : v.w));
}
// Bytes [x, y) (0 <= x < y <= 16) of the 16-byte aligned output block at
// `blk`, as naturally aligned 8/4/2/1-byte stores.
__device__ __forceinline__ void store_part(uint8_t* chars, int64_t blk, const uint4& v, uint32_t x, uint32_t y) {
    if (x == 0 && y == 16) {
        *reinterpret_cast<uint4*>(chars + blk) = v;
        return;
    }
    while (x < y) {
        const uint32_t w = dword_of(v, x >> 2);
        if ((x & 7) == 0 && x + 8 <= y) {
            *reinterpret_cast<uint2*>(chars + blk + x) = make_uint2(w, dword_of(v, (x >> 2) + 1));
            x += 8;
        } else if ((x & 3) == 0 && x + 4 <= y) {
            *reinterpret_cast<uint32_t*>(chars + blk + x) = w;
            x += 4;
        } else if ((x & 1) == 0 && x + 2 <= y) {
            *reinterpret_cast<uint16_t*>(chars + blk + x) = static_cast<uint16_t>(w >> (8 * (x & 3)));
            x += 2;
        } else {
            chars[blk + x] = static_cast<uint8_t>(w >> (8 * (x & 3)));
            x += 1;
        }
    }
}
// 16 bytes at LDS byte address A of a dword array: dword-aligned reads and
// v_alignbyte (byte-unaligned ds_read_b128 is much slower).  Bytes before A
// may be read (A >= 1 .. 3 bytes past a 4-aligned start is fine); the caller
// keeps 20 readable bytes past A.  A may be below the row start when the
// caller masks (block pulls).
__device__ __forceinline__ uint4 lds16(const uint32_t* w, uint32_t A) {
    const uint32_t i = A >> 2, sh = A & 3u;
    const uint32_t w0 = w[i], w1 = w[i + 1], w2 = w[i + 2], w3 = w[i + 3], w4 = w[i + 4];
    return make_uint4(__builtin_amdgcn_alignbyte(w1, w0, sh), __builtin_amdgcn_alignbyte(w2, w1, sh),
                      __builtin_amdgcn_alignbyte(w3, w2, sh), __builtin_amdgcn_alignbyte(w4, w3, sh));
}


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
    const int64_t* tile_chars;
    const unsigned long long* bsum;
    int per;
    int64_t nrows_total;
    int64_t* total;
    int64_t capacity;
    int32_t* overflow;
    uint32_t* validity;
    int64_t* offsets;
    uint8_t* chars;
    uint32_t dict_chars_bytes, dict_bytes;
    int debug;  // ablation: 2 = no characters, 4 = no offsets/validity stores, 8 = prologue only
    int wpw;    // writer waves per workgroup
    uint32_t* znext;  // the next decode's flags/bsum/flist[0] block, cleared here (or null)
    uint32_t znext_words;
    // armed regex page filter (pq_decode_regex_async): the dictionary's match
    // bytes (k_regex_dict ran before), or null; pages with a satisfying row
    // get flag 0 (the flags were set to 1 by k_regex_dict)
    const uint8_t* match;
    int match_neg;
    uint8_t* page_flags;
    const uint32_t* codes32 = nullptr;  // wide chunks (k_pipe_wwide)
    const uint4* pad16 = nullptr;       // wide chunks: 16-byte entry slots (k_pipe_wwide<true>), or null
};


// One 512-row tile of k_pipe_write: rows 8l .. 8l + 7 of lane l hold the codes
// `cur` (0xFFFF: NULL; indices at or past dict_n: NULL); R0 is the tile's
// first output row, G0 its first output byte, m its rows.
template <bool kArmed>
__device__ __forceinline__ void write_tile(const WriteArgs& a, WriteLds& S, const uint32_t* dwa, const uint32_t* dtab,
                                           uint32_t dict_n, int64_t R0, int64_t G0, uint32_t m, uint32_t page,
                                           const uint32_t cur[kRowsPerLane]) {
    constexpr bool armed = kArmed;
    // this lane's rows 8l .. 8l + 7: lengths, dictionary offsets, validity
    uint32_t len[kRowsPerLane], src[kRowsPerLane], vb = 0, acc = 0, sat = 0;
#pragma unroll
    for (int k = 0; k < kRowsPerLane; k++) {
        const bool valid = cur[k] < dict_n;
        const uint32_t e = valid ? dtab[cur[k]] : 0u;
        len[k] = armed ? ((e >> 16) & 0x7FFFu) : (e >> 16);
        if (armed) sat |= e;
        src[k] = e & 0xFFFFu;
        vb |= (valid ? 1u : 0u) << k;
        acc += len[k];
    }
    if (armed && __ballot(sat >> 31) && lane() == 0)  // the page filter: a row whose entry satisfies it
        a.page_flags[page] = 0;
    const uint32_t incl = wave_incl_scan(acc);
    const uint32_t total = bcast_last(incl);
    {
        // the lane's eight rows as two 16-byte stores of offsets and one
        // of sources (row-per-element stores would hit each bank 8 and 4
        // times); rows past m get the tile end and are never read as rows
        static_assert(kRowsPerLane == 8, "row layout");
        uint32_t o[kRowsPerLane];
        o[0] = incl - acc;
#pragma unroll
        for (int k = 1; k < kRowsPerLane; k++) o[k] = o[k - 1] + len[k - 1];
        uint4* po = reinterpret_cast<uint4*>(&S.off[lane() * kRowsPerLane]);
        po[0] = make_uint4(o[0], o[1], o[2], o[3]);
        po[1] = make_uint4(o[4], o[5], o[6], o[7]);
        *reinterpret_cast<uint4*>(&S.src[lane() * kRowsPerLane]) =
            make_uint4(src[0] | (src[1] << 16), src[2] | (src[3] << 16), src[4] | (src[5] << 16),
                       src[6] | (src[7] << 16));
    }
    S.vb[lane()] = static_cast<uint8_t>(vb);
    if (lane() == 0) S.off[m] = total;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    if (!probe(a.debug, 4)) {
        // offsets: rows 2j', 2j' + 1 per lane as one 16-byte store when
        // the tile starts on an even row (coalesced), else row j = 64k + lane
        if ((R0 & 1) == 0) {
#pragma unroll
            for (int k = 0; k < kRowsPerLane / 2; k++) {
                const uint32_t j = k * 2 * kWave + 2 * lane();
                if (j + 1 < m) {
                    const uint2 o = *reinterpret_cast<const uint2*>(&S.off[j]);
                    const int64_t v0 = G0 + o.x, v1 = G0 + o.y;
                    *reinterpret_cast<uint4*>(a.offsets + R0 + j) =
                        make_uint4(static_cast<uint32_t>(v0), static_cast<uint32_t>(static_cast<uint64_t>(v0) >> 32),
                                   static_cast<uint32_t>(v1), static_cast<uint32_t>(static_cast<uint64_t>(v1) >> 32));
                } else if (j < m) {
                    a.offsets[R0 + j] = G0 + S.off[j];
                }
            }
        } else {
#pragma unroll
            for (int k = 0; k < kRowsPerLane; k++) {
                const uint32_t j = k * kWave + lane();
                if (j < m) a.offsets[R0 + j] = G0 + S.off[j];
            }
        }
        // validity words [R0 >> 5, (R0 + m - 1) >> 5]: tile word t = vb bytes 4t .. 4t + 3
        const int64_t gfirst = R0 >> 5, glast = (R0 + m - 1) >> 5;
        const uint32_t sh = static_cast<uint32_t>(R0 & 31);
        const int64_t g = gfirst + lane();
        if (g <= glast) {
            auto tw = [&](int t) -> uint32_t {
                return (t >= 0 && t < kWave / 4) ? reinterpret_cast<const uint32_t*>(S.vb)[t] : 0u;
            };
            const int t = static_cast<int>(lane());
            const uint32_t val = (tw(t) << sh) | (sh ? (tw(t - 1) >> (32 - sh)) : 0u);
            // the column's last word belongs to its last tile alone
            const bool whole = g * 32 >= R0 && (g * 32 + 32 <= R0 + m || R0 + m == a.nrows_total);
            if (whole) a.validity[g] = val;
            else if (val) atomicOr(&a.validity[g], val);
        }
    }
    if (R0 + m == a.nrows_total && lane() == 0) {
        a.offsets[a.nrows_total] = G0 + total;
        *a.total = G0 + total;
    }
    if (total == 0 || probe(a.debug, 2)) return;
    if (G0 + total > a.capacity) {  // output too small: the host grows it and re-runs
        if (lane() == 0) atomicOr(a.overflow, 1);
        return;
    }
    // characters, 64 consecutive rows per step: each lane copies its
    // row from the LDS dictionary to HBM as unaligned 16-byte moves
    // (the last one overlapping the row's earlier bytes), rows under
    // 16 bytes as two overlapping 8/4/2-byte moves, so no store leaves
    // its row and the L2 merges the partial lines.  Rows longer than
    // kLongRow are copied afterwards by the whole wave, 16-byte
    // aligned blocks across the lanes.  (Assembling aligned blocks in
    // LDS first costs more than it saves: byte-unaligned LDS accesses
    // are slow; scripts/probe/unaligned_store.hip)
    const int64_t G1 = G0 + total;
    if (probe(a.debug, 128)) {  // timing only: the tile's bytes as aligned 16-byte blocks of zeros
        const int64_t b0 = G0 & ~static_cast<int64_t>(15);
        for (int64_t blk = b0 + 16 * static_cast<int64_t>(lane()); blk < G1; blk += 16 * kWave) {
            const uint4 v = make_uint4(0u, 0u, 0u, 0u);
            if (blk >= G0 && blk + 16 <= G1) *reinterpret_cast<uint4*>(a.chars + blk) = v;
            else store_part(a.chars, blk, v, static_cast<uint32_t>(max(blk, G0) - blk),
                            static_cast<uint32_t>(min(blk + 16, G1) - blk));
        }
        return;
    }
    for (uint32_t g0 = 0; g0 < m; g0 += kWave) {
        const uint32_t r = g0 + lane();
        uint32_t s0 = 0, ln = 0, sa = 0;
        if (r < m) {
            s0 = S.off[r];
            ln = S.off[r + 1] - s0;
            sa = kFront + S.src[r];
        }
        const bool lng = ln > kLongRow;
        if (!lng && ln) {
            uint8_t* d = a.chars + G0 + s0;
            if (ln >= 16) {
                for (uint32_t x = 0; x + 16 < ln; x += 16) {
                    const uint4 v = lds16(dwa, sa + x);
                    *reinterpret_cast<U16B*>(d + x) = U16B{v.x, v.y, v.z, v.w};
                }
                const uint4 v = lds16(dwa, sa + ln - 16);
                *reinterpret_cast<U16B*>(d + ln - 16) = U16B{v.x, v.y, v.z, v.w};
            } else {
                const uint4 v = lds16(dwa, sa);           // bytes 0 .. 15 of the row's source
                const uint32_t t = ln >= 8 ? ln - 8 : (ln >= 4 ? ln - 4 : (ln >= 2 ? ln - 2 : 0u));
                const uint4 u = lds16(dwa, sa + t);       // bytes t .. t + 15
                if (ln >= 8) {
                    *reinterpret_cast<U8B*>(d) = U8B{v.x, v.y};
                    *reinterpret_cast<U8B*>(d + t) = U8B{u.x, u.y};
                } else if (ln >= 4) {
                    *reinterpret_cast<U4B*>(d) = U4B{v.x};
                    *reinterpret_cast<U4B*>(d + t) = U4B{u.x};
                } else if (ln >= 2) {
                    *reinterpret_cast<U2B*>(d) = U2B{static_cast<uint16_t>(v.x)};
                    *reinterpret_cast<U2B*>(d + t) = U2B{static_cast<uint16_t>(u.x)};
                } else {
                    d[0] = static_cast<uint8_t>(v.x);
                }
            }
        }
        uint64_t lm = __ballot(lng);
        while (lm) {  // long rows: the whole wave, aligned destination blocks
            const uint32_t l = static_cast<uint32_t>(__builtin_ctzll(lm));
            lm &= lm - 1;
            const int64_t A0 = G0 + __builtin_amdgcn_readlane(s0, l);
            const int64_t A1 = A0 + __builtin_amdgcn_readlane(ln, l);
            const uint32_t src0 = __builtin_amdgcn_readlane(sa, l);
            const int64_t b0 = A0 & ~static_cast<int64_t>(15);
            for (int64_t blk = b0 + 16 * static_cast<int64_t>(lane()); blk < A1; blk += 16 * kWave) {
                const uint4 v = lds16(dwa, static_cast<uint32_t>(src0 + (blk - A0)));
                store_part(a.chars, blk, v, static_cast<uint32_t>(max(blk, A0) - blk),
                           static_cast<uint32_t>(min(blk + 16, A1) - blk));
            }
        }
    }
    (void)G1;
}

template <bool kArmed>
__global__ void __launch_bounds__(kWriteMax * 64) k_pipe_write(WriteArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    if (a.znext)  // the other flags/bsum/flist block, for the next decode (unused by this one)
        for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < a.znext_words; i += gridDim.x * blockDim.x) a.znext[i] = 0;
    // [kFront zero bytes][dictionary payload][entry table][per-wave scratch]
    uint32_t* dwa = reinterpret_cast<uint32_t*>(smem);
    uint32_t* dw = reinterpret_cast<uint32_t*>(smem + kFront);
    uint32_t* dtab = reinterpret_cast<uint32_t*>(smem + kFront + a.dict_chars_bytes);
    const uint32_t wv = threadIdx.x / kWave;
    WriteLds& S = reinterpret_cast<WriteLds*>(smem + a.dict_bytes)[wv];
    const DevDict d = a.dicts[a.dict_id];
    const uint32_t dict_n = static_cast<uint32_t>(a.dict_count[a.dict_id]);
    constexpr bool armed = kArmed;
    // each wavefront owns a contiguous run of tiles (consecutive rows): the
    // descriptors of up to 64 tiles are loaded at once, one per lane, and the
    // next tile's codes are loaded before this tile's stores are issued
    const int per = a.per;
    __shared__ unsigned long long red[kWriteMax];
    auto wave_sum64 = [](unsigned long long v) {
        for (int d = 1; d < kWave; d <<= 1) {
            const uint32_t lo = static_cast<uint32_t>(__shfl_xor(static_cast<int>(v), d));
            const uint32_t hi = static_cast<uint32_t>(__shfl_xor(static_cast<int>(v >> 32), d));
            v += (static_cast<unsigned long long>(hi) << 32) | lo;
        }
        return v;
    };
    // first output byte of the range: the workgroups before this one (bsum,
    // summed by k_pipe_codes), then this workgroup's earlier tiles.  Both
    // sums load together with the dictionary (one wait, one barrier).
    unsigned long long acc = 0, in = 0;
    const int ta = min(a.ntiles, static_cast<int>(blockIdx.x * a.wpw + wv) * per);
    const int tb = min(a.ntiles, ta + per);
    {
        for (uint32_t b = threadIdx.x; b < blockIdx.x; b += blockDim.x) acc += a.bsum[b];
        const int tfirst = min(a.ntiles, static_cast<int>(blockIdx.x * a.wpw) * per);
        for (int q = tfirst + static_cast<int>(lane()); q < ta; q += kWave) in += static_cast<unsigned long long>(a.tile_chars[q]);
    }
    {
        const uint4* src = reinterpret_cast<const uint4*>(a.bytes + d.off);
        uint4* dst = reinterpret_cast<uint4*>(dw);
        copy_blocks(dst, src, a.dict_chars_bytes / 16, threadIdx.x, blockDim.x);
        if (armed) {
            // entry = pos | len << 16 | satisfies-the-predicate << 31 (the
            // host arms only dictionaries under 32 KiB: len < 2^15)
            const uint64_t* es = a.entries + d.entry_base;
            for (uint32_t k = threadIdx.x; k < dict_n; k += blockDim.x) {
                const uint64_t e = es[k];
                const uint32_t sat = (a.match[k] != 0) != (a.match_neg != 0) ? 1u : 0u;
                dtab[k] = static_cast<uint32_t>(e & 0xFFFFu) | (static_cast<uint32_t>(e >> 32) << 16) | (sat << 31);
            }
        } else {
            copy_map(dtab, a.entries + d.entry_base, dict_n, threadIdx.x, blockDim.x, [](uint64_t e) {
                return static_cast<uint32_t>(e & 0xFFFFu) | (static_cast<uint32_t>(e >> 32) << 16);
            });
        }
    }
    acc = wave_sum64(acc);
    if (lane() == 0) red[wv] = acc;
    in = wave_sum64(in);
    __syncthreads();
    int64_t Grun = static_cast<int64_t>(in);
    for (int w = 0; w < a.wpw; w++) Grun += static_cast<int64_t>(red[w]);
    if (probe(a.debug, 8)) return;
    uint4 cv0, cv1, cv2, cv3;
    bool cv_loaded = false;
    for (int c0 = ta; c0 < tb; c0 += kWave) {
        const int cn = min(kWave, tb - c0);
        int64_t myR0 = 0, myG0 = 0;
        uint32_t mym = 0;
        uint32_t myc = 0, myp = 0;
        if (static_cast<int>(lane()) < cn) {
            const DevTile T = a.tiles[c0 + lane()];
            myp = static_cast<uint32_t>(T.page);
            myR0 = a.pages[T.page].first_row + T.row0;
            mym = static_cast<uint32_t>(T.nrows);
            myc = static_cast<uint32_t>(a.tile_chars[c0 + lane()]);
        }
        {  // tile characters < 2^25 each: a 32-bit scan over <= 64 tiles
            const uint32_t inc = wave_incl_scan(myc);
            myG0 = Grun + static_cast<int64_t>(inc - myc);
            Grun += static_cast<int64_t>(bcast_last(inc));
        }
        auto rl64 = [](int64_t v, int i) -> int64_t {
            const uint32_t lo = __builtin_amdgcn_readlane(static_cast<uint32_t>(v), i);
            const uint32_t hi = __builtin_amdgcn_readlane(static_cast<uint32_t>(static_cast<uint64_t>(v) >> 32), i);
            return static_cast<int64_t>((static_cast<uint64_t>(hi) << 32) | lo);
        };
        // codes of kWBatch tiles at a time -> LDS: the only global loads of
        // the tile loop, so one wait (which also drains this wave's earlier
        // stores: loads and stores share vmcnt) per batch, not per tile
        const uint32_t l8 = lane() * kRowsPerLane;
        for (int ib = 0; ib < cn; ib += kWBatch) {
            // four named registers (an indexed array would go to scratch)
            static_assert(kWBatch == 4, "batch registers");
            auto ld = [&](int i) -> uint4 {
                uint4 v = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
                if (i < cn) {
                    const int64_t R = rl64(myR0, i);
                    const uint32_t mm = __builtin_amdgcn_readlane(mym, i);
                    if (l8 < mm) {
                        const U16B x = *reinterpret_cast<const U16B*>(a.codes + R + l8);
                        v = make_uint4(x.x, x.y, x.z, x.w);
                    }
                }
                return v;
            };
            if (!probe(a.debug, 1 << 23) || !cv_loaded) {  // bit 23 (timing only): the first batch's codes reused
                cv0 = ld(ib); cv1 = ld(ib + 1); cv2 = ld(ib + 2); cv3 = ld(ib + 3);
                cv_loaded = true;
            }
        for (int i = ib; i < min(cn, ib + kWBatch); i++) {
            const int64_t R0 = rl64(myR0, i);
            const int64_t G0 = rl64(myG0, i);
            const uint32_t m = __builtin_amdgcn_readlane(mym, i);
            uint32_t cur[kRowsPerLane];
            {
                const int u = i - ib;  // register select (no dynamic indexing into cv)
                const uint4 w = u == 0 ? cv0 : (u == 1 ? cv1 : (u == 2 ? cv2 : cv3));
                const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
                for (int k = 0; k < kRowsPerLane; k++)
                    cur[k] = l8 + k < m ? (ww[k >> 1] >> (16 * (k & 1))) & 0xFFFFu : kNull;
            }
            write_tile<kArmed>(a, S, dwa, dtab, dict_n, R0, G0, m, __builtin_amdgcn_readlane(myp, i), cur);
        }
        }
    }
}


// ── the writer for wide dictionaries (k_pipe_wwide) ────────────────────────
// Dictionaries the writer's LDS cannot hold, or of more than 65,535 entries
// (pyarrow's 1 MiB dictionary pages): k_pipe_write's structure (persistent
// workgroups, a contiguous tile range per wave, first output bytes from the
// per-workgroup character sums k_pipe_big filed) over 32-bit codes, with the
// entry words (len << 32 | payload position) and the characters read from
// HBM, where a dictionary of a few MB stays in L2 across the decode.
struct __attribute__((aligned(16))) WideLds {
    uint32_t off[kTileRows + 4];  // tile-relative first byte per row (+ the end at [m])
    uint32_t src[kTileRows];      // dictionary payload byte per row
    uint8_t vb[kWave];            // validity bits of rows 8l .. 8l + 7
};
static_assert(sizeof(WideLds) % 16 == 0, "per-wave scratch alignment");
constexpr int kWideBatch = 2;  // tiles whose codes a wave loads at once (8 u32 per lane each)
// kPad: the dictionary's 16-byte entry slots (launch_dict_big's pad16): one
// load per row gives the length and up to 15 characters, kept per row in LDS
// (after every wave's WideLds) until the row-per-lane character stores; rows
// of 16 or more bytes read the entry word and the payload as without
constexpr uint32_t kWideRowBytes = kTileRows * 16;
constexpr uint32_t kWidePadVb = (kTileRows + 4) * 4;                 // k_pipe_wwide<true> per wave: offsets,
constexpr uint32_t kWidePadRows = (kWidePadVb + kWave + 15) / 16 * 16;  // validity bytes, 16-byte row slots
constexpr uint32_t kWidePadWave = kWidePadRows + kWideRowBytes;

template <bool kPad>
__global__ void __launch_bounds__(kWriteMax * 64) k_pipe_wwide(WriteArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    if (a.znext)  // the other flags/bsum/flist block, for the next decode (unused by this one)
        for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < a.znext_words; i += gridDim.x * blockDim.x) a.znext[i] = 0;
    const uint32_t wv = threadIdx.x / kWave;
    // per wave: WideLds, or (kPad) the offsets, the validity bytes and the
    // rows' slots (a row of 16+ bytes keeps its payload position in its
    // slot's first word)
    uint8_t* wbase = smem + wv * (kPad ? kWidePadWave : static_cast<uint32_t>(sizeof(WideLds)));
    uint32_t* offp = reinterpret_cast<uint32_t*>(wbase);
    uint8_t* vbp = wbase + (kPad ? kWidePadVb : offsetof(WideLds, vb));
    uint32_t* srcp = reinterpret_cast<uint32_t*>(wbase + offsetof(WideLds, src));  // (not kPad)
    uint4* rows = reinterpret_cast<uint4*>(wbase + kWidePadRows);                   // (kPad)
    auto srcof = [&](uint32_t r) -> uint32_t { return kPad ? rows[r].x : srcp[r]; };
    const DevDict d = a.dicts[a.dict_id];
    const uint32_t dict_n = static_cast<uint32_t>(max(a.dict_count[a.dict_id], 0));
    const uint64_t* es = a.entries + d.entry_base;
    const uint8_t* dsrc = a.bytes + d.off;  // the dictionary payload slot (>= 16 zero bytes past its end)
    const int per = a.per;
    const int ta = min(a.ntiles, static_cast<int>(blockIdx.x * a.wpw + wv) * per);
    const int tb = min(a.ntiles, ta + per);
    __shared__ unsigned long long red[kWriteMax];
    auto wave_sum64 = [](unsigned long long v) {
        for (int dd = 1; dd < kWave; dd <<= 1) {
            const uint32_t lo = static_cast<uint32_t>(__shfl_xor(static_cast<int>(v), dd));
            const uint32_t hi = static_cast<uint32_t>(__shfl_xor(static_cast<int>(v >> 32), dd));
            v += (static_cast<unsigned long long>(hi) << 32) | lo;
        }
        return v;
    };
    unsigned long long acc = 0, in = 0;
    for (uint32_t b = threadIdx.x; b < blockIdx.x; b += blockDim.x) acc += a.bsum[b];
    {
        const int tfirst = min(a.ntiles, static_cast<int>(blockIdx.x * a.wpw) * per);
        for (int q = tfirst + static_cast<int>(lane()); q < ta; q += kWave) in += static_cast<unsigned long long>(a.tile_chars[q]);
    }
    acc = wave_sum64(acc);
    if (lane() == 0) red[wv] = acc;
    in = wave_sum64(in);
    __syncthreads();
    int64_t Grun = static_cast<int64_t>(in);
    for (int w = 0; w < a.wpw; w++) Grun += static_cast<int64_t>(red[w]);
    if (probe(a.debug, 8)) return;
    const uint32_t l8 = lane() * kRowsPerLane;
    auto rl64 = [](int64_t v, int i) -> int64_t {
        const uint32_t lo = __builtin_amdgcn_readlane(static_cast<uint32_t>(v), i);
        const uint32_t hi = __builtin_amdgcn_readlane(static_cast<uint32_t>(static_cast<uint64_t>(v) >> 32), i);
        return static_cast<int64_t>((static_cast<uint64_t>(hi) << 32) | lo);
    };
    for (int c0 = ta; c0 < tb; c0 += kWave) {
        const int cn = min(kWave, tb - c0);
        int64_t myR0 = 0, myG0 = 0;
        uint32_t mym = 0, myc = 0;
        if (static_cast<int>(lane()) < cn) {
            const DevTile T = a.tiles[c0 + lane()];
            myR0 = a.pages[T.page].first_row + T.row0;
            mym = static_cast<uint32_t>(T.nrows);
            myc = static_cast<uint32_t>(a.tile_chars[c0 + lane()]);
        }
        {
            const uint32_t inc = wave_incl_scan(myc);
            myG0 = Grun + static_cast<int64_t>(inc - myc);
            Grun += static_cast<int64_t>(bcast_last(inc));
        }
        for (int ib = 0; ib < cn; ib += kWideBatch) {
            static_assert(kWideBatch == 2, "batch registers");
            // kPad: row 64k + l of the tile in lane l, register k (a gather
            // instruction then reads 64 consecutive rows: rows of one RLE run
            // share a slot, so its lanes share cache lines); else rows
            // 8l .. 8l + 7 in lane l
            auto ld = [&](int i, uint4& lo, uint4& hi) {
                lo = hi = make_uint4(kNull32, kNull32, kNull32, kNull32);
                if (i < cn) {
                    const int64_t R = rl64(myR0, i);
                    const uint32_t mm = __builtin_amdgcn_readlane(mym, i);
                    if constexpr (kPad) {
                        uint32_t c[8];
#pragma unroll
                        for (int k = 0; k < 8; k++) {
                            const uint32_t r = k * kWave + lane();
                            c[k] = r < mm ? a.codes32[R + r] : kNull32;
                        }
                        lo = make_uint4(c[0], c[1], c[2], c[3]);
                        hi = make_uint4(c[4], c[5], c[6], c[7]);
                    } else if (l8 + 8 <= mm) {
                        const U16B* p = reinterpret_cast<const U16B*>(a.codes32 + R + l8);
                        const U16B x = p[0], y = p[1];
                        lo = make_uint4(x.x, x.y, x.z, x.w);
                        hi = make_uint4(y.x, y.y, y.z, y.w);
                    } else if (l8 < mm) {
                        uint32_t c[8];
#pragma unroll
                        for (int k = 0; k < 8; k++) c[k] = l8 + k < mm ? a.codes32[R + l8 + k] : kNull32;
                        lo = make_uint4(c[0], c[1], c[2], c[3]);
                        hi = make_uint4(c[4], c[5], c[6], c[7]);
                    }
                }
            };
            uint4 c0lo, c0hi, c1lo, c1hi;
            ld(ib, c0lo, c0hi);
            ld(ib + 1, c1lo, c1hi);
            for (int i = ib; i < min(cn, ib + kWideBatch); i++) {
                const int64_t R0 = rl64(myR0, i);
                const int64_t G0 = rl64(myG0, i);
                const uint32_t m = __builtin_amdgcn_readlane(mym, i);
                const bool first = i == ib;
                const uint4 lo = first ? c0lo : c1lo, hi = first ? c0hi : c1hi;
                const uint32_t cur[kRowsPerLane] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
                uint32_t len[kRowsPerLane], src[kRowsPerLane], total = 0;
                if constexpr (kPad) {
                    // rows 64k + l: entry slots (all eight loads in flight)
                    uint4 sl[kRowsPerLane];
#pragma unroll
                    for (int k = 0; k < kRowsPerLane; k++)
                        sl[k] = dict_n ? a.pad16[min(cur[k], dict_n - 1u)] : make_uint4(0u, 0u, 0u, 0u);
                    uint32_t far = 0;
                    uint32_t* vbw = reinterpret_cast<uint32_t*>(vbp);
#pragma unroll
                    for (int k = 0; k < kRowsPerLane; k++) {
                        const bool valid = cur[k] < dict_n;
                        len[k] = valid ? (sl[k].w >> 24) : 0u;
                        src[k] = 0;
                        far |= (len[k] == 0xFFu ? 1u : 0u) << k;
                        rows[k * kWave + lane()] = sl[k];
                        const uint64_t bm = __ballot(valid);  // validity words 2k, 2k + 1
                        if (lane() == 0) {
                            vbw[2 * k] = static_cast<uint32_t>(bm);
                            vbw[2 * k + 1] = static_cast<uint32_t>(bm >> 32);
                        }
                    }
                    if (__ballot(far != 0)) {  // rows of 16 or more bytes: the entry word
#pragma unroll
                        for (int k = 0; k < kRowsPerLane; k++)
                            if ((far >> k) & 1u) {
                                const uint64_t e = es[cur[k]];
                                len[k] = static_cast<uint32_t>(e >> 32);
                                rows[k * kWave + lane()].x = static_cast<uint32_t>(e);
                            }
                    }
                    // tile-relative first bytes: one wave scan per 64 rows
#pragma unroll
                    for (int k = 0; k < kRowsPerLane; k++) {
                        const uint32_t inc = wave_incl_scan(len[k]);
                        offp[k * kWave + lane()] = total + inc - len[k];
                        total += bcast_last(inc);
                    }
                } else {
                    uint32_t vb = 0, acc8 = 0;
                    // this lane's rows 8l .. 8l + 7: entry words (all eight loads in flight)
                    uint64_t e[kRowsPerLane];
#pragma unroll
                    for (int k = 0; k < kRowsPerLane; k++) e[k] = dict_n ? es[min(cur[k], dict_n - 1u)] : 0ull;
#pragma unroll
                    for (int k = 0; k < kRowsPerLane; k++) {
                        const bool valid = cur[k] < dict_n;
                        len[k] = valid ? static_cast<uint32_t>(e[k] >> 32) : 0u;
                        src[k] = valid ? static_cast<uint32_t>(e[k]) : 0u;
                        vb |= (valid ? 1u : 0u) << k;
                        acc8 += len[k];
                    }
                    const uint32_t incl = wave_incl_scan(acc8);
                    total = bcast_last(incl);
                    uint32_t o[kRowsPerLane];
                    o[0] = incl - acc8;
#pragma unroll
                    for (int k = 1; k < kRowsPerLane; k++) o[k] = o[k - 1] + len[k - 1];
                    uint4* po = reinterpret_cast<uint4*>(&offp[lane() * kRowsPerLane]);
                    po[0] = make_uint4(o[0], o[1], o[2], o[3]);
                    po[1] = make_uint4(o[4], o[5], o[6], o[7]);
                    uint4* ps = reinterpret_cast<uint4*>(&srcp[lane() * kRowsPerLane]);
                    ps[0] = make_uint4(src[0], src[1], src[2], src[3]);
                    ps[1] = make_uint4(src[4], src[5], src[6], src[7]);
                    vbp[lane()] = static_cast<uint8_t>(vb);
                }
                if (lane() == 0) offp[m] = total;
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                if (!probe(a.debug, 4)) {  // offsets and validity words as k_pipe_write stores them
                    if ((R0 & 1) == 0) {
#pragma unroll
                        for (int k = 0; k < kRowsPerLane / 2; k++) {
                            const uint32_t j = k * 2 * kWave + 2 * lane();
                            if (j + 1 < m) {
                                const uint2 o = *reinterpret_cast<const uint2*>(&offp[j]);
                                const int64_t v0 = G0 + o.x, v1 = G0 + o.y;
                                *reinterpret_cast<uint4*>(a.offsets + R0 + j) =
                                    make_uint4(static_cast<uint32_t>(v0), static_cast<uint32_t>(static_cast<uint64_t>(v0) >> 32),
                                               static_cast<uint32_t>(v1), static_cast<uint32_t>(static_cast<uint64_t>(v1) >> 32));
                            } else if (j < m) {
                                a.offsets[R0 + j] = G0 + offp[j];
                            }
                        }
                    } else {
#pragma unroll
                        for (int k = 0; k < kRowsPerLane; k++) {
                            const uint32_t j = k * kWave + lane();
                            if (j < m) a.offsets[R0 + j] = G0 + offp[j];
                        }
                    }
                    const int64_t gfirst = R0 >> 5, glast = (R0 + m - 1) >> 5;
                    const uint32_t sh = static_cast<uint32_t>(R0 & 31);
                    const int64_t g = gfirst + lane();
                    if (g <= glast) {
                        auto tw = [&](int t) -> uint32_t {
                            return (t >= 0 && t < kWave / 4) ? reinterpret_cast<const uint32_t*>(vbp)[t] : 0u;
                        };
                        const int t = static_cast<int>(lane());
                        const uint32_t val = (tw(t) << sh) | (sh ? (tw(t - 1) >> (32 - sh)) : 0u);
                        const bool whole = g * 32 >= R0 && (g * 32 + 32 <= R0 + m || R0 + m == a.nrows_total);
                        if (whole) a.validity[g] = val;
                        else if (val) atomicOr(&a.validity[g], val);
                    }
                }
                if (R0 + m == a.nrows_total && lane() == 0) {
                    a.offsets[a.nrows_total] = G0 + total;
                    *a.total = G0 + total;
                }
                if (total == 0 || probe(a.debug, 2)) continue;
                if (G0 + total > a.capacity) {
                    if (lane() == 0) atomicOr(a.overflow, 1);
                    continue;
                }
                // characters, 64 consecutive rows per group, row per lane.
                // Rows of <= 16 bytes: two 8-byte loads per row (bytes 0..7 and
                // ln-8..ln-1; the slot's zero padding covers reads past the
                // payload) for four groups before any of their stores, then
                // two overlapping 8/4/2-byte stores inside the row.
                for (uint32_t h = 0; h < m; h += 4 * kWave) {
                    uint32_t s0[4], ln[4];
                    U8B A[4], B[4];
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        const uint32_t r = h + q * kWave + lane();
                        s0[q] = 0;
                        ln[q] = 0;
                        uint32_t sa = 0;
                        if (r < m) {
                            s0[q] = offp[r];
                            ln[q] = offp[r + 1] - s0[q];
                            sa = srcof(r);
                        }
                        const uint32_t l16 = ln[q] <= 16 ? ln[q] : 0u;
                        if (kPad && ln[q] <= 15) {  // from the row's slot: bytes 0..7 and ln-8 .. ln-1
                            const uint4 x = rows[r < m ? r : 0u];
                            const uint64_t lo = (static_cast<uint64_t>(x.y) << 32) | x.x;
                            const uint64_t hi = (static_cast<uint64_t>(x.w) << 32) | x.z;
                            const uint32_t o = l16 >= 8 ? l16 - 8 : 0u;
                            const uint64_t b = o ? ((lo >> (8 * o)) | (hi << (64 - 8 * o))) : lo;
                            A[q] = U8B{x.x, x.y};
                            B[q] = U8B{static_cast<uint32_t>(b), static_cast<uint32_t>(b >> 32)};
                        } else {
                            A[q] = *reinterpret_cast<const U8B*>(dsrc + sa);
                            B[q] = *reinterpret_cast<const U8B*>(dsrc + sa + (l16 >= 8 ? l16 - 8 : 0u));
                        }
                    }
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        const uint32_t L = ln[q];
                        uint8_t* dd = a.chars + G0 + s0[q];
                        if (L >= 8 && L <= 16) {
                            *reinterpret_cast<U8B*>(dd) = A[q];
                            *reinterpret_cast<U8B*>(dd + L - 8) = B[q];
                        } else if (L >= 4 && L < 8) {
                            *reinterpret_cast<U4B*>(dd) = U4B{A[q].x};
                            *reinterpret_cast<U4B*>(dd + L - 4) = U4B{__builtin_amdgcn_alignbyte(A[q].y, A[q].x, L - 4)};
                        } else if (L >= 2 && L < 4) {
                            *reinterpret_cast<U2B*>(dd) = U2B{static_cast<uint16_t>(A[q].x)};
                            *reinterpret_cast<U2B*>(dd + L - 2) = U2B{static_cast<uint16_t>(A[q].x >> (8 * (L - 2)))};
                        } else if (L == 1) {
                            dd[0] = static_cast<uint8_t>(A[q].x);
                        }
                    }
                    // rows of 17 .. kLongRow bytes: the lane's own loop; longer rows: the wave
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        const uint32_t r = h + q * kWave + lane();
                        const uint32_t L = ln[q];
                        if (L > 16 && L <= kLongRow) {
                            const uint8_t* sp = dsrc + srcof(r);
                            uint8_t* dd = a.chars + G0 + s0[q];
                            for (uint32_t x = 0; x + 16 < L; x += 16)
                                *reinterpret_cast<U16B*>(dd + x) = *reinterpret_cast<const U16B*>(sp + x);
                            *reinterpret_cast<U16B*>(dd + L - 16) = *reinterpret_cast<const U16B*>(sp + L - 16);
                        }
                        uint64_t lm = __ballot(L > kLongRow);
                        while (lm) {
                            const uint32_t l = static_cast<uint32_t>(__builtin_ctzll(lm));
                            lm &= lm - 1;
                            const uint32_t rl = h + q * kWave + l;
                            const uint32_t LL = __builtin_amdgcn_readlane(L, l);
                            const uint8_t* sp = dsrc + srcof(rl);
                            uint8_t* dd = a.chars + G0 + __builtin_amdgcn_readlane(s0[q], l);
                            for (uint32_t x = 16 * lane(); x < LL; x += 16 * kWave) {
                                const uint32_t xx = min(x, LL - 16);  // the last block overlaps (same bytes)
                                *reinterpret_cast<U16B*>(dd + xx) = *reinterpret_cast<const U16B*>(sp + xx);
                            }
                        }
                    }
                }
            }
        }
    }
}


// ── pages of more than kPipeSmallRows rows (arrow layout) ──────────────────
// One workgroup per page, its payload staged in LDS.  A stream of ~1-2k runs
// is too long for the lane walk above, so its run headers are found by a
// speculative parse instead:
//   1. every byte position j of both streams is parsed as if a run header
//      started there (rle_decoder.hpp:36-50, 76-95): the next header's
//      position, or kBStop for a bad header or the end of the stream;
//   2. kBJumpLog pointer-doubling rounds turn that into kBJump-run jumps;
//   3. one lane per stream follows the jumps from the stream start, listing
//      every kBJump-th header of the real chain (~100 dependent LDS reads
//      instead of ~1500 header parses);
//   4. one lane per listed header re-parses its kBJump runs exactly into run
//      records with untruncated counts (the jump table's space is reused);
//   5. a scan of the listed headers' value counts gives every record its
//      first value; records past the page's value count are dropped, the one
//      crossing it is truncated and an exhausted stream gets its zero run
//      (rle_decoder.hpp:20-23): the records k_pipe_runs writes for a page;
//   6. the page's 512-row tiles: def levels (one wave per tile), a scan of
//      the tiles' non-null counts, then dictionary indices and codes as in
//      k_pipe_codes3, each tile's first record found by binary search.
// Anything outside the fast shape (a bad header before the value count,
// record overflow, levels above max_def) is decoded by the exact serial decoder
// (exact_page), by wave 0 of the page's workgroup.
constexpr int kBigWaves = 12;
constexpr int kBigThreads = kBigWaves * kWave;
constexpr uint32_t kBStop = 0xFFFFu;
constexpr int kBJumpLog = 4;
constexpr uint32_t kBJump = 1u << kBJumpLog;
constexpr uint32_t kBigPerThread = kBigSegBytes / kBigThreads;  // jump-table slots per thread (one segment)
constexpr uint32_t kBCountCap = 1u << 20;                       // count clamp (pages hold <= 32768 values)
static_assert(kBigSegBytes % kBigThreads == 0, "jump table split");
static_assert(kBigMaxBytes + 32 < kBStop, "u16 positions");
static_assert(kBigMaxBytes <= 2 * kBigSegBytes, "at most two jump-table segments");

struct BigLayout {  // dynamic LDS of k_pipe_big for a page of `size` payload bytes
    uint32_t P, H, nseg, LC, stage, tab, esum, ent, meta, lens, mark, tvb, misc, total;
};
__host__ __device__ inline BigLayout big_layout(uint32_t size, uint32_t nlens) {
    BigLayout L{};
    L.P = (size + 16 + 15) / 16 * 16;            // = the payload slot (capi.hip)
    // the jump table covers the page in one segment, or (pages over
    // kBigSegBytes) in two halves one after the other
    L.nseg = size > kBigOneSeg ? 2u : 1u;
    L.H = L.nseg == 1 ? L.P : ((size + 1) / 2 + 15) / 16 * 16;  // positions per segment (a multiple of 16)
    L.LC = L.P / (2 * kBJump) + 8;               // listed headers per stream (runs are >= 2 bytes)
    L.stage = 0;                                 // P bytes: the payload slot
    L.tab = L.stage + L.P;                       // u16 per position of a segment; then H / 4 run records
    L.esum = L.tab + 2 * L.H;                    // u32 per listed header: values, then their exclusive scan
    L.ent = L.esum + 8 * L.LC;                   // u32 per listed header: position
    // u32 per listed header: its re-parse's record count and flags, in place
    // of its position (step 4 reads every position of a pass of headers
    // before any of them is overwritten)
    L.meta = L.ent;
    L.tvb = L.esum;                              // per tile: validity bits of rows 8l .. 8l + 7 (phase 6:
                                                 // over esum / ent, dead after phase 5)
    const uint32_t xl = 16u * L.LC;
    const uint32_t x = xl > static_cast<uint32_t>(kBigTiles * kWave) ? xl : static_cast<uint32_t>(kBigTiles * kWave);
    L.lens = L.esum + x;                         // u16 per dictionary entry: length
    L.mark = L.lens + (2 * nlens + 15) / 16 * 16;  // per wave: u16 per row of a tile
    L.misc = L.mark + kBigWaves * kTileRows * 2;  // tile non-null counts, first ranks, scan partials, flags
    L.total = L.misc + 4 * (2 * kBigTiles + kBigWaves + 16);
    return L;
}

// A run header at LDS byte q of the staged page (the walk_runs parse).
struct BigHdr {
    uint32_t hl, g, lit, qh, vraw;
};
__device__ __forceinline__ BigHdr big_hdr(const uint32_t* stw, uint32_t q) {
    const uint64_t x = lds_u64(stw, q);
    const uint32_t x0 = static_cast<uint32_t>(x), x1 = static_cast<uint32_t>(x >> 32);
    const uint32_t st0 = ~x0 & 0x80808080u;
    BigHdr h;
    h.hl = st0 ? (__builtin_ctz(st0) >> 3) + 1 : ((~x1 & 0x80u) ? 5u : 9u);
    const uint32_t lm = (h.hl >= 4) ? 0xFFFFFFFFu : ((1u << (8 * (h.hl & 3))) - 1u);
    const uint32_t x0m = x0 & lm;
    const uint32_t top = (h.hl >= 5) ? (x1 << 28) : 0u;
    const uint32_t ind = (x0m & 0x7Fu) | ((x0m >> 1) & 0x3F80u) | ((x0m >> 2) & 0x1FC000u) |
                         ((x0m >> 3) & 0xFE00000u) | top;
    h.g = ind >> 1;
    h.lit = ind & 1u;
    h.qh = q + h.hl;
    const uint32_t va = __builtin_amdgcn_alignbyte(x1, x0, h.hl);
    const uint32_t vb = x1 >> (8 * ((h.hl - 4) & 3));
    h.vraw = (h.hl < 4) ? va : vb;
    return h;
}
// zero-count runs, headers past the stream, RLE values cut by its end
__device__ __forceinline__ bool big_bad(const BigHdr& h, uint32_t e, uint32_t nbv) {
    return h.hl > 5 || h.qh > e || h.g == 0 || (!h.lit && h.qh + nbv > e);
}

// Largest k < nr with start(rec[k]) <= v (rec[0] starts at 0, starts
// increase); wave-uniform, called by the whole wave.  Each round the 64 lanes
// test 64 evenly spaced records and keep the stride after the last one that
// starts <= v: two dependent LDS reads for up to 4096 records.
__device__ __forceinline__ uint32_t big_search(const uint2* rec, uint32_t nr, uint32_t v) {
    uint32_t lo = 0, span = nr;
    while (span > 1) {
        const uint32_t st = (span + kWave - 1) / kWave;
        const uint32_t d = lane() * st;
        const bool le = d < span && rr_start(rec[lo + min(d, span - 1)]) <= v;
        const uint64_t b = __ballot(le);  // bit 0 set: rec[lo] starts <= v
        const uint32_t j = 63u - static_cast<uint32_t>(__builtin_clzll(b | 1ull));
        lo += j * st;
        span = min(st, span - j * st);
    }
    return lo;
}

// x where c holds, else 0, as an and with an opaque mask: a select whose
// operand is a load would be turned into a branch around the load, which
// serialises the eight rows' LDS chains of a lane.
__device__ __forceinline__ uint32_t keep_if(bool c, uint32_t x) {
    uint32_t m = c ? 0xFFFFFFFFu : 0u;
    __asm__("" : "+v"(m));
    return x & m;
}

// Bits [b, b + bw) of the staged page, bw <= 16.  The stage holds the page
// and its slot's zero padding (nw words, >= 16 bytes past the page end), so
// bits past the end read as zero without a bound per word, like lds_bits;
// offsets past the padding (a literal run cut by the page end) read as zero.
__device__ __forceinline__ uint32_t big_bits(const uint32_t* stw, uint32_t nw, uint32_t b, uint32_t bw) {
    const uint32_t wi = b >> 5;
    const bool in = wi + 1 < nw;
    const uint32_t i0 = in ? wi : 0u;
    const uint32_t x = __builtin_amdgcn_alignbit(stw[i0 + 1], stw[i0], b & 31u);
    return keep_if(in, x & ((1u << bw) - 1u));
}

// Marks the starts of records k0 + 1 .. that begin inside [v0, v0 + m):
// mark[start - v0] = record - k0.
__device__ __forceinline__ void big_mark(uint16_t* mark, const uint2* rec, uint32_t nr, uint32_t k0, uint32_t v0,
                                         uint32_t m) {
    const uint32_t l8 = lane() * 8;
    if (l8 < m) *reinterpret_cast<uint4*>(mark + l8) = make_uint4(0u, 0u, 0u, 0u);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    for (uint32_t kb = k0 + 1;; kb += kWave) {
        const uint32_t k = kb + lane();
        const uint32_t st = k < nr ? rr_start(rec[k]) : 0xFFFFFFFFu;
        const bool in = k < nr && st < v0 + m;
        if (in) mark[st - v0] = static_cast<uint16_t>(k - k0);
        if (!__ballot(in)) break;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Per lane: the record (relative to k0) of values v0 + 8l .. v0 + 8l + 7.
__device__ __forceinline__ void big_runs8(const uint16_t* mark, uint32_t l8, uint32_t m, uint32_t rm[8]) {
    uint4 mk = make_uint4(0u, 0u, 0u, 0u);
    if (l8 < m) mk = *reinterpret_cast<const uint4*>(mark + l8);
    const uint32_t w[4] = {mk.x, mk.y, mk.z, mk.w};
    uint32_t run = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        run = max(run, (w[k >> 1] >> (16 * (k & 1))) & 0xFFFFu);
        rm[k] = run;
    }
    const uint32_t ex = wave_shr1(wave_incl_max(run));
#pragma unroll
    for (int k = 0; k < 8; k++) rm[k] = max(ex, rm[k]);
}

// Exclusive scan of v[0 .. m) in place (all threads of the workgroup);
// `part` holds kBigWaves words.
__device__ void big_scan(uint32_t* v, uint32_t m, uint32_t* part) {
    const uint32_t tid = threadIdx.x, wv = tid / kWave;
    const uint32_t per = (m + kBigThreads - 1) / kBigThreads;
    const uint32_t a0 = min(m, tid * per), a1 = min(m, a0 + per);
    uint32_t s = 0;
    for (uint32_t i = a0; i < a1; i++) s += v[i];
    const uint32_t inc = wave_incl_scan(s);
    if (lane() == kWave - 1) part[wv] = inc;
    __syncthreads();
    uint32_t base = inc - s;
    for (uint32_t w = 0; w < wv; w++) base += part[w];
    for (uint32_t i = a0; i < a1; i++) {
        const uint32_t x = v[i];
        v[i] = base;
        base += x;
    }
    __syncthreads();
}

// kWide: 32-bit codes (a.codes32) and index bit widths up to 24, entry
// lengths from the HBM entry table (dictionaries of more than 65,535 entries)
template <bool kWide>
__global__ void __launch_bounds__(kBigThreads) k_pipe_big(CodeArgs a, const int32_t* __restrict__ bigp,
                                                          uint32_t* __restrict__ info, uint32_t nlens,
                                                          uint32_t lds_cap) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int p = bigp[blockIdx.x];
    const DevPage pg = a.pages[p];
    const uint8_t* page = a.bytes + pg.off;
    const uint32_t size = static_cast<uint32_t>(max(pg.size, 0));
    const uint32_t n = static_cast<uint32_t>(max(pg.nvals, 0));
    const BigLayout Ly = big_layout(size, nlens);
    const uint32_t nw = Ly.P / 4;  // staged words: the page and its slot's zero padding
    uint32_t* stw = reinterpret_cast<uint32_t*>(smem + Ly.stage);
    uint16_t* tab = reinterpret_cast<uint16_t*>(smem + Ly.tab);
    uint32_t* esum = reinterpret_cast<uint32_t*>(smem + Ly.esum);
    uint32_t* ent = reinterpret_cast<uint32_t*>(smem + Ly.ent);
    uint16_t* lens = reinterpret_cast<uint16_t*>(smem + Ly.lens);
    uint8_t* tvb = smem + Ly.tvb;
    uint32_t* misc = reinterpret_cast<uint32_t*>(smem + Ly.misc);
    uint32_t* tnn = misc;                     // [kBigTiles]
    uint32_t* tk0 = misc + kBigTiles;         // [kBigTiles]
    uint32_t* part = misc + 2 * kBigTiles;    // [kBigWaves]
    uint32_t* sh = part + kBigWaves;          // [0] flag, [1] def list, [2] idx list, [3] def records, [4] idx records
    const uint32_t tid = threadIdx.x, wv = tid / kWave;
    const uint32_t md = static_cast<uint32_t>(a.max_def), bwd = level_bw(a.max_def);
    const uint32_t ntp = (n + kTileRows - 1) / kTileRows;
    const uint32_t dict_n = static_cast<uint32_t>(a.dict_count[a.dict_id]);
    const uint32_t ebase = static_cast<uint32_t>(a.dicts[a.dict_id].entry_base);
    const uint32_t nl = min(dict_n, nlens);

    // anything outside the fast shape: the exact serial decoder, by wave 0
    // of this workgroup (the page in HBM; LDS only for its small scratch),
    // so no further launch is needed after the big pages
    auto to_exact = [&](uint32_t why) {
        if (probe(a.debug, 1 << 27)) {  // diagnostics: which step sent the page to the exact decoder
            if (tid == 0) set_err(a.page_err + p, a.err_any, PQ_ERR_BUFFER, why, static_cast<uint32_t>(p), size);
            return;
        }
        if (tid == 0) info[p] = kFallback;
        if (wv == 0) exact_page_body<kWide>(a, *reinterpret_cast<CodeLds*>(smem), p, dict_n, ebase);
    };
    // (a layout past the launch's LDS never happens when the host sized it
    // with big_lds_max; kept as the guard against reading outside it)
    if (n > static_cast<uint32_t>(kBigTiles) * kTileRows || size > kBigMaxBytes || Ly.total > lds_cap) return to_exact(1);

    // 0. the payload slot and the dictionary's entry lengths -> LDS (before
    //    the prologue, which then reads the stage instead of HBM)
    copy_blocks(reinterpret_cast<uint4*>(stw), reinterpret_cast<const uint4*>(page), Ly.P / 16, tid, kBigThreads);
    copy_map(lens, a.entries + ebase, nl, tid, kBigThreads, [](uint64_t e) { return static_cast<uint16_t>(e >> 32); });
    if (tid < 8) sh[tid] = 0;
    __syncthreads();
    // prologue (column_reader.cpp:146-182), workgroup-uniform; any error -> exact_page
    auto rd32 = [&](uint32_t at) { return static_cast<uint32_t>(lds_u64(stw, at)); };
    bool flag = false;
    uint32_t pos = 0, dbase = 0, dlen = 0, bwi = 0;
    if (a.max_def > 0) {
        if (size < 4) flag = true;
        else {
            dlen = rd32(0);
            pos = 4;
            if (static_cast<uint64_t>(pos) + dlen > size) flag = true;
            else { dbase = 4; pos += dlen; }
        }
    }
    if (!flag && a.max_rep > 0) {
        if (pos + 4 > size) flag = true;
        else {
            const uint32_t rl = rd32(pos);
            pos += 4;
            if (static_cast<uint64_t>(pos) + rl > size) flag = true;
            else pos += rl;
        }
    }
    if (!flag) {
        if (pos + 1 > size) flag = true;
        else { bwi = rd32(pos) & 0xFFu; pos += 1; }
    }
    if (!flag && bwi > (kWide ? 24u : 16u)) flag = true;
    if (flag) {
        __syncthreads();  // every wave has read the stage before wave 0 reuses it
        return to_exact(2);
    }
    const bool hasd = a.max_def > 0;
    const uint32_t dend = dbase + dlen, ibase = pos, iend = size;
    if (probe(a.debug, 0x10000)) return;  // timing: staging only
    // 1. speculative headers at every byte, two bytes per thread and one
    //    dword store (bytes outside both streams get entries no chain reads:
    //    a next position is always inside its stream, else kBStop)
    auto next_at = [&](uint32_t j) -> uint32_t {
        const bool isi = j >= ibase;
        const uint32_t e = isi ? iend : dend, bw = isi ? bwi : bwd;
        const BigHdr h = big_hdr(stw, j);
        // g clamps at 2^16: a longer literal run leaves any stream (<= 24 KiB) either way
        const uint32_t nx = h.lit ? h.qh + __umul24(min(h.g, 0x10000u), bw) : h.qh + (bw + 7) / 8;
        return (j >= size || big_bad(h, e, (bw + 7) / 8) || nx >= e) ? kBStop : nx;
    };
    // (pages over kBigSegBytes: steps 1-3 per half of the page; a jump that
    // leaves the half stops at the first position past it, where step 3
    // goes on in the next half)
    const uint32_t rcap = Ly.H / 4;  // run records in the jump table's space
    const uint32_t rcap_d = hasd ? min(rcap / 2, dlen / 2 + 2 * kBJump + 2) : 0u;
    const uint32_t rcap_i = rcap - rcap_d;
    uint32_t* tab32 = reinterpret_cast<uint32_t*>(tab);
    const bool walker = tid == 0 || tid == kWave, isd_w = tid == 0;
    uint32_t wq = isd_w ? dbase : ibase, wk = 0;  // step 3's chain position and list length (walker threads)
    bool wdone = !walker || (isd_w && !hasd);
    // one body for both shapes; the one-segment instance (kOne) compiles
    // the round-3 loops exactly (no segment offsets or bounds)
    auto segment = [&](uint32_t sg, auto one_t) -> bool {
        constexpr bool kOne = decltype(one_t)::value;
        const uint32_t base = kOne ? 0u : sg * Ly.H, lim = kOne ? size : min(size, base + Ly.H);
        const uint32_t npair = (lim - base + 1) / 2;
        for (uint32_t jp = tid; jp < npair; jp += kBigThreads)
            tab32[jp] = next_at(base + 2 * jp) | (next_at(base + 2 * jp + 1) << 16);
        __syncthreads();
        if (probe(a.debug, 0x20000)) return false;  // timing: + header parse
        // 2. kBJump-run jumps by pointer doubling, two positions per thread
        //    (one dword of the table read and written)
        {
            auto hop = [&](uint32_t t) {  // kBStop and positions past the segment stay
                if constexpr (kOne) {
                    const uint32_t u = tab[t == kBStop ? 0u : t];
                    return t == kBStop ? kBStop : u;
                } else {
                    const bool in = t >= base && t < lim;
                    const uint32_t u = tab[in ? t - base : 0u];
                    return in ? u : t;
                }
            };
            for (int r = 0; r < kBJumpLog; r++) {
                uint32_t nv[kBigPerThread / 2];
#pragma unroll
                for (uint32_t i = 0; i < kBigPerThread / 2; i++) {
                    if (i * kBigThreads >= npair) break;  // (uniform)
                    const uint32_t jp = tid + i * kBigThreads;
                    uint32_t w = kBStop | (kBStop << 16);
                    if (jp < npair) {
                        const uint32_t x = tab32[jp];
                        w = hop(x & 0xFFFFu) | (hop(x >> 16) << 16);
                    }
                    nv[i] = w;
                }
                __syncthreads();
#pragma unroll
                for (uint32_t i = 0; i < kBigPerThread / 2; i++) {
                    if (i * kBigThreads >= npair) break;
                    const uint32_t jp = tid + i * kBigThreads;
                    if (jp < npair) tab32[jp] = nv[i];
                }
                __syncthreads();
            }
        }
        if (probe(a.debug, 4096)) return false;  // timing: jump table only
        // 3. one lane per stream follows the jumps: every kBJump-th header
        //    (and the first header past a segment end)
        if (walker && !wdone) {
            const uint32_t e = isd_w ? dend : iend, rc = isd_w ? rcap_d : rcap_i;
            const uint32_t lcap = rc > kBJump + 1 ? min(Ly.LC, (rc - kBJump - 1) / kBJump + 1) : 0u;
            uint32_t* L = ent + (isd_w ? 0u : Ly.LC);
            for (;;) {
                if (!kOne && wq < e && wq >= lim) break;  // listed by the next segment
                if (wk >= lcap) { wk = ~0u; wdone = true; break; }
                L[wk++] = wq;
                if (wq >= e) { wdone = true; break; }
                const uint32_t t = tab[wq - base];
                if (t == kBStop) { wdone = true; break; }
                wq = t;
            }
        }
        if (!kOne) __syncthreads();  // the next segment rewrites the table
        return true;
    };
    if (Ly.nseg == 1) {
        if (!segment(0u, std::true_type{})) return;
    } else {
        for (uint32_t sg = 0; sg < Ly.nseg; sg++)
            if (!segment(sg, std::false_type{})) return;
    }
    if (walker) sh[isd_w ? 1 : 2] = wk;
    __syncthreads();
    const uint32_t nld = sh[1], nli = sh[2];
    if (probe(a.debug, 8192)) return;  // timing: + chain walk
    if (nld == ~0u || nli == ~0u) return to_exact(3);
    // 4. exact runs of each listed header: untruncated counts, bad-header step
    uint2* recd = reinterpret_cast<uint2*>(smem + Ly.tab);
    uint2* reci = recd + rcap_d;
    const uint32_t ne = nld + nli;
    uint32_t* meta = reinterpret_cast<uint32_t*>(smem + Ly.meta);
    // (passes of kBigThreads headers: every position of a pass is read before
    // the barrier, its meta written over it after; the next pass's first
    // position, a stop of this one, is still unwritten)
    for (uint32_t i0 = 0; i0 < ne; i0 += kBigThreads) {
        const uint32_t i = i0 + tid;
        const bool isd = i < nld;
        const uint32_t li = isd ? i : i - nld;
        const uint32_t slot = isd ? i : Ly.LC + li;
        uint32_t q = i < ne ? ent[slot] : 0u;
        // the next listed header: kBJump runs on, or fewer where a jump
        // stopped at a segment end
        const uint32_t stop = i < ne && Ly.nseg > 1 && li + 1 < (isd ? nld : nli) ? ent[slot + 1] : 0xFFFFFFFFu;
        __syncthreads();
        if (i >= ne) continue;
        const uint32_t e = isd ? dend : iend, bw = isd ? bwd : bwi, nbv = (bw + 7) / 8;
        const uint32_t vmask = nbv >= 3 ? 0xFFFFFFu : (nbv == 2 ? 0xFFFFu : (nbv ? 0xFFu : 0u));
        const uint32_t litpay = bw ? 0x80000000u : 0u, litmul = bw ? 8u : 0u;
        uint2* out = (isd ? recd : reci) + li * kBJump;
        uint32_t s = 0, sum = 0, bad = kBJump, ended = 0;
        for (; s < kBJump; s++) {
            if (q >= e) { ended = 1; break; }
            if (q == stop) break;
            const BigHdr h = big_hdr(stw, q);
            if (big_bad(h, e, nbv)) { bad = s; break; }
            const uint32_t c = h.lit ? min(h.g, kBCountCap / 8) * 8 : min(h.g, kBCountCap);
            out[s] = make_uint2(c, h.lit ? (litpay | (h.qh * litmul)) : (h.vraw & vmask));
            sum = min(sum + c, kBCountCap);
            // (g clamps at 2^16: a longer literal run ends past the stream either way)
            const uint32_t nql = h.qh + __umul24(min(h.g, 0x10000u), bw);
            q = h.lit ? min(nql, e) : h.qh + nbv;
        }
        if (s == kBJump && q >= e) ended = 1;
        esum[i] = sum;
        meta[slot] = s | (bad << 8) | (ended << 16);
    }
    __syncthreads();
    // 5. first value of every record: scan of the headers' counts, then
    //    truncation at the page's value count and the exhaustion run
    big_scan(esum, ne, part);
    const uint32_t dtot = nld < ne ? esum[nld] : 0u;
    for (uint32_t i = tid; i < ne; i += kBigThreads) {
        const bool isd = i < nld;
        const uint32_t li = isd ? i : i - nld, nlst = isd ? nld : nli;
        const uint32_t mt = meta[isd ? i : Ly.LC + li];
        const uint32_t nr = mt & 0xFFu, bad = (mt >> 8) & 0xFFu, ended = mt >> 16;
        const uint32_t base = esum[i] - (isd ? 0u : dtot);
        if (base >= n) continue;
        uint2* out = (isd ? recd : reci) + li * kBJump;
        const uint32_t room = (isd ? rcap_d : rcap_i) - li * kBJump;
        uint32_t c0 = base, kept = 0;
        for (uint32_t s = 0; s < nr && c0 < n; s++) {
            const uint32_t c = out[s].x;
            out[s].x = c0 | (min(c, n - c0) << 16);
            c0 += c;
            kept = s + 1;
        }
        if (c0 >= n) {
            sh[isd ? 3 : 4] = li * kBJump + kept;
        } else if (bad < kBJump || (li + 1 == nlst && (!ended || nr >= room))) {
            atomicOr(&sh[0], 1u);  // a bad header before the value count (or a broken chain)
        } else if (li + 1 == nlst) {  // exhausted: the rest of the values are 0
            out[nr] = make_uint2(c0 | ((n - c0) << 16), 0u);
            sh[isd ? 3 : 4] = li * kBJump + nr + 1;
        } else if (nr < kBJump) {
            // a header list entry cut short at a segment end: its unused slots
            // repeat its last record (same start: every search and mark of
            // step 6 then finds a copy of that record, never a hole)
            if (nr == 0) atomicOr(&sh[0], 1u);  // (not produced by step 3; kept exact)
            else
                for (uint32_t s = nr; s < kBJump; s++) out[s] = out[nr - 1];
        }
    }
    __syncthreads();
    if (probe(a.debug, 16384)) return;  // timing: + exact records
    const uint32_t nd = hasd ? sh[3] : 0u, ni = sh[4];
    if (sh[0] || (hasd && nd == 0) || ni == 0) return to_exact(4 | (sh[0] << 4) | ((nd == 0) << 5) | ((ni == 0) << 6));
    const int32_t t0 = a.page_tile0[p];
    const int64_t first_row = pg.first_row;
    uint16_t* mark = reinterpret_cast<uint16_t*>(smem + Ly.mark) + wv * kTileRows;
    const uint32_t l8 = lane() * 8;

    // 6a. def levels per tile -> validity bits, non-null counts
    for (uint32_t ti = wv; ti < ntp; ti += kBigWaves) {
        const uint32_t r0 = ti * kTileRows, m = min(n - r0, static_cast<uint32_t>(kTileRows));
        uint32_t vb = 0;
        bool above = false;
        if (hasd) {
            const uint32_t rd0 = big_search(recd, nd, r0);
            big_mark(mark, recd, nd, rd0, r0, m);
            uint32_t rm[8];
            big_runs8(mark, l8, m, rm);
#pragma unroll
            for (int k = 0; k < 8; k++) {  // selects, not branches
                const uint32_t j = l8 + k;
                const uint2 R = recd[rd0 + rm[k]];
                const uint32_t lb = big_bits(stw, nw, rr_pay(R) + __umul24(r0 + j - rr_start(R), bwd), bwd);
                const uint32_t lvl = keep_if(rr_lit(R), lb) | keep_if(!rr_lit(R), rr_pay(R));
                vb |= (j < m && lvl == md ? 1u : 0u) << k;
                above |= j < m && lvl > md;
            }
        } else {
            vb = l8 >= m ? 0u : (m - l8 >= 8 ? 0xFFu : ((1u << (m - l8)) - 1u));
        }
        if (__ballot(above) && lane() == 0) atomicOr(&sh[0], 1u);  // levels above max_def: exact decoder
        tvb[ti * kWave + lane()] = static_cast<uint8_t>(vb);
        const uint32_t nn = bcast_last(wave_incl_scan(__popc(vb)));
        if (lane() == 0) tnn[ti] = nn;
        __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    if (probe(a.debug, 32768)) return;  // timing: + def levels
    if (sh[0]) return to_exact(8);
    if (wv == 0) {  // first rank of each tile (ntp <= 64)
        const uint32_t v = lane() < ntp ? tnn[lane()] : 0u;
        const uint32_t inc = wave_incl_scan(v);
        if (lane() < ntp) tk0[lane()] = inc - v;
    }
    if (tid == 0) info[p] = kBig;
    __syncthreads();
    // 6b. dictionary indices of each tile's ranks -> codes, tile characters
    for (uint32_t ti = wv; ti < ntp; ti += kBigWaves) {
        const uint32_t r0 = ti * kTileRows, m = min(n - r0, static_cast<uint32_t>(kTileRows));
        const uint32_t vb = tvb[ti * kWave + lane()];
        const uint32_t nnl = __popc(vb);
        const uint32_t rbase = wave_incl_scan(nnl) - nnl;
        const uint32_t nn = tnn[ti], k0 = tk0[ti];
        uint32_t ri0 = 0;
        if (nn) {
            uint32_t rm[8];
            ri0 = big_search(reci, ni, k0);
            big_mark(mark, reci, ni, ri0, k0, nn);
            big_runs8(mark, l8, nn, rm);
            __builtin_amdgcn_wave_barrier();
            if (l8 < nn) {  // record of every rank of the tile
                uint4 w;
                w.x = rm[0] | (rm[1] << 16);
                w.y = rm[2] | (rm[3] << 16);
                w.z = rm[4] | (rm[5] << 16);
                w.w = rm[6] | (rm[7] << 16);
                *reinterpret_cast<uint4*>(mark + l8) = w;
            }
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        uint32_t chars = 0, cw8[8], far = 0;
        const int64_t R0 = first_row + r0;
#pragma unroll
        for (int k = 0; k < 8; k++) {  // selects, not branches (NULL rows read record ri0)
            const bool nz = (vb >> k) & 1u;
            const uint32_t rk = rbase + __popc(vb & ((1u << k) - 1u));
            const uint2 R = reci[ri0 + keep_if(nz, mark[nz ? rk : 0u])];
            const uint32_t lb = big_bits(stw, nw, rr_pay(R) + __umul24(k0 + rk - rr_start(R), bwi), bwi);
            const uint32_t v = keep_if(rr_lit(R), lb) | keep_if(!rr_lit(R), rr_pay(R));
            // kWide: the raw index of every non-NULL row (the dictionary may
            // still be decoding: k_wide_chars and the writer test it)
            const bool ok = kWide ? nz : (nz && v < dict_n);
            const uint32_t code = keep_if(ok, v) | keep_if(!ok, kWide ? kNull32 : kNull);
            if (!kWide) {
                const bool inl = ok && v < nl;
                chars += keep_if(inl, lens[inl ? v : 0u]);
                far |= (ok && !inl ? 1u : 0u) << k;
            }
            cw8[k] = code;
        }
        if (!kWide && __ballot(far != 0)) {  // entries past the LDS length table (dictionaries over kBigLens)
#pragma unroll
            for (int k = 0; k < 8; k++)
                if ((far >> k) & 1u) chars += static_cast<uint32_t>(a.entries[ebase + cw8[k]] >> 32);
        }
        if (kWide) {
            store_codes8w(a.codes32, R0, l8, m, cw8);
        } else {
            store_codes8(a.codes, R0, l8, m, cw8);
            chars = wave_sum(chars);
            tile_done(a, t0 + static_cast<int>(ti), chars);
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// Wide pipe: each tile's characters from its raw 32-bit codes, once the
// dictionary is decoded (k_pipe_big<true> ran beside that decode): one wave
// per tile, the entry words of a lane's eight rows loaded at once; codes at or
// past the dictionary's entry count are NULL rows (the writer skips them too).
constexpr int kWideCharWaves = 4;
__global__ void __launch_bounds__(kWideCharWaves * 64) k_wide_chars(CodeArgs a) {
    const int t = static_cast<int>(blockIdx.x) * kWideCharWaves + static_cast<int>(threadIdx.x / kWave);
    if (t >= a.ntiles) return;
    const DevTile T = a.tiles[t];
    const uint32_t m = static_cast<uint32_t>(T.nrows), l8 = lane() * 8;
    const int64_t R0 = a.pages[T.page].first_row + T.row0;
    const uint32_t dict_n = static_cast<uint32_t>(max(a.dict_count[a.dict_id], 0));
    const uint64_t* es = a.entries + a.dicts[a.dict_id].entry_base;
    uint32_t c[8];
#pragma unroll
    for (int k = 0; k < 8; k++) c[k] = kNull32;
    if (l8 + 8 <= m) {
        const U16B* p = reinterpret_cast<const U16B*>(a.codes32 + R0 + l8);
        const U16B x = p[0], y = p[1];
        c[0] = x.x; c[1] = x.y; c[2] = x.z; c[3] = x.w; c[4] = y.x; c[5] = y.y; c[6] = y.z; c[7] = y.w;
    } else {
#pragma unroll
        for (int k = 0; k < 8; k++)
            if (l8 + k < m) c[k] = a.codes32[R0 + l8 + k];
    }
    uint32_t chars = 0;
    if (dict_n) {
        uint64_t e[8];
#pragma unroll
        for (int k = 0; k < 8; k++) e[k] = es[min(c[k], dict_n - 1u)];
#pragma unroll
        for (int k = 0; k < 8; k++) chars += c[k] < dict_n ? static_cast<uint32_t>(e[k] >> 32) : 0u;
    }
    chars = wave_sum(chars);
    tile_done(a, t, chars);
}

// The same with the entry lengths as bytes in LDS (launch_dict_big's lens8,
// dictionaries up to kWideLensLds entries): persistent workgroups of
// kWideLWaves waves stage the table once, then each wave takes kWideLBatch
// consecutive tiles per step, all their codes loaded before the first
// lookup (row 64j + l of a tile in lane l: the lanes of an RLE run read one
// LDS byte).  A length byte of 255 (255 or more) is read from the entry table.
constexpr int kWideLWaves = 16;
constexpr int kWideLBatch = 4;
constexpr uint32_t kWideLensLds = 120 * 1024;
__global__ void __launch_bounds__(kWideLWaves * 64) k_wide_chars_lds(CodeArgs a, uint32_t cap) {
    extern __shared__ __attribute__((aligned(16))) uint8_t l8s[];
    const uint32_t dict_n = min(static_cast<uint32_t>(max(a.dict_count[a.dict_id], 0)), cap);
    copy_blocks(reinterpret_cast<uint4*>(l8s), reinterpret_cast<const uint4*>(a.lens8), (dict_n + 15) / 16,
                threadIdx.x, blockDim.x);
    __syncthreads();
    const uint64_t* es = a.entries + a.dicts[a.dict_id].entry_base;
    const int wv = static_cast<int>(threadIdx.x / kWave);
    for (int b = (static_cast<int>(blockIdx.x) * kWideLWaves + wv) * kWideLBatch; b < a.ntiles;
         b += static_cast<int>(gridDim.x) * kWideLWaves * kWideLBatch) {
        // the batch's tile descriptors (lane k: tile b + k), then their rows
        uint32_t td_m = 0;
        int64_t td_r = 0;
        if (lane() < static_cast<uint32_t>(kWideLBatch) && b + static_cast<int>(lane()) < a.ntiles) {
            const DevTile T = a.tiles[b + lane()];
            td_m = static_cast<uint32_t>(T.nrows);
            td_r = a.pages[T.page].first_row + T.row0;
        }
        uint32_t c[kWideLBatch][8];
#pragma unroll
        for (int k = 0; k < kWideLBatch; k++) {
            const uint32_t m = __shfl(td_m, k);
            const int64_t R0 = __shfl(td_r, k);
            // row 64j + l in lane l (lanes of one RLE run then read one LDS byte)
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const uint32_t r = j * kWave + lane();
                c[k][j] = r < m ? a.codes32[R0 + r] : kNull32;
            }
        }
#pragma unroll
        for (int k = 0; k < kWideLBatch; k++) {
            if (b + k >= a.ntiles) break;  // (uniform)
            uint32_t chars = 0, far = 0;
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const uint32_t v = c[k][j];
                const uint32_t ln = v < dict_n ? static_cast<uint32_t>(l8s[v]) : 0u;
                far |= (ln == 255u ? 1u : 0u) << j;
                chars += ln;
            }
            if (__ballot(far != 0)) {  // (255 or more: the entry table's length)
#pragma unroll
                for (int j = 0; j < 8; j++)
                    if ((far >> j) & 1u) chars += static_cast<uint32_t>(es[c[k][j]] >> 32) - 255u;
            }
            tile_done(a, b + k, wave_sum(chars));
        }
    }
}

// ── regex page filter over the codes (README.md:54-64, SURVEY §8a R-REGEX) ─
// After k_pipe_runs / k_pipe_big / k_pipe_codes3: one wave per
// tile tests its rows' codes against the dictionary's match bits (the pattern
// ran once per entry, k_regex_dict).  A page whose tiles hold no non-null
// value that matches (with --neg-regex: that fails to match) stays reported.
// NULL rows and out-of-range indices (code 0xFFFF) never count.
constexpr int kMatchWaves = 4;
constexpr int kMatchBatch = 4;  // tiles whose codes a wave loads before testing any
// Persistent workgroups; each first packs the dictionary's match bytes into
// an LDS bit mask (a u16 code indexes at most 64 Ki entries: 8 KiB), then
// each wave takes kMatchBatch consecutive tiles per step (grid-stride), all
// their codes loaded before the first test, and tests them with LDS reads.
__global__ void __launch_bounds__(kMatchWaves * 64) k_pipe_match(const DevTile* __restrict__ tiles, int ntiles,
                                                                 const DevPage* __restrict__ pages,
                                                                 const uint16_t* __restrict__ codes,
                                                                 const uint8_t* __restrict__ match,
                                                                 const int32_t* __restrict__ dict_count, int dict_id,
                                                                 int neg, uint8_t* __restrict__ page_flags) {
    __shared__ uint32_t mbits[65536 / 32];
    const uint32_t dn = min(static_cast<uint32_t>(max(dict_count[dict_id], 0)), 65535u);
    const uint32_t nwd = (dn + 31) / 32;
    for (uint32_t wd = threadIdx.x; wd < nwd; wd += blockDim.x) {
        uint32_t m = 0;
        if (wd * 32 + 32 <= dn) {  // 32 bytes as eight dwords (match bytes are 0 or 1)
            const uint8_t* src = match + wd * 32;
            for (uint32_t q = 0; q < 8; q++) {
                uint32_t x;
                __builtin_memcpy(&x, src + 4 * q, 4);
                x = (x | (x >> 7) | (x >> 14) | (x >> 21)) & 0xFu;  // bytes 0..3 -> bits 0..3
                m |= x << (4 * q);
            }
        } else {
            for (uint32_t k = 0; k < 32; k++) {
                const uint32_t e = wd * 32 + k;
                m |= (e < dn && match[e] != 0 ? 1u : 0u) << k;
            }
        }
        // a NULL / out-of-range code never satisfies either predicate: its
        // bit is set where it must not count (neg flips the test below)
        mbits[wd] = m;
    }
    __syncthreads();
    const int nw = static_cast<int>(gridDim.x) * kMatchWaves;
    const uint32_t l8 = lane() * 8;
    for (int t0 = (static_cast<int>(blockIdx.x) * kMatchWaves + static_cast<int>(threadIdx.x / kWave)) * kMatchBatch;
         t0 < ntiles; t0 += nw * kMatchBatch) {
        U16B v[kMatchBatch];
        uint32_t m[kMatchBatch];
        int pg[kMatchBatch];
#pragma unroll
        for (int i = 0; i < kMatchBatch; i++) {
            m[i] = 0;
            pg[i] = -1;
            v[i] = U16B{0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
            if (t0 + i < ntiles) {
                const DevTile T = tiles[t0 + i];
                pg[i] = T.page;
                m[i] = static_cast<uint32_t>(T.nrows);
                if (l8 < m[i]) v[i] = *reinterpret_cast<const U16B*>(codes + pages[T.page].first_row + T.row0 + l8);
            }
        }
#pragma unroll
        for (int i = 0; i < kMatchBatch; i++) {
            const uint32_t w[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
            bool hit = false;
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const uint32_t c = (w[k >> 1] >> (16 * (k & 1))) & 0xFFFFu;
                const bool live = l8 + k < m[i] && c < dn;
                const uint32_t bit = (mbits[live ? (c >> 5) : 0u] >> (c & 31u)) & 1u;
                hit |= live && (bit != static_cast<uint32_t>(neg != 0));
            }
            if (__ballot(hit) && lane() == 0) page_flags[pg[i]] = 0;
        }
    }
}

// The same filter over the wide pipe's 32-bit codes: the match mask in
// dynamic LDS ((entries + 31) / 32 words, the host bounds the entry count by
// kMatchWideMax), two 16-byte code loads per lane and tile.
constexpr uint32_t kMatchWideMax = 1u << 20;
__global__ void __launch_bounds__(kMatchWaves * 64) k_pipe_match_w(const DevTile* __restrict__ tiles, int ntiles,
                                                                   const DevPage* __restrict__ pages,
                                                                   const uint32_t* __restrict__ codes,
                                                                   const uint8_t* __restrict__ match,
                                                                   const int32_t* __restrict__ dict_count, int dict_id,
                                                                   uint32_t cap, int neg, uint8_t* __restrict__ page_flags) {
    extern __shared__ __attribute__((aligned(16))) uint32_t mbw[];
    const uint32_t dn = min(static_cast<uint32_t>(max(dict_count[dict_id], 0)), cap);
    const uint32_t nwd = (dn + 31) / 32;
    for (uint32_t wd = threadIdx.x; wd < nwd; wd += blockDim.x) {
        uint32_t m = 0;
        if (wd * 32 + 32 <= dn) {
            const uint8_t* src = match + wd * 32;
            for (uint32_t q = 0; q < 8; q++) {
                uint32_t x;
                __builtin_memcpy(&x, src + 4 * q, 4);
                x = (x | (x >> 7) | (x >> 14) | (x >> 21)) & 0xFu;
                m |= x << (4 * q);
            }
        } else {
            for (uint32_t k = 0; k < 32; k++) {
                const uint32_t e = wd * 32 + k;
                m |= (e < dn && match[e] != 0 ? 1u : 0u) << k;
            }
        }
        mbw[wd] = m;
    }
    __syncthreads();
    const int nw = static_cast<int>(gridDim.x) * kMatchWaves;
    const uint32_t l8 = lane() * 8;
    for (int t0 = (static_cast<int>(blockIdx.x) * kMatchWaves + static_cast<int>(threadIdx.x / kWave)) * kMatchBatch;
         t0 < ntiles; t0 += nw * kMatchBatch) {
        U16B v[kMatchBatch][2];
        uint32_t m[kMatchBatch];
        int pg[kMatchBatch];
#pragma unroll
        for (int i = 0; i < kMatchBatch; i++) {
            m[i] = 0;
            pg[i] = -1;
            v[i][0] = v[i][1] = U16B{kNull32, kNull32, kNull32, kNull32};
            if (t0 + i < ntiles) {
                const DevTile T = tiles[t0 + i];
                pg[i] = T.page;
                m[i] = static_cast<uint32_t>(T.nrows);
                if (l8 < m[i]) {  // (codes past the tile's rows are read, never tested; the buffer has 64 spare rows)
                    const U16B* p = reinterpret_cast<const U16B*>(codes + pages[T.page].first_row + T.row0 + l8);
                    v[i][0] = p[0];
                    v[i][1] = p[1];
                }
            }
        }
#pragma unroll
        for (int i = 0; i < kMatchBatch; i++) {
            const uint32_t w[8] = {v[i][0].x, v[i][0].y, v[i][0].z, v[i][0].w, v[i][1].x, v[i][1].y, v[i][1].z, v[i][1].w};
            bool hit = false;
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const uint32_t c = w[k];
                const bool live = l8 + k < m[i] && c < dn;
                const uint32_t bit = (mbw[live ? (c >> 5) : 0u] >> (c & 31u)) & 1u;
                hit |= live && (bit != static_cast<uint32_t>(neg != 0));
            }
            if (__ballot(hit) && lane() == 0) page_flags[pg[i]] = 0;
        }
    }
}

}  // namespace

// The launch's LDS: the largest layout any page up to max_page_bytes takes.
// Past kBigOneSeg the jump table is half a page, so a page just under
// kBigOneSeg (one segment) can need more than the largest page.
static uint32_t big_lds_max(uint32_t max_page_bytes, uint32_t nlens) {
    uint32_t t = big_layout(max_page_bytes, nlens).total;
    if (max_page_bytes > kBigOneSeg) t = max(t, big_layout(kBigOneSeg, nlens).total);
    return t;
}

uint32_t pipe_big_lds(uint32_t max_page_bytes, uint32_t nlens) { return big_lds_max(max_page_bytes, nlens); }

bool pipe_match_wide_ok(uint32_t entries_cap) { return entries_cap <= kMatchWideMax; }

PipePlan plan_pipe_lds(uint32_t dict_bytes, int wpw) {
    PipePlan pl{};
    pl.lds = dict_bytes + static_cast<uint32_t>(wpw) * static_cast<uint32_t>(sizeof(WriteLds));
    const uint32_t all = pl.lds;
    pl.blocks_per_cu = all <= 160u * 1024 ? static_cast<int>((160u * 1024) / all) : 0;
    if (pl.blocks_per_cu > 4) pl.blocks_per_cu = 4;
    if (pl.blocks_per_cu > 0) {  // registers may allow fewer
        // (planned on the plain instance; the armed one, 2 KiB more static LDS,
        // runs the same grid: its workgroups never wait on one another)
        const int occ = resident_blocks(reinterpret_cast<const void*>(k_pipe_write<false>), wpw * kWave, pl.lds);
        pl.blocks_per_cu = min(pl.blocks_per_cu, occ);
    }
    return pl;
}

void launch_pipe_runs(hipStream_t s, const uint8_t* bytes, const DevPage* pages, int npages, int32_t max_def,
                      int32_t max_rep, uint2* runs, uint32_t* info, int pages_per_wave, int32_t* flist,
                      int debug, const RunDicts* dicts, uint32_t stage_max, uint32_t slot_max, uint32_t dict_max,
                      int cus) {
    (void)flist;  // flist[0] is cleared by the caller (capi.hip: one memset of flags, bsum, flist[0])
    const int nd = dicts ? dicts->ndicts : 0;
    if (npages <= 0 && nd <= 0) return;
    int ppw = pages_per_wave > 0 && pages_per_wave <= kRunPages ? pages_per_wave : kRunPages;
    if (pages_per_wave == 0) {  // auto: about two waves per SIMD over the chip, 4 .. 32 pages each
        const int target = max(1, npages / max(1, cus * 4 * 2));
        ppw = 4;
        while (ppw * 2 <= min(target, kRunPages)) ppw *= 2;
    }
    const int per = kRunWaves * ppw;
    const RunDictArgs d = dicts ? RunDictArgs{dicts->dicts, nd, dicts->entries, dicts->dict_count, dicts->dict_err,
                                              dicts->err_any}
                                : RunDictArgs{nullptr, 0, nullptr, nullptr, nullptr, nullptr};
    // window per wave: ppw page slots (slot_max: the largest small page's
    // slot; 0: unknown, kRunStage), at most kRunStage; the leading
    // workgroups' dictionary pages need dict_max + 32 bytes in all
    uint32_t wstage = slot_max ? static_cast<uint32_t>(ppw) * slot_max : kRunStage;
    wstage = min(kRunStage, (wstage + 15) / 16 * 16);
    if (nd) {  // dict_index_block needs the page + 32 bytes within the kRunWaves windows (+ 32 each)
        const uint32_t per_wave = (dict_max + 32 + kRunWaves - 1) / kRunWaves;
        const uint32_t ws = ((per_wave > 32 ? per_wave - 32 : 0u) + 15) / 16 * 16;
        wstage = max(wstage, min(kRunStage, ws));
    }
    const uint32_t lds = kRunWaves * (wstage / 4 + 8) * 4;
    ensure_dyn_lds(reinterpret_cast<const void*>(k_pipe_runs), lds);
    hipLaunchKernelGGL(k_pipe_runs, dim3(nd + (max(npages, 0) + per - 1) / per), dim3(kRunWaves * kWave), lds, s,
                       bytes, pages, npages, max_def, max_rep, runs, info, ppw, flist,
                       stage_max ? min(stage_max, kStage3 - 16) : kStage3 - 16, d, debug, wstage);
}

// k_pipe_write's grid and tiles per wavefront (k_pipe_codes files each tile's
// characters under the workgroup that will write it).
static void write_shape(const PipeLaunch& P, int* grid, int* per) {
    const int need = (P.ntiles + P.write_waves - 1) / P.write_waves;
    *grid = max(1, min(need, P.grid));
    const int nw = *grid * P.write_waves;
    *per = max(1, (P.ntiles + nw - 1) / nw);
}

void launch_pipe_codes(hipStream_t s, const PipeLaunch& P, bool count_pass) {
    if (P.ntiles <= 0 || (!count_pass && !P.has_small)) return;
    int wgrid = 0, per = 0;
    write_shape(P, &wgrid, &per);
    CodeArgs a{P.bytes, P.pages, P.tiles, P.ntiles, P.page_tile0, P.max_def, P.max_rep, P.dicts, P.dict_id,
               P.entries, P.dict_count, P.runs, P.info, P.tile_nn, P.codes, P.tile_chars, P.page_err, P.err_any,
               P.bsum, per, P.debug, P.write_waves};
    if (count_pass) {
        const dim3 grid((P.ntiles + kCodeWaves - 1) / kCodeWaves);
        hipLaunchKernelGGL(k_pipe_codes<true>, grid, dim3(kCodeWaves * kWave), 0, s, a);
        return;
    }
    // persistent: the entry-length table (u16 per entry) is loaded once per workgroup
    const uint32_t lt_n = P.dict_entries_cap;
    const uint32_t lds = (lt_n * 2 + 15) / 16 * 16;
    const void* fn = reinterpret_cast<const void*>(k_pipe_codes3);
    // resident workgroups per CU (LDS and registers), so the grid is one wave of blocks
    const int waves = kCodeWaves3;
    const int bpc = max(1, resident_blocks(fn, waves * kWave, lds));
    const int need = (P.ntiles + waves - 1) / waves;
    const int grid = max(1, min(need, P.cus * bpc));
    // also decodes the pages the run-table passes marked (flist)
    // (only k_pipe_big pages: nothing to do, k_pipe_big decoded its own
    // fallback pages exactly)
    if (P.has_small) hipLaunchKernelGGL(k_pipe_codes3, dim3(grid), dim3(kCodeWaves3 * kWave), lds, s, a, lt_n, P.flist);
}

PipePlan plan_pipe_wide(int wpw, bool pad) {
    PipePlan pl{};
    pl.lds = static_cast<uint32_t>(wpw) * (pad ? kWidePadWave : static_cast<uint32_t>(sizeof(WideLds)));
    pl.blocks_per_cu = min(4, static_cast<int>((160u * 1024) / pl.lds));
    const int occ = resident_blocks(pad ? reinterpret_cast<const void*>(k_pipe_wwide<true>)
                                        : reinterpret_cast<const void*>(k_pipe_wwide<false>),
                                    wpw * kWave, pl.lds);
    pl.blocks_per_cu = min(pl.blocks_per_cu, occ);
    return pl;
}

void launch_pipe_write(hipStream_t s, const PipeLaunch& P) {
    if (P.ntiles <= 0) return;
    if (P.codes32) {  // wide dictionary: codes and dictionary from HBM
        int grid = 0, per = 0;
        write_shape(P, &grid, &per);
        WriteArgs a{P.bytes, P.pages, P.tiles, P.ntiles, P.dicts, P.dict_id, P.entries, P.dict_count, nullptr,
                    P.tile_chars, P.bsum, per, P.nrows_total, P.total, P.capacity, P.overflow, P.validity, P.offsets,
                    P.chars, 0u, 0u, P.debug, P.write_waves, P.znext, P.znext_words, nullptr, 0, nullptr};
        a.codes32 = P.codes32;
        // (the plan sized P.lds for the slots whenever the dictionary has them)
        const uint32_t need_pad = static_cast<uint32_t>(P.write_waves) * kWidePadWave;
        if (P.pad16 && P.lds >= need_pad && !(P.debug & (1 << 29))) {  // (bit 29: entry words, for A/B)
            a.pad16 = P.pad16;
            ensure_dyn_lds(reinterpret_cast<const void*>(k_pipe_wwide<true>), P.lds);
            hipLaunchKernelGGL(k_pipe_wwide<true>, dim3(grid), dim3(P.write_waves * kWave), P.lds, s, a);
        } else {
            ensure_dyn_lds(reinterpret_cast<const void*>(k_pipe_wwide<false>), P.lds);
            hipLaunchKernelGGL(k_pipe_wwide<false>, dim3(grid), dim3(P.write_waves * kWave), P.lds, s, a);
        }
        return;
    }
    ensure_dyn_lds(reinterpret_cast<const void*>(k_pipe_write<false>), P.lds);
    ensure_dyn_lds(reinterpret_cast<const void*>(k_pipe_write<true>), P.lds);
    int grid = 0, per = 0;
    write_shape(P, &grid, &per);  // P.grid: resident workgroups (plan_pipe_lds + occupancy)
    WriteArgs a{P.bytes, P.pages, P.tiles, P.ntiles, P.dicts, P.dict_id, P.entries, P.dict_count, P.codes,
                P.tile_chars, P.bsum, per, P.nrows_total, P.total, P.capacity, P.overflow, P.validity, P.offsets,
                P.chars, P.dict_chars_bytes, P.dict_bytes, P.debug, P.write_waves, P.znext, P.znext_words,
                P.match, P.match_neg, P.page_flags};
    if (P.match)
        hipLaunchKernelGGL(k_pipe_write<true>, dim3(grid), dim3(P.write_waves * kWave), P.lds, s, a);
    else
        hipLaunchKernelGGL(k_pipe_write<false>, dim3(grid), dim3(P.write_waves * kWave), P.lds, s, a);
}

void launch_pipe_big(hipStream_t s, const PipeLaunch& P, const int32_t* big_pages, int nbig, uint32_t max_page_bytes) {
    const bool wide = P.codes32 != nullptr;  // lengths from the HBM entry table
    const uint32_t nlens = wide ? 0u : min(P.dict_entries_cap, kBigLens);
    if (nbig <= 0) return;
    int wgrid = 0, per = 0;
    write_shape(P, &wgrid, &per);  // tile characters are filed under k_pipe_write's workgroups
    CodeArgs a{P.bytes, P.pages, P.tiles, P.ntiles, P.page_tile0, P.max_def, P.max_rep, P.dicts, P.dict_id,
               P.entries, P.dict_count, P.runs, P.info, P.tile_nn, P.codes, P.tile_chars, P.page_err, P.err_any,
               P.bsum, per, P.debug, P.write_waves};
    a.codes32 = P.codes32;
    const uint32_t lds = big_lds_max(max_page_bytes, nlens);
    if (wide) {
        ensure_dyn_lds(reinterpret_cast<const void*>(k_pipe_big<true>), lds);
        hipLaunchKernelGGL(k_pipe_big<true>, dim3(nbig), dim3(kBigThreads), lds, s, a, big_pages,
                           const_cast<uint32_t*>(P.info), nlens, lds);
    } else {
        ensure_dyn_lds(reinterpret_cast<const void*>(k_pipe_big<false>), lds);
        hipLaunchKernelGGL(k_pipe_big<false>, dim3(nbig), dim3(kBigThreads), lds, s, a, big_pages,
                           const_cast<uint32_t*>(P.info), nlens, lds);
    }
}

void launch_wide_chars(hipStream_t s, const PipeLaunch& P) {
    if (P.ntiles <= 0 || !P.codes32) return;
    int wgrid = 0, per = 0;
    write_shape(P, &wgrid, &per);  // tile characters are filed under k_pipe_wwide's workgroups
    CodeArgs a{P.bytes, P.pages, P.tiles, P.ntiles, P.page_tile0, P.max_def, P.max_rep, P.dicts, P.dict_id,
               P.entries, P.dict_count, P.runs, P.info, P.tile_nn, P.codes, P.tile_chars, P.page_err, P.err_any,
               P.bsum, per, P.debug, P.write_waves};
    a.codes32 = P.codes32;
    if (P.lens8 && P.lens8_cap <= kWideLensLds && !(P.debug & (1 << 28))) {  // (bit 28: k_wide_chars, for A/B)
        const uint32_t lds = (P.lens8_cap + 15) / 16 * 16 + 16;
        ensure_dyn_lds(reinterpret_cast<const void*>(k_wide_chars_lds), kWideLensLds + 16);
        a.lens8 = P.lens8;
        const int need = (P.ntiles + kWideLWaves * kWideLBatch - 1) / (kWideLWaves * kWideLBatch);
        hipLaunchKernelGGL(k_wide_chars_lds, dim3(std::max(1, std::min(P.cus, need))), dim3(kWideLWaves * kWave), lds, s, a,
                           P.lens8_cap);
        return;
    }
    hipLaunchKernelGGL(k_wide_chars, dim3((P.ntiles + kWideCharWaves - 1) / kWideCharWaves), dim3(kWideCharWaves * kWave),
                       0, s, a);
}

void launch_pipe_match(hipStream_t s, const PipeLaunch& P, const uint8_t* match, int neg, uint8_t* page_flags,
                       bool flags_set) {
    if (!flags_set) (void)hipMemsetAsync(page_flags, 1, static_cast<size_t>(P.npages), s);
    if (P.ntiles <= 0) return;
    const int need = (P.ntiles + kMatchWaves * kMatchBatch - 1) / (kMatchWaves * kMatchBatch);
    const int grid = max(1, min(need, 4 * max(P.cus, 1)));
    if (P.codes32) {  // the wide pipe's codes (P.dict_entries_cap <= kMatchWideMax: pipe_match_wide_ok)
        const uint32_t cap = min(P.dict_entries_cap, kMatchWideMax);
        const uint32_t lds = max(16u, (cap + 31) / 32 * 4);
        ensure_dyn_lds(reinterpret_cast<const void*>(k_pipe_match_w), lds);
        hipLaunchKernelGGL(k_pipe_match_w, dim3(grid), dim3(kMatchWaves * kWave), lds, s, P.tiles, P.ntiles, P.pages,
                           P.codes32, match, P.dict_count, P.dict_id, cap, neg, page_flags);
        return;
    }
    hipLaunchKernelGGL(k_pipe_match, dim3(grid), dim3(kMatchWaves * kWave), 0, s,
                       P.tiles, P.ntiles, P.pages, P.codes, match, P.dict_count, P.dict_id, neg, page_flags);
}

}  // namespace pqk
