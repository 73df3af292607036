// regex.hip — bit-parallel Glushkov NFA page filter on gfx950.
//
// k_regex_dict   one workgroup per dictionary page: every entry is matched
//                once (dictionary-first, SURVEY §8a R-REGEX), result bytes
//                in dict_match[].
// k_regex_pages  one wavefront per data page: decode levels (and indices) with
//                the same state machine as the decode kernels, then
//                dictionary pages test match bits of their indices, PLAIN
//                pages run the NFA, one string per lane, bytes from LDS.
// A page is REPORTED (flag 1) iff no non-null value satisfies the predicate
// (match, or non-match under --neg-regex); NULLs satisfy neither.
#include <algorithm>
#include <cstring>

#include "kernels/device_common.hpp"
#include "kernels/kernels.hpp"
#include "kernels/lane_walk.hpp"
#include "pq_gpu.h"
#include "regex/regex.hpp"

namespace pqre {
namespace {

using pqk::ColumnParams;
using pqk::DevDict;
using pqk::DevErr;
using pqk::DevPage;
using pqk::kTileRows;
using pqk::kWave;
using namespace pqk::dev;

constexpr int kWavesPerBlock = 4;
constexpr uint32_t kStageWords = 1024;

// Stage the program into LDS (whole workgroup).
__device__ void load_prog(DevProg* dst, const DevProg* src) {
    const uint4* s = reinterpret_cast<const uint4*>(src);
    uint4* d = reinterpret_cast<uint4*>(dst);
    for (uint32_t i = threadIdx.x; i < sizeof(DevProg) / 16; i += blockDim.x) d[i] = s[i];
    __syncthreads();
}

// NFA over one string; byte(i) yields the i-th byte.
template <class B>
__device__ __forceinline__ bool nfa_match(const DevProg& P, uint32_t n, B&& byte) {
    if (n == 0) return P.empty_string != 0;
    if (P.nonempty_trivial) return true;
    uint64_t D = 0;
    for (uint32_t i = 0; i < n; i++) {
        uint64_t f = i == 0 ? P.first_at0 : P.first_mid;
        for (uint32_t k = 0; k < P.nchunks; k++) f |= P.ftab[k][(D >> (8 * k)) & 0xFF];
        D = f & P.cls[byte(i)];
        if (D & P.last) return true;
        if (D == 0 && P.first_mid == 0) return false;
    }
    return (D & P.accept_end) != 0;
}

// One entry per thread, entries spread over gridDim.y workgroups per
// dictionary; string bytes come 16 at a time (unaligned global loads; the
// payload slot has >= 16 zero bytes after the page), not one load per byte.
struct __attribute__((packed, aligned(1))) U16B { uint32_t x, y, z, w; };
__global__ void __launch_bounds__(256) k_regex_dict(const DevProg* __restrict__ prog,
                                                    const uint8_t* __restrict__ bytes,
                                                    const DevDict* __restrict__ dicts,
                                                    const uint64_t* __restrict__ entries,
                                                    const int32_t* __restrict__ dict_count,
                                                    uint8_t* __restrict__ dict_match,
                                                    uint8_t* __restrict__ fill1, int64_t nfill1,
                                                    uint32_t* __restrict__ zero, int64_t nzero) {
    __shared__ DevProg P;
    {
        const int64_t t = (static_cast<int64_t>(blockIdx.x) * gridDim.y + blockIdx.y) * blockDim.x + threadIdx.x;
        const int64_t nt = static_cast<int64_t>(gridDim.x) * gridDim.y * blockDim.x;
        for (int64_t i = t; i < nfill1; i += nt) fill1[i] = 1;
        for (int64_t i = t; i < nzero; i += nt) zero[i] = 0;
    }
    load_prog(&P, prog);
    const DevDict d = dicts[blockIdx.x];
    const int32_t n = dict_count[blockIdx.x];
    const uint8_t* base = bytes + d.off;
    for (int32_t k = blockIdx.y * blockDim.x + threadIdx.x; k < n; k += blockDim.x * gridDim.y) {
        const uint64_t e = entries[d.entry_base + k];
        const uint8_t* s = base + static_cast<uint32_t>(e);
        const uint32_t len = static_cast<uint32_t>(e >> 32);
        uint32_t w0 = 0, w1 = 0, w2 = 0, w3 = 0, blk = ~0u;
        dict_match[d.entry_base + k] = nfa_match(P, len, [&](uint32_t i) {
            if ((i >> 4) != blk) {
                blk = i >> 4;
                const U16B v = *reinterpret_cast<const U16B*>(s + 16 * blk);
                w0 = v.x; w1 = v.y; w2 = v.z; w3 = v.w;
            }
            const uint32_t q = (i >> 2) & 3u;
            const uint32_t w = q == 0 ? w0 : (q == 1 ? w1 : (q == 2 ? w2 : w3));
            return (w >> (8 * (i & 3u))) & 0xFFu;
        });
    }
}

struct PageLds {
    uint32_t stage[kStageWords];
    uint32_t lv[kTileRows];
    uint32_t a[kTileRows];
    uint32_t b[kTileRows];
};


__global__ void __launch_bounds__(256) k_regex_pages(const DevProg* __restrict__ prog,
                                                     const uint8_t* __restrict__ bytes,
                                                     const DevPage* __restrict__ pages, int npages,
                                                     const DevDict* __restrict__ dicts,
                                                     const uint64_t* __restrict__ entries,
                                                     const int32_t* __restrict__ dict_count,
                                                     const uint8_t* __restrict__ dict_match,
                                                     ColumnParams cp, int neg,
                                                     uint8_t* __restrict__ page_flags,
                                                     DevErr* __restrict__ page_err,
                                                     int32_t* __restrict__ err_any) {
    __shared__ DevProg P;
    __shared__ PageLds lds_all[kWavesPerBlock];
    load_prog(&P, prog);
    const int wv = threadIdx.x / kWave;
    const int p = blockIdx.x * kWavesPerBlock + wv;
    if (p >= npages) return;
    PageLds& L = lds_all[wv];
    const DevPage pg = pages[p];
    DevErr* err = page_err + p;
    const uint8_t* g = bytes + pg.off;
    const uint32_t size = static_cast<uint32_t>(pg.size);
    Src s{nullptr, g, size};
    if (size <= kStageWords * 4) {
        stage_page(L.stage, g, size);
        s.lds = L.stage;
    }
    const int32_t nv = pg.nvals;
    uint32_t pos = 0;
    Rle def;
    const bool has_def = cp.max_def > 0;
    if (has_def) {
        if (pos + 4 > size) { set_err(err, err_any, PQ_ERR_BUFFER, pos, 4, size); return; }
        uint32_t def_len = src_u32(s, pos);
        pos += 4;
        if (static_cast<uint64_t>(pos) + def_len > size) { set_err(err, err_any, PQ_ERR_BUFFER, pos, def_len, size); return; }
        rle_init(def, pos, def_len, level_bw(cp.max_def));
        pos += def_len;
    }
    if (cp.max_rep > 0) {
        if (pos + 4 > size) { set_err(err, err_any, PQ_ERR_BUFFER, pos, 4, size); return; }
        uint32_t rep_len = src_u32(s, pos);
        pos += 4;
        if (static_cast<uint64_t>(pos) + rep_len > size) { set_err(err, err_any, PQ_ERR_BUFFER, pos, rep_len, size); return; }
        pos += rep_len;
    }
    const bool dict = pg.mode == pqk::MODE_DICT;
    Rle ix;
    uint32_t dict_n = 0, entry_base = 0;
    if (dict) {
        if (pos + 1 > size) { set_err(err, err_any, PQ_ERR_BUFFER, pos, 1, size); return; }
        uint32_t bw = src_byte(s, pos);
        pos += 1;
        rle_init(ix, pos, size - pos, bw);
        dict_n = static_cast<uint32_t>(dict_count[pg.dict]);
        entry_base = static_cast<uint32_t>(dicts[pg.dict].entry_base);
    }
    bool any = false;
    for (int32_t r0 = 0; r0 < nv; r0 += kTileRows) {
        const uint32_t m = min(static_cast<uint32_t>(nv - r0), static_cast<uint32_t>(kTileRows));
        int rc = 0;
        if (has_def) rc = rle_decode(def, s, m, [&](uint32_t j, uint32_t v) { L.lv[j] = v & 0xFFFFu; });
        else for (uint32_t j = lane(); j < m; j += kWave) L.lv[j] = static_cast<uint32_t>(cp.max_def);
        __builtin_amdgcn_wave_barrier();
        uint32_t nn = 0, above = 0;
        for (uint32_t j0 = 0; j0 < m; j0 += kWave) {
            uint32_t j = j0 + lane();
            int32_t d = j < m ? static_cast<int16_t>(L.lv[j]) : -32768;
            bool isnn = dict ? d == cp.max_def : d >= cp.max_def;
            nn += __popcll(__ballot(isnn));
            above |= __ballot(d > cp.max_def) != 0;
        }
        if (rc == 0 && dict && above) rc = PQ_ERR_UNSUPPORTED;
        if (rc) { set_err(err, err_any, rc, 0, 0, size); return; }
        if (dict) {
            rc = rle_decode(ix, s, nn, [&](uint32_t j, uint32_t v) { L.a[j] = v; });
            if (rc) { set_err(err, err_any, rc, 0, 0, size); return; }
            __builtin_amdgcn_wave_barrier();
            for (uint32_t k0 = 0; k0 < nn; k0 += kWave) {
                uint32_t k = k0 + lane();
                bool sat = false;
                if (k < nn) {
                    uint32_t idx = L.a[k];
                    bool ok = static_cast<int32_t>(idx) >= 0 && idx < dict_n;
                    sat = ok && ((dict_match[entry_base + idx] != 0) != (neg != 0));
                }
                any |= __ballot(sat) != 0;
            }
        } else {
            int failed = 0;
            if (lane() == 0) {  // PLAIN BYTE_ARRAY chain (column_reader.cpp:249-253)
                for (uint32_t k = 0; k < nn; k++) {
                    if (static_cast<uint64_t>(pos) + 4 > size) { set_err(err, err_any, PQ_ERR_BUFFER, pos, 4, size); failed = 1; break; }
                    uint32_t len = src_u32(s, pos);
                    pos += 4;
                    if (static_cast<uint64_t>(pos) + len > size) { set_err(err, err_any, PQ_ERR_BUFFER, pos, len, size); failed = 1; break; }
                    L.a[k] = pos;
                    L.b[k] = len;
                    pos += len;
                }
            }
            failed = __shfl(failed, 0, kWave);
            pos = __shfl(pos, 0, kWave);
            if (failed) return;
            __builtin_amdgcn_wave_barrier();
            if (!any) {
                for (uint32_t k0 = 0; k0 < nn && !any; k0 += kWave) {
                    uint32_t k = k0 + lane();
                    bool sat = false;
                    if (k < nn) {
                        uint32_t st = L.a[k], len = L.b[k];
                        bool mt = nfa_match(P, len, [&](uint32_t i) { return src_byte(s, st + i); });
                        sat = mt != (neg != 0);
                    }
                    any |= __ballot(sat) != 0;
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
    if (lane() == 0) page_flags[p] = any ? 0 : 1;
}


// ── lane-per-page DFA scan ──────────────────────────────────────────────────
// One lane per data page (a wavefront scans 64 pages at once): def levels
// and dictionary indices with the reference's RLE state machine
// (lane_walk.hpp), PLAIN strings streamed through a 16-byte register window
// into the DFA (one LDS lookup per byte).  Once its page has a satisfying
// value a lane stops matching but still walks the rest of the page (levels,
// indices, the length chain), so a later decode error fails the scan.
__device__ __forceinline__ uint32_t dfa_step_full(const uint16_t* T, uint32_t e, uint32_t b) {
    return *reinterpret_cast<const uint16_t*>(reinterpret_cast<const uint8_t*>(T) + e + 2 * b);
}

// i < rem ? t : e, as one compare into VCC and one select: opaque to the
// compiler, so the 64 per-byte compares of a block are not hoisted into SGPR
// masks that spill (and no copy of rem is made per byte).
template <class I>
__device__ __forceinline__ uint32_t sel_below(I i, uint32_t rem, uint32_t t, uint32_t e) {
    uint32_t r;
    __asm__("v_cmp_lt_u32 vcc, %3, %2\n\tv_cndmask_b32 %0, %4, %1, vcc"
            : "=v"(r)
            : "v"(t), "v"(rem), "n"(static_cast<uint32_t>(i)), "v"(e)
            : "vcc");
    return r;
}

__device__ __forceinline__ void lane_err(DevErr* e, int32_t* any, int code, uint32_t pos, uint32_t need,
                                         uint32_t size) {
    e->code = code;
    e->pos = static_cast<int32_t>(pos);
    e->need = static_cast<int32_t>(need);
    e->size = static_cast<int32_t>(size);
    atomicOr(any, 1);
}

__global__ void __launch_bounds__(256) k_regex_lanes(const uint8_t* __restrict__ dfa_img, uint32_t dfa_bytes,
                                                     const uint8_t* __restrict__ bytes,
                                                     const DevPage* __restrict__ pages, int npages,
                                                     const DevDict* __restrict__ dicts,
                                                     const int32_t* __restrict__ dict_count,
                                                     const uint8_t* __restrict__ dict_match,
                                                     ColumnParams cp, int neg,
                                                     uint8_t* __restrict__ page_flags,
                                                     DevErr* __restrict__ page_err,
                                                     int32_t* __restrict__ err_any) {
    extern __shared__ __attribute__((aligned(16))) uint8_t dsm[];
    {
        const uint4* src = reinterpret_cast<const uint4*>(dfa_img);
        uint4* dst = reinterpret_cast<uint4*>(dsm);
        copy_blocks(dst, src, dfa_bytes / 16, threadIdx.x, blockDim.x);
    }
    __syncthreads();
    const DevDfa* D = reinterpret_cast<const DevDfa*>(dsm);
    const uint16_t* T = reinterpret_cast<const uint16_t*>(dsm + sizeof(DevDfa));
    const uint32_t nc = D->nclasses;
    const bool empty_ok = D->empty_string != 0;
    const bool trivial = D->nonempty_trivial != 0;
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= npages) return;
    const DevPage pg = pages[p];
    const uint8_t* page = bytes + pg.off;
    const uint32_t size = static_cast<uint32_t>(pg.size);
    const uint32_t nv = static_cast<uint32_t>(max(pg.nvals, 0));
    DevErr* err = page_err + p;
    auto rd8 = [&](uint32_t a) { return gld8(page, a); };
    const bool dict = pg.mode == pqk::MODE_DICT;
    const uint32_t md = static_cast<uint32_t>(cp.max_def);
    uint32_t pos = 0, nn = nv;
    // def levels (column_reader.cpp:146-170)
    if (cp.max_def > 0) {
        if (pos + 4 > size) { lane_err(err, err_any, PQ_ERR_BUFFER, pos, 4, size); return; }
        const uint32_t dl = static_cast<uint32_t>(gld8(page, pos));
        pos += 4;
        if (static_cast<uint64_t>(pos) + dl > size) { lane_err(err, err_any, PQ_ERR_BUFFER, pos, dl, size); return; }
        LRle r = lrle(pos, dl, level_bw(cp.max_def));
        const uint32_t bwd = r.bw;
        nn = 0;
        bool above = false;
        const int rc = lane_rle(r, rd8, nv, [&](uint32_t kind, uint32_t k, uint32_t arg) {
            if (kind == 0) {
                if (dict ? arg == md : arg >= md) nn += k;
                above |= arg > md;
            } else {
                for (uint32_t i = 0; i < k; i++) {
                    const uint32_t v = gbits(page, size, static_cast<uint64_t>(arg) + i * bwd, bwd);
                    if (dict ? v == md : v >= md) nn++;
                    above |= v > md;
                }
            }
        });
        if (rc) { lane_err(err, err_any, rc, 0, 0, size); return; }
        if (dict && above) { lane_err(err, err_any, PQ_ERR_UNSUPPORTED, 0, 0, size); return; }
        pos += dl;
    }
    if (cp.max_rep > 0) {
        if (pos + 4 > size) { lane_err(err, err_any, PQ_ERR_BUFFER, pos, 4, size); return; }
        const uint32_t rl = static_cast<uint32_t>(gld8(page, pos));
        pos += 4;
        if (static_cast<uint64_t>(pos) + rl > size) { lane_err(err, err_any, PQ_ERR_BUFFER, pos, rl, size); return; }
        pos += rl;
    }
    bool any = false;
    if (dict) {  // indices -> dictionary match bits (column_reader.cpp:174-196)
        if (pos + 1 > size) { lane_err(err, err_any, PQ_ERR_BUFFER, pos, 1, size); return; }
        const uint32_t bw = static_cast<uint32_t>(gld8(page, pos)) & 0xFFu;
        pos += 1;
        const uint32_t dict_n = static_cast<uint32_t>(dict_count[pg.dict]);
        const uint8_t* mt = dict_match + dicts[pg.dict].entry_base;
        auto sat = [&](uint32_t v) {
            return static_cast<int32_t>(v) >= 0 && v < dict_n && ((mt[v] != 0) != (neg != 0));
        };
        LRle r = lrle(pos, size - pos, bw);
        const int rc = lane_rle(r, rd8, nn, [&](uint32_t kind, uint32_t k, uint32_t arg) {
            if (any || k == 0) return;
            if (kind == 0) {
                any = sat(arg);
            } else {
                for (uint32_t i = 0; i < k && !any; i++)
                    any = sat(gbits(page, size, static_cast<uint64_t>(arg) + static_cast<uint64_t>(i) * bw, bw));
            }
        });
        if (rc) { lane_err(err, err_any, rc, 0, 0, size); return; }
    } else if (nn) {  // PLAIN: u32 length + bytes per value (column_reader.cpp:249-253)
        const uint32_t slot_end = (size + 15) / 16 * 16 + 16;  // readable bytes of the slot
        auto win = [&](uint32_t at) {
            const bool ok = at + 16 <= slot_end;
            const uint4 v = *reinterpret_cast<const uint4*>(page + (ok ? at : 0u));
            return ok ? v : make_uint4(0, 0, 0, 0);
        };
        const bool full = D->full != 0;
        const uint32_t negv = neg != 0;
        uint32_t k = 0, cur = pos;
        int ecode = 0;
        uint32_t epos = 0, eneed = 0;
        // (a page that already matched still walks its whole length chain:
        // an error further on fails the scan as it fails the page's decode)
        while (__ballot(k < nn && !ecode)) {
            // 1. the next kCollect strings' (offset, length): length chain
            //    (ByteBuffer reads, column_reader.cpp:249-253) and its errors
            constexpr uint32_t kCollect = 8;
            uint32_t soff[kCollect], slen[kCollect];
            uint32_t cnt = 0;
#pragma unroll
            for (uint32_t c = 0; c < kCollect; c++) {
                soff[c] = 0;
                slen[c] = 0;
                if (k < nn && !ecode) {
                    if (static_cast<uint64_t>(cur) + 4 > size) {
                        ecode = PQ_ERR_BUFFER; epos = cur; eneed = 4;
                    } else {
                        const uint32_t len = static_cast<uint32_t>(gld8(page, cur));
                        cur += 4;
                        if (static_cast<uint64_t>(cur) + len > size) {
                            ecode = PQ_ERR_BUFFER; epos = cur; eneed = len;
                        } else {
                            soff[c] = cur;
                            slen[c] = len;
                            cur += len;
                            k++;
                            cnt = c + 1;
                        }
                    }
                }
            }
            // 2. match them, one string per lane at a time, 16-byte blocks
            uint4 N0 = win(soff[0] & ~15u), N1 = win((soff[0] & ~15u) + 16);
#pragma unroll
            for (uint32_t c = 0; c < kCollect; c++) {
                if (!__ballot(c < cnt)) break;
                const bool act = c < cnt && !any && !ecode;
                const uint32_t off = soff[c], len = act ? slen[c] : 0u;
                const uint32_t o = off & 15u, sh = o & 3, q = o >> 2;
                uint32_t wb = off - o;
                uint4 W0 = N0, W1 = N1, W2 = win(wb + 32);
                if (c + 1 < kCollect) {  // prefetch the next string's first blocks
                    const uint32_t nb = soff[c + 1] & ~15u;
                    N0 = win(nb);
                    N1 = win(nb + 16);
                }
                uint32_t e = full ? (DFA_START * kDfaRowBytes) : DFA_START;
                // (ballots only: lanes of other branches are inactive here)
                for (uint32_t b0 = 0; __ballot(len > b0); b0 += 16) {
                    const uint32_t w[8] = {W0.x, W0.y, W0.z, W0.w, W1.x, W1.y, W1.z, W1.w};
                    uint32_t A[4];
#pragma unroll
                    for (uint32_t j = 0; j < 4; j++) {
                        uint32_t lo = w[j], hi = w[j + 1];
                        lo = q == 1 ? w[j + 1] : lo; hi = q == 1 ? w[j + 2] : hi;
                        lo = q == 2 ? w[j + 2] : lo; hi = q == 2 ? w[j + 3] : hi;
                        lo = q == 3 ? w[j + 3] : lo; hi = q == 3 ? w[j + 4] : hi;
                        A[j] = __builtin_amdgcn_alignbyte(hi, lo, sh);
                    }
                    const uint32_t rem = len > b0 ? len - b0 : 0u;
                    if (full) {
#pragma unroll
                        for (uint32_t i = 0; i < 16; i++) {
                            const uint32_t t = dfa_step_full(T, e, (A[i >> 2] >> (8 * (i & 3))) & 0xFFu);
                            e = i < rem ? t : e;
                        }
                    } else {
#pragma unroll
                        for (uint32_t i = 0; i < 16; i++) {
                            const uint32_t bt = (A[i >> 2] >> (8 * (i & 3))) & 0xFFu;
                            const uint32_t t = T[(e & 0x7FFFu) * nc + D->cls_of[bt]];
                            e = i < rem ? t : e;
                        }
                    }
                    wb += 16;
                    W0 = W1;
                    W1 = W2;
                    W2 = win(wb + 32);
                }
                const uint32_t st = full ? e / kDfaRowBytes : (e & 0x7FFFu);
                const bool acc = full ? dfa_step_full(T, e, 256) != 0 : (e >> 15) != 0;
                const bool m = len == 0 ? empty_ok : (trivial || st == DFA_ACCEPT || acc);
                if (act) any = (static_cast<uint32_t>(m) != negv);
            }
        }
        if (ecode) {
            lane_err(err, err_any, ecode, epos, eneed, size);
            return;
        }
    }
    page_flags[p] = any ? 0 : 1;
}

// ── windowed PLAIN scan ─────────────────────────────────────────────────────
// Chunks without dictionary pages.  Each wave takes windows of consecutive
// pages (one contiguous image range, <= win_bytes) with a static grid stride,
// and per window:
//   staging   the window's bytes -> LDS with coalesced 16-byte loads, eight
//             in flight per lane (copy_blocks); the next window's descriptors
//             load while this one is scanned.  (A loader wave feeding two LDS
//             buffers per scanning wave by LDS-DMA measured slower on C3, 0.47
//             vs 0.40 ms: one loader per CU could not keep up, and the second
//             buffer cost a third of the scanning waves);
//   strings   the u32 length chain of every page (column_reader.cpp:249-253)
//             is walked by L = 64 / pages lanes per page: each lane takes a
//             byte segment of the page and finds its first candidate string
//             start (a position whose u32 length fits the page; 16 positions
//             per aligned read) and walks that chain to the segment end; the
//             segments link when each starts where the previous one left
//             (one shuffle), a scan places every segment's strings in the
//             page's list, and the chains are re-walked to emit them.  A page
//             whose segments do not link, or whose chain fails before its
//             value count, is walked again by one lane in the reference order
//             (exact errors).  (C3: 0.068 ms against 0.082 for one lane per
//             page);
//   DFA       all 64 lanes run the DFA over the listed strings, four strings
//             per lane interleaved, one LDS lookup per byte; table entries are
//             bare row offsets (the accept-at-end flag sits in column 256 of
//             a row, read once per string), and the per-byte end-of-string
//             selects are kept out of SGPR masks (C3: 0.119 ms, was 0.166).
// waves per workgroup: as many as the LDS holds (host), <= 3 per SIMD (the
// next window's bytes ride in registers)
constexpr uint32_t kPlainWavesMax = 12;
constexpr uint32_t kStrPerLane = 4;  // strings interleaved per lane (independent DFA chains)

// The u32 at byte a of the staged window (>= 8 readable bytes past a).
__device__ __forceinline__ uint32_t st_u32(const uint32_t* st, uint32_t a) {
    const uint32_t i = a >> 2, sh = a & 3u;
    return __builtin_amdgcn_alignbyte(st[i + 1], st[i], sh);
}



// kSink (anchored patterns, full tables): a batch stops after its first block
// once every longer string sits in an absorbing state (DEAD); a template
// parameter, as the test costs unanchored patterns more than it saves
template <bool kSink>
__global__ void __launch_bounds__(kPlainWavesMax * 64) k_regex_plain(const uint8_t* __restrict__ dfa_img,
                                                                  uint32_t dfa_bytes, uint32_t win_bytes,
                                                                  const uint8_t* __restrict__ bytes,
                                                                  const DevPage* __restrict__ pages,
                                                                  const pqk::DevBatch* __restrict__ wins,
                                                                  int nwins, int32_t* __restrict__ ticket,
                                                                  ColumnParams cp, int neg,
                                                                  uint8_t* __restrict__ page_flags,
                                                                  DevErr* __restrict__ page_err,
                                                                  int32_t* __restrict__ err_any,
                                                                  const uint16_t* __restrict__ index_in,
                                                                  uint16_t* __restrict__ index_out) {
    extern __shared__ __attribute__((aligned(16))) uint8_t dsm[];
    // Full tables are rebuilt in LDS as bytes: T8[state << 8 | byte] = next
    // state, A8[state] = accepts at the string end (a full table has < 64
    // states).  The DFA step is then one v_perm (state and byte into the
    // address) and one ds_read_u8, against a shift, an add and a ds_read_u16
    // over the u16 byte-offset rows.  Class tables are copied as they are.
    const DevDfa* Dg = reinterpret_cast<const DevDfa*>(dfa_img);
    if (Dg->full) {
        const uint4* src = reinterpret_cast<const uint4*>(dfa_img);
        uint4* dst = reinterpret_cast<uint4*>(dsm);
        copy_blocks(dst, src, static_cast<uint32_t>(sizeof(DevDfa)) / 16, threadIdx.x, blockDim.x);
        const uint16_t* Tg = reinterpret_cast<const uint16_t*>(dfa_img + sizeof(DevDfa));
        uint8_t* T8w = dsm + sizeof(DevDfa);
        const uint32_t nst = Dg->nstates;
        for (uint32_t i = threadIdx.x; i < nst * 256; i += blockDim.x)
            T8w[i] = static_cast<uint8_t>(Tg[(i >> 8) * (kDfaRowBytes / 2) + (i & 255)] / kDfaRowBytes);
        for (uint32_t st = threadIdx.x; st < nst; st += blockDim.x)
            T8w[nst * 256 + st] = Tg[st * (kDfaRowBytes / 2) + 256] != 0 ? 1 : 0;
    } else {
        const uint4* src = reinterpret_cast<const uint4*>(dfa_img);
        uint4* dst = reinterpret_cast<uint4*>(dsm);
        copy_blocks(dst, src, dfa_bytes / 16, threadIdx.x, blockDim.x);
    }
    __syncthreads();
    const DevDfa* D = reinterpret_cast<const DevDfa*>(dsm);
    const uint16_t* T = reinterpret_cast<const uint16_t*>(dsm + sizeof(DevDfa));
    const uint8_t* T8 = dsm + sizeof(DevDfa);
    const uint8_t* A8 = T8 + D->nstates * 256;
    // T8 as an LDS address constant: dsm is this kernel's only LDS object, so
    // it starts at LDS address 0 and the table lookup needs no base add (the
    // dsm-relative form costs a VALU add per lookup).  The host verifies the
    // kernel has no static LDS before it launches it (regex_plain_lds_ok).
    using lds_u8 = const __attribute__((address_space(3))) uint8_t;
    lds_u8* T8c = reinterpret_cast<lds_u8*>(static_cast<uintptr_t>(sizeof(DevDfa)));
    const uint32_t nc = D->nclasses;
    const bool full = D->full != 0;
    const bool empty_ok = D->empty_string != 0;
    const bool trivial = D->nonempty_trivial != 0;
    const uint32_t negv = neg & 1;  // bits 8..15: timing ablation (1: no DFA pass, 2: no chain walk,
    const int dbg = pqk::dev::kProbes ? (neg >> 8) & 0xFF : 0;  // 4: exact walk for every page; probe build only)
    const uint32_t wv = threadIdx.x / kWave;
    const uint32_t wpb = blockDim.x / kWave;
    const uint32_t md = static_cast<uint32_t>(cp.max_def);
    (void)ticket;
    // scanning wave c (1 .. wpb - 1) of workgroup g takes windows
    // (g * K + c - 1) + i * nwt, i = 0, 1, ...; buffer i & 1
    const uint32_t K = wpb;
    const int32_t nwt = static_cast<int32_t>(gridDim.x * K);
    // ── scanning waves ──────────────────────────────────────────────────
    const uint32_t c = wv;
    uint8_t* wbase = dsm + dfa_bytes + c * regex_plain_wave_lds(win_bytes);
    uint8_t* cur = wbase;  // the window (+32 zero bytes)
    uint16_t* list = reinterpret_cast<uint16_t*>(wbase + win_bytes + 32);  // window offset of each string
    uint32_t* pref = reinterpret_cast<uint32_t*>(wbase + win_bytes + 32 + win_bytes / 2);
    uint32_t* lbase = pref + 64;
    uint32_t* pcnt = lbase + 64;
    uint32_t* hit = pcnt + 64;  // [0..1]: satisfied-page mask of the window
    int32_t w = static_cast<int32_t>(blockIdx.x * K + c);
    if (w >= nwins) return;
    // descriptors two windows ahead: the batch of window i + 2 and the
    // pages of window i + 1 load while window i is scanned
    pqk::DevBatch B = wins[w];
    pqk::DevBatch Bn{};
    if (w + nwt < nwins) Bn = wins[w + nwt];
    DevPage pg{};
    if (lane() < static_cast<uint32_t>(B.np)) pg = pages[B.p0 + static_cast<int32_t>(lane())];
    // the next window's bytes ride in registers while this window is scanned
    // (windows of <= kPrefetchBlocks * 1 KiB; larger ones are copied in place)
    constexpr uint32_t kPrefetchBlocks = 8;  // 16-byte blocks per lane
    // (eight named registers: an array carried around the loop went to scratch)
    uint4 R0, R1, R2, R3, R4, R5, R6, R7;
    bool held = false;
    // The memory waits of the loop (gfx9: loads and stores share vmcnt, and
    // a wait for an older load also waits for every later one): the window is
    // staged at the END of the previous iteration, where the single wait
    // covers its prefetch (issued before the DFA pass), the descriptors
    // loaded at the top and the index stores, all long complete; a window's
    // page flags are stored at the top of the next iteration, so no wait
    // ever covers a fresh store.  (Staged at the top, the wait for the
    // prefetch fell right after its issue.)
    copy_blocks(reinterpret_cast<uint4*>(cur), reinterpret_cast<const uint4*>(bytes + B.img_lo), B.img_bytes / 16,
                lane(), kWave);
    if (lane() < 2) reinterpret_cast<uint4*>(cur + B.img_bytes)[lane()] = make_uint4(0, 0, 0, 0);
    // a warm scan: a window's string-index entries (<= 256 strings, rows
    // b.row0 .. b.row0 + b.nrows - 1), loaded into registers one window
    // ahead (entry k in lane k % 64, half k / 128 of word (k / 64) % 2)
    auto ix_load = [&](const pqk::DevBatch& b, uint32_t& v01, uint32_t& v23) -> bool {
        const uint32_t tot = b.nrows;
        if (!index_in || tot == 0 || tot > 4 * kWave) return false;
        auto at = [&](uint32_t j) -> uint32_t {  // (clamped indices: unconditional loads)
            const uint32_t k = j * kWave + lane();
            return index_in[b.row0 + (k < tot ? k : 0u)];
        };
        const uint32_t a0 = at(0), a1 = at(1), a2 = at(2), a3 = at(3);
        v01 = a0 | (a1 << 16);
        v23 = a2 | (a3 << 16);
        return true;
    };
    uint32_t ix01 = 0, ix23 = 0;
    bool ix_held = ix_load(B, ix01, ix23);
    bool pf_on = false;  // the previous window's page flag (one lane per page)
    int32_t pf_at = 0;
    uint8_t pf_v = 0;
    for (;;) {
        const pqk::DevBatch Bc = B;
        const DevPage pgc = pg;
        const int32_t wn = w + nwt;
        if (pf_on) page_flags[pf_at] = pf_v;
        // every load for the next window at once, before this window's work:
        // its page descriptors, the batch after it, its bytes (registers, up
        // to kPrefetchBlocks KiB) and a warm scan's index entries; the one
        // wait at the end of the iteration covers them all (no load of the
        // loop depends on another load of the same iteration)
        DevPage pgn{};
        pqk::DevBatch Bnn{};
        uint32_t ixn01 = 0, ixn23 = 0;
        bool ixn_held = false;
        held = false;
        if (wn < nwins) {
            if (lane() < static_cast<uint32_t>(Bn.np)) pgn = pages[Bn.p0 + static_cast<int32_t>(lane())];
            if (wn + nwt < nwins) Bnn = wins[wn + nwt];
            held = Bn.img_bytes <= kPrefetchBlocks * kWave * 16;
            if (held) {  // (clamped indices: unconditional loads, no branch around them)
                const uint4* src = reinterpret_cast<const uint4*>(bytes + Bn.img_lo);
                const uint32_t nb = Bn.img_bytes / 16, b = lane();
                auto at = [&](uint32_t k) { return src[b + k * kWave < nb ? b + k * kWave : 0u]; };
                R0 = at(0); R1 = at(1); R2 = at(2); R3 = at(3);
                R4 = at(4); R5 = at(5); R6 = at(6); R7 = at(7);
            }
            ixn_held = ix_load(Bn, ixn01, ixn23);
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint32_t* stage = reinterpret_cast<const uint32_t*>(cur);
        if (lane() == 0) {
            hit[0] = 0;
            hit[1] = 0;
        }
        __builtin_amdgcn_wave_barrier();
        const uint32_t np = static_cast<uint32_t>(Bc.np);
        // The strings of the window's pages, as window offsets in `list`:
        // from the chunk's string index when an earlier scan built it
        // (REQUIRED chunks: string k of page p is row first_row(p) + k), else
        // by the lane-parallel walk below (which then files the index).
        const bool pl = lane() < np;
        const uint32_t mpay = static_cast<uint32_t>(pgc.off - Bc.img_lo);
        uint32_t cnt = 0, lb = mpay / 4;
        if (index_in) {
            const int64_t fr0 = static_cast<int64_t>(
                static_cast<uint64_t>(static_cast<uint32_t>(__shfl(static_cast<int>(pgc.first_row), 0))) |
                (static_cast<uint64_t>(static_cast<uint32_t>(__shfl(static_cast<int>(pgc.first_row >> 32), 0))) << 32));
            const int64_t fr = pl ? pgc.first_row : fr0;
            cnt = pl ? static_cast<uint32_t>(max(pgc.nvals, 0)) : 0u;
            lb = static_cast<uint32_t>(fr - fr0);
            const uint32_t tot = Bc.nrows;  // (= the pages' values; rows from Bc.row0 = fr0)
            if (ix_held) {
                const uint32_t v[4] = {ix01 & 0xFFFFu, ix01 >> 16, ix23 & 0xFFFFu, ix23 >> 16};
#pragma unroll
                for (uint32_t j = 0; j < 4; j++)
                    if (j * kWave + lane() < tot) list[j * kWave + lane()] = static_cast<uint16_t>(v[j]);
            } else {
                for (uint32_t k = lane(); k < tot; k += kWave) list[k] = index_in[Bc.row0 + k];
            }
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        } else {
            // ── strings: L lanes per page ───────────────────────────────────
            const uint32_t lg = np <= 1 ? 0u : 32u - __builtin_clz(np - 1);  // ceil log2
            const uint32_t L = kWave >> lg;
            const uint32_t q = lane() / L, sg = lane() % L;
            const bool act = q < np && !(dbg & 2);
            const uint32_t qs = min(q, 63u);
            const uint64_t poff = (static_cast<uint64_t>(__shfl(static_cast<int>(pgc.off >> 32), static_cast<int>(qs))) << 32) |
                                  static_cast<uint32_t>(__shfl(static_cast<int>(pgc.off), static_cast<int>(qs)));
            const uint32_t size = static_cast<uint32_t>(max(__shfl(pgc.size, static_cast<int>(qs)), 0));
            const uint32_t nvq = static_cast<uint32_t>(max(__shfl(pgc.nvals, static_cast<int>(qs)), 0));
            const uint32_t pay = static_cast<uint32_t>(poff - Bc.img_lo);
            // levels (segment 0 lanes; any problem -> the exact walk below)
            uint32_t pos0 = 0, nn = nvq;
            bool bad = false;
            if (act && sg == 0 && (cp.max_def > 0 || cp.max_rep > 0)) {
                const uint32_t* pw = reinterpret_cast<const uint32_t*>(cur + pay);
                auto rd8 = [&](uint32_t a) { return lds_u64(pw, a); };
                if (cp.max_def > 0) {
                    if (pos0 + 4 > size) bad = true;
                    else {
                        const uint32_t dl = static_cast<uint32_t>(rd8(pos0));
                        pos0 += 4;
                        if (static_cast<uint64_t>(pos0) + dl > size) bad = true;
                        else {
                            LRle r = lrle(pos0, dl, level_bw(cp.max_def));
                            const uint32_t bwd = r.bw;
                            nn = 0;
                            bad = lane_rle(r, rd8, nvq, [&](uint32_t kind, uint32_t k, uint32_t arg) {
                                if (kind == 0) {
                                    if (arg >= md) nn += k;
                                } else {
                                    for (uint32_t i = 0; i < k; i++)
                                        if (lds_bits(pw, size, static_cast<uint64_t>(arg) + i * bwd, bwd) >= md) nn++;
                                }
                            }) != 0;
                            pos0 += dl;
                        }
                    }
                }
                if (!bad && cp.max_rep > 0) {
                    if (pos0 + 4 > size) bad = true;
                    else {
                        const uint32_t rl = static_cast<uint32_t>(rd8(pos0));
                        pos0 += 4;
                        if (static_cast<uint64_t>(pos0) + rl > size) bad = true;
                        else pos0 += rl;
                    }
                }
            }
            const int src0 = static_cast<int>(q * L);
            pos0 = static_cast<uint32_t>(__shfl(static_cast<int>(pos0), src0));
            nn = static_cast<uint32_t>(__shfl(static_cast<int>(nn), src0));
            bad = __shfl(static_cast<int>(bad), src0) != 0;
            // this lane's segment of [pos0, size) and its first candidate string
            // start (a position whose u32 length fits the page), 16 positions
            // per aligned 16-byte read
            const uint32_t span = size > pos0 ? size - pos0 : 0u;
            const uint32_t lo = pos0 + static_cast<uint32_t>((static_cast<uint64_t>(span) * sg) / L);
            const uint32_t hi = sg + 1 == L ? size : pos0 + static_cast<uint32_t>((static_cast<uint64_t>(span) * (sg + 1)) / L);
            const uint32_t A = pay;  // window byte of the page's payload
            uint32_t c0 = ~0u;
            if (act && !bad) {
                if (sg == 0) {
                    c0 = pos0;
                } else {
                    // (a plausible start holds a length below 2^16, pages
                    // fitting a window of < 64 KiB: its bytes 2 and 3 are
                    // zero; only those positions are tested, in order)
                    for (uint32_t a = (A + lo) & ~15u; a < A + hi && c0 == ~0u; a += 16) {
                        const uint4 v = *reinterpret_cast<const uint4*>(cur + a);
                        const uint32_t d4 = stage[(a >> 2) + 4];
                        const uint32_t d[5] = {v.x, v.y, v.z, v.w, d4};
                        uint32_t zb = 0;  // bit j: byte a + j is zero (j < 20)
    #pragma unroll
                        for (uint32_t j = 0; j < 5; j++) {
                            const uint32_t z = ~(((d[j] & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | d[j] | 0x7F7F7F7Fu);
                            zb |= (((z >> 7) & 1u) | ((z >> 14) & 2u) | ((z >> 21) & 4u) | ((z >> 28) & 8u)) << (4 * j);
                        }
                        uint32_t cm = (zb >> 2) & (zb >> 3) & 0xFFFFu;
                        while (cm) {
                            const uint32_t k = static_cast<uint32_t>(__builtin_ctz(cm));
                            cm &= cm - 1;
                            const uint32_t cpos = a + k - A;
                            if (cpos < lo) continue;
                            if (cpos >= hi) break;
                            const uint32_t len = st_u32(stage, a + k);
                            if (cpos + 4 <= size && len <= size - cpos - 4) {
                                c0 = cpos;
                                break;
                            }
                        }
                    }
                }
            }
            // its chain to the segment end: exit position, strings, and whether a
            // read failed (at the exit)
            uint32_t ex = c0, n = 0;
            bool fail = false;
            if (act && c0 != ~0u) {
                while (ex < hi) {
                    if (ex + 4 > size) { fail = true; break; }
                    const uint32_t len = st_u32(stage, A + ex);
                    if (len > size - ex - 4) { fail = true; break; }
                    ex += 4 + len;
                    n++;
                }
            }
            // link: every segment must start where the previous one left (no
            // failed chain before the last segment); else the exact walk
            const uint32_t prev = static_cast<uint32_t>(__shfl(static_cast<int>(ex), static_cast<int>(lane()) - 1));
            const uint32_t pfail = static_cast<uint32_t>(__shfl(static_cast<int>(fail), static_cast<int>(lane()) - 1));
            const uint32_t start = c0;
            const bool mism = act && !bad && (c0 == ~0u || (sg > 0 && (pfail || prev != c0)));
            // page-local placement of each segment's strings
            const uint32_t inc = wave_incl_scan(n);
            const uint32_t pbase = static_cast<uint32_t>(__shfl(static_cast<int>(inc - n), src0));
            const uint32_t before = inc - n - pbase;
            const uint32_t last = min(src0 + L - 1, 63u);
            const uint32_t total = static_cast<uint32_t>(__shfl(static_cast<int>(inc), static_cast<int>(last))) - pbase;
            // exact walk needed: unlinked segments, a level problem, or fewer than
            // nn strings before the chain fails / the page ends
            const uint64_t mm = __ballot(act && (mism || bad));
            const uint32_t pmis = ((mm >> src0) & ((L >= 64 ? ~0ull : ((1ull << L) - 1ull)))) != 0 ? 1u : 0u;
            const bool page_ok = act && !pmis && total >= nn && !(dbg & 4);
            // emit: this segment's strings with page index < nn
            if (page_ok && start != ~0u && before < nn) {
                const uint32_t keep = min(n, nn - before);
                uint16_t* lst = list + pay / 4 + before;
                uint32_t pos = start;
                for (uint32_t i = 0; i < keep; i++) {
                    const uint32_t len = st_u32(stage, A + pos);
                    lst[i] = static_cast<uint16_t>(A + pos + 4);
                    pos += 4 + len;
                }
            }
            if (act && sg == 0) pcnt[q] = page_ok ? nn : ~0u;  // ~0: exact walk
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            // exact walk (one lane per page) where the segments did not settle it
            cnt = pl && !(dbg & 2) ? pcnt[lane()] : 0u;
            if (pl && cnt == ~0u) {
                cnt = 0;
                const uint32_t* pw = reinterpret_cast<const uint32_t*>(cur + mpay);
                auto rd8 = [&](uint32_t a) { return lds_u64(pw, a); };
                DevErr* err = page_err + Bc.p0 + static_cast<int32_t>(lane());
                const uint32_t msize = static_cast<uint32_t>(max(pgc.size, 0));
                uint32_t pos = 0, mnn = static_cast<uint32_t>(max(pgc.nvals, 0));
                int code = 0;
                uint32_t epos = 0, eneed = 0;
                if (cp.max_def > 0) {
                    if (pos + 4 > msize) { code = PQ_ERR_BUFFER; epos = pos; eneed = 4; }
                    else {
                        const uint32_t dl = static_cast<uint32_t>(rd8(pos));
                        pos += 4;
                        if (static_cast<uint64_t>(pos) + dl > msize) { code = PQ_ERR_BUFFER; epos = pos; eneed = dl; }
                        else {
                            LRle r = lrle(pos, dl, level_bw(cp.max_def));
                            const uint32_t bwd = r.bw;
                            const uint32_t nv = mnn;
                            mnn = 0;
                            code = lane_rle(r, rd8, nv, [&](uint32_t kind, uint32_t k, uint32_t arg) {
                                if (kind == 0) {
                                    if (arg >= md) mnn += k;
                                } else {
                                    for (uint32_t i = 0; i < k; i++)
                                        if (lds_bits(pw, msize, static_cast<uint64_t>(arg) + i * bwd, bwd) >= md) mnn++;
                                }
                            });
                            pos += dl;
                        }
                    }
                }
                if (!code && cp.max_rep > 0) {
                    if (pos + 4 > msize) { code = PQ_ERR_BUFFER; epos = pos; eneed = 4; }
                    else {
                        const uint32_t rl = static_cast<uint32_t>(rd8(pos));
                        pos += 4;
                        if (static_cast<uint64_t>(pos) + rl > msize) { code = PQ_ERR_BUFFER; epos = pos; eneed = rl; }
                        else pos += rl;
                    }
                }
                uint16_t* lst = list + mpay / 4;  // this page's list region (<= slot / 4 entries)
                for (uint32_t k = 0; k < mnn && !code; k++) {  // column_reader.cpp:249-253
                    if (static_cast<uint64_t>(pos) + 4 > msize) { code = PQ_ERR_BUFFER; epos = pos; eneed = 4; break; }
                    const uint32_t len = static_cast<uint32_t>(rd8(pos));
                    pos += 4;
                    if (static_cast<uint64_t>(pos) + len > msize) { code = PQ_ERR_BUFFER; epos = pos; eneed = len; break; }
                    lst[cnt++] = static_cast<uint16_t>(mpay + pos);  // window offset (the length is at offset - 4)
                    pos += len;
                }
                if (code) {
                    lane_err(err, err_any, code, epos, eneed, msize);
                    cnt = 0;
                }
            }
        }
        // the window's first row: with the index being filed (REQUIRED chunk,
        // pages of consecutive rows), string g of the window is row fr0 + g and
        // its entry is stored below, coalesced, where the DFA pass reads it
        // (a failed page files no index: collect() drops it)
        const int64_t fr0 = static_cast<int64_t>(
            static_cast<uint64_t>(static_cast<uint32_t>(__shfl(static_cast<int>(pgc.first_row), 0))) |
            (static_cast<uint64_t>(static_cast<uint32_t>(__shfl(static_cast<int>(pgc.first_row >> 32), 0))) << 32));
        uint16_t* const idx_w = index_in ? nullptr : index_out;
        // flatten: string g of the window -> (page lane, k)
        const uint32_t pinc = wave_incl_scan(cnt);
        pref[lane()] = pinc;
        lbase[lane()] = lb;
        const uint32_t wtotal = bcast_last(pinc);
        __builtin_amdgcn_wave_barrier();
        const uint64_t sinks = kSink && full ? (static_cast<uint64_t>(D->sink_hi) << 32) | D->sink_lo : 0ull;
        for (uint32_t g0 = 0; g0 < ((dbg & 1) ? 0u : wtotal); g0 += kStrPerLane * kWave) {
            uint32_t e2[kStrPerLane], off2[kStrPerLane], len2[kStrPerLane], pg2[kStrPerLane];
            bool ok2[kStrPerLane];
#pragma unroll
            for (uint32_t h = 0; h < kStrPerLane; h++) {
                const uint32_t g = g0 + h * kWave + lane();
                ok2[h] = g < wtotal;
                // first page lane whose inclusive count exceeds g
                uint32_t lo2 = 0;
#pragma unroll
                for (uint32_t stp = 32; stp >= 1; stp >>= 1)
                    if (pref[lo2 + stp - 1] <= g) lo2 += stp;
                const uint32_t gl = ok2[h] ? lo2 : 0u;
                const uint32_t bef = gl ? pref[gl - 1] : 0u;
                const uint32_t ent = ok2[h] ? list[lbase[gl] + (g - bef)] : 4u;
                if (idx_w && ok2[h]) idx_w[fr0 + g] = static_cast<uint16_t>(ent);
                off2[h] = ent;
                len2[h] = ok2[h] ? st_u32(stage, ent - 4) : 0u;
                pg2[h] = gl;
                e2[h] = DFA_START;
            }
            uint32_t maxl = 0;
#pragma unroll
            for (uint32_t h = 0; h < kStrPerLane; h++) maxl = max(maxl, len2[h]);
            for (uint32_t b0 = 0; __ballot(maxl > b0); b0 += 16) {
                // after the first block: stop when every longer string sits in
                // an absorbing state (an anchored pattern's DEAD); one test per
                // batch, as a test per block costs more than it saves
                if (kSink && b0 == 16) {
                    bool live = false;
#pragma unroll
                    for (uint32_t h = 0; h < kStrPerLane; h++) live |= len2[h] > 16 && !((sinks >> (e2[h] & 63u)) & 1u);
                    if (!__ballot(live)) break;
                }
                uint32_t Aw[kStrPerLane][4], rem[kStrPerLane];
#pragma unroll
                for (uint32_t h = 0; h < kStrPerLane; h++) {
                    const uint32_t a = off2[h] + b0;
                    const uint32_t i0 = a >> 2, sh = a & 3;
                    uint32_t d[5];
#pragma unroll
                    for (uint32_t j = 0; j < 5; j++) d[j] = stage[i0 + j];
#pragma unroll
                    for (uint32_t j = 0; j < 4; j++) Aw[h][j] = __builtin_amdgcn_alignbyte(d[j + 1], d[j], sh);
                    rem[h] = len2[h] > b0 ? len2[h] - b0 : 0u;
                }
                // the chains advance one byte each per step, interleaved
                if (full) {
#pragma unroll
                    for (uint32_t i = 0; i < 16; i++) {
#pragma unroll
                        for (uint32_t h = 0; h < kStrPerLane; h++) {
                            // address = state << 8 | byte i of the block (one v_perm)
                            const uint32_t a = __builtin_amdgcn_perm(e2[h], Aw[h][i >> 2], 0x0C0C0400u | (i & 3));
                            const uint32_t t = T8c[a];
                            e2[h] = sel_below(i, rem[h], t, e2[h]);
                        }
                    }
                } else {
#pragma unroll
                    for (uint32_t i = 0; i < 16; i++) {
#pragma unroll
                        for (uint32_t h = 0; h < kStrPerLane; h++) {
                            const uint32_t bt = (Aw[h][i >> 2] >> (8 * (i & 3))) & 0xFFu;
                            const uint32_t t = T[(e2[h] & 0x7FFFu) * nc + D->cls_of[bt]];
                            e2[h] = i < rem[h] ? t : e2[h];
                        }
                    }
                }
            }
#pragma unroll
            for (uint32_t h = 0; h < kStrPerLane; h++) {
                const uint32_t e = e2[h];
                const uint32_t st = full ? e : (e & 0x7FFFu);
                const bool acc = full ? A8[e] != 0 : (e >> 15) != 0;
                const bool m = len2[h] == 0 ? empty_ok : (trivial || st == DFA_ACCEPT || acc);
                const bool sat = ok2[h] && (static_cast<uint32_t>(m) != negv);
                if (sat) atomicOr(&hit[pg2[h] >> 5], 1u << (pg2[h] & 31));
            }
        }
        __builtin_amdgcn_wave_barrier();
        pf_on = pl;
        pf_at = Bc.p0 + static_cast<int32_t>(lane());
        pf_v = ((hit[lane() >> 5] >> (lane() & 31)) & 1u) ? 0 : 1;
        __builtin_amdgcn_wave_barrier();
        if (wn >= nwins) break;
        // the next window -> LDS (this one's DFA pass is done with `cur`)
        if (held) {
            const uint32_t nb = Bn.img_bytes / 16;
            uint4* dst = reinterpret_cast<uint4*>(cur);
            const uint32_t b = lane();
            if (b < nb) dst[b] = R0;
            if (b + 1 * kWave < nb) dst[b + 1 * kWave] = R1;
            if (b + 2 * kWave < nb) dst[b + 2 * kWave] = R2;
            if (b + 3 * kWave < nb) dst[b + 3 * kWave] = R3;
            if (b + 4 * kWave < nb) dst[b + 4 * kWave] = R4;
            if (b + 5 * kWave < nb) dst[b + 5 * kWave] = R5;
            if (b + 6 * kWave < nb) dst[b + 6 * kWave] = R6;
            if (b + 7 * kWave < nb) dst[b + 7 * kWave] = R7;
        } else {
            copy_blocks(reinterpret_cast<uint4*>(cur), reinterpret_cast<const uint4*>(bytes + Bn.img_lo), Bn.img_bytes / 16,
                        lane(), kWave);
        }
        if (lane() < 2) reinterpret_cast<uint4*>(cur + Bn.img_bytes)[lane()] = make_uint4(0, 0, 0, 0);
        B = Bn;
        Bn = Bnn;
        pg = pgn;
        w = wn;
        ix01 = ixn01;
        ix23 = ixn23;
        ix_held = ixn_held;
    }
    if (pf_on) page_flags[pf_at] = pf_v;
}

}  // namespace

DeviceProgram* upload_program(const Program& p, hipStream_t s) {
    DevProg h;
    build_dev(p, &h);
    auto* dp = new DeviceProgram{nullptr};
    if (hipMalloc(reinterpret_cast<void**>(&dp->d), sizeof(DevProg)) != hipSuccess) {
        delete dp;
        return nullptr;
    }
    if (hipMemcpyAsync(dp->d, &h, sizeof h, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess) {
        (void)hipFree(dp->d);
        delete dp;
        return nullptr;
    }
    return dp;
}

void free_device_program(DeviceProgram* p) {
    if (!p) return;
    if (p->d) (void)hipFree(p->d);
    delete p;
}

void launch_regex_dict(hipStream_t s, const DeviceProgram* prog, const uint8_t* bytes,
                       const DevDict* dicts, int ndicts, const uint64_t* entries,
                       const int32_t* dict_count, uint8_t* dict_match, uint8_t* fill1, int64_t nfill1,
                       uint32_t* zero, int64_t nzero) {
    if (ndicts <= 0) return;
    hipLaunchKernelGGL(k_regex_dict, dim3(ndicts, 16), dim3(256), 0, s, prog->d, bytes, dicts, entries,
                       dict_count, dict_match, fill1, nfill1, zero, nzero);
}

void launch_regex_lanes(hipStream_t s, const uint8_t* dfa, uint32_t dfa_bytes, const uint8_t* bytes,
                        const DevPage* pages, int npages, const DevDict* dicts, const int32_t* dict_count,
                        const uint8_t* dict_match, ColumnParams cp, int neg, uint8_t* page_flags,
                        DevErr* page_err, int32_t* err_any) {
    if (npages <= 0) return;
    pqk::ensure_dyn_lds(reinterpret_cast<const void*>(k_regex_lanes), kDfaMaxBytes);
    const int blocks = (npages + 255) / 256;
    hipLaunchKernelGGL(k_regex_lanes, dim3(blocks), dim3(256), dfa_bytes, s, dfa, dfa_bytes, bytes, pages, npages,
                       dicts, dict_count, dict_match, cp, neg, page_flags, page_err, err_any);
}

uint32_t regex_plain_waves(uint32_t dfa_bytes, uint32_t win_bytes) {
    const uint32_t per = regex_plain_wave_lds(win_bytes);
    if (dfa_bytes + per > 160u * 1024) return 0;
    return std::min<uint32_t>(kPlainWavesMax, (160u * 1024 - dfa_bytes) / per);
}

uint32_t regex_plain_lds(uint32_t dfa_bytes, uint32_t win_bytes) {
    return dfa_bytes + regex_plain_waves(dfa_bytes, win_bytes) * regex_plain_wave_lds(win_bytes);
}

void launch_regex_plain(hipStream_t s, const uint8_t* dfa, uint32_t dfa_bytes, uint32_t win_bytes,
                        const uint8_t* bytes, const DevPage* pages, const pqk::DevBatch* wins, int nwins,
                        int32_t* ticket, int grid, ColumnParams cp, int neg, uint8_t* page_flags,
                        DevErr* page_err, int32_t* err_any, const uint16_t* index_in, uint16_t* index_out, bool sink) {
    if (nwins <= 0) return;
    void (*fn)(const uint8_t*, uint32_t, uint32_t, const uint8_t*, const DevPage*, const pqk::DevBatch*, int, int32_t*,
               ColumnParams, int, uint8_t*, DevErr*, int32_t*, const uint16_t*, uint16_t*) =
        sink ? k_regex_plain<true> : k_regex_plain<false>;
    pqk::ensure_dyn_lds(reinterpret_cast<const void*>(fn), 160 * 1024);
    hipLaunchKernelGGL(fn, dim3(grid), dim3(regex_plain_waves(dfa_bytes, win_bytes) * kWave),
                       regex_plain_lds(dfa_bytes, win_bytes), s, dfa, dfa_bytes, win_bytes, bytes, pages, wins, nwins, ticket,
                       cp, neg, page_flags, page_err, err_any, index_in, index_out);
}

// k_regex_plain reads its byte-state table through a constant LDS address
// (T8c): that holds only while the kernel has no static LDS, so that the
// dynamic block dsm starts at LDS address 0.  Checked once from the code
// object's own attributes; when it fails the caller takes k_regex_lanes.
bool regex_plain_lds_ok() {
    static const bool ok = [] {
        hipFuncAttributes a{};
        for (const void* k : {reinterpret_cast<const void*>(k_regex_plain<true>), reinterpret_cast<const void*>(k_regex_plain<false>)})
            if (hipFuncGetAttributes(&a, k) != hipSuccess || a.sharedSizeBytes != 0) return false;
        return true;
    }();
    return ok;
}

int regex_plain_occupancy(uint32_t lds) {  // the LDS sets it: one workgroup of regex_plain_waves waves per CU
    return lds <= 160u * 1024 ? 1 : 0;
}

void launch_regex_pages(hipStream_t s, const DeviceProgram* prog, const uint8_t* bytes,
                        const DevPage* pages, int npages, const DevDict* dicts,
                        const uint64_t* entries, const int32_t* dict_count,
                        const uint8_t* dict_match, ColumnParams cp, int neg, uint8_t* page_flags,
                        DevErr* page_err, int32_t* err_any) {
    if (npages <= 0) return;
    int blocks = (npages + kWavesPerBlock - 1) / kWavesPerBlock;
    hipLaunchKernelGGL(k_regex_pages, dim3(blocks), dim3(256), 0, s, prog->d, bytes, pages, npages,
                       dicts, entries, dict_count, dict_match, cp, neg, page_flags, page_err,
                       err_any);
}

}  // namespace pqre
