// fixed_fast.hip — tile-parallel PLAIN fixed-width decode (SURVEY §8a R-PLAIN,
// R-LEVELS) for INT32 / INT64 / FLOAT / DOUBLE / INT96 chunks whose data
// pages are all PLAIN.
//
// decode.hip's k_fixed gives each page one wavefront that walks its 512-row
// tiles in order; arrow-layout pages hold 20k rows, so a 10M-row chunk is
// only 500 wavefronts.  Here the work is split by tile:
//   k_fixed_req      REQUIRED columns: every tile copies its rows' bytes
//                    straight from the page (column_reader.cpp:241-248 is a
//                    memcpy per value) with 16-byte loads/stores, and sets its
//                    validity bits.
//   k_fixed_levels   OPTIONAL columns, one wavefront per page: the def-level
//                    stream (exact scalar walk, stream.hpp) -> validity bits
//                    of the page's rows, per-tile ranks of the first non-null
//                    row, and the PLAIN bounds check (ByteBuffer::check on the
//                    first rank whose read overruns, after all levels, as the
//                    reference orders it).
//   k_fixed_scatter  OPTIONAL columns, one wavefront per tile: row -> rank by
//                    a popcount prefix of the validity bits, value bytes from
//                    pos + rank * width; NULL rows are zero.
#include "kernels/device_common.hpp"
#include "kernels/kernels.hpp"
#include "kernels/lane_walk.hpp"
#include "kernels/run_walk.hpp"
#include "kernels/run_spec.hpp"
#include "kernels/stream.hpp"
#include "pq_gpu.h"

namespace pqk {
namespace {

using namespace dev;

constexpr int kTilesPerBlock = 4;
constexpr uint32_t kLitCapF = 16;

// Validity bits of rows [R, R + cnt) (cnt <= 64) from a 64-bit lane ballot
// `vm` (bit j = row R + j); words fully inside [lo_row, hi_row) are stored,
// others ORed (a neighbouring page or tile owns their other bits).
__device__ __forceinline__ void put_valid64(uint32_t* validity, int64_t R, uint32_t cnt, uint64_t vm,
                                            int64_t lo_row, int64_t hi_row) {
    const uint32_t wi = static_cast<uint32_t>(R >> 5), sh = static_cast<uint32_t>(R & 31);
    if (lane() < 3) {
        const uint32_t part = lane() == 0 ? static_cast<uint32_t>(vm << sh)
                            : lane() == 1 ? static_cast<uint32_t>(sh ? (vm >> (32 - sh)) : (vm >> 32))
                                          : (sh ? static_cast<uint32_t>(vm >> (64 - sh)) : 0u);
        const int64_t wlo = static_cast<int64_t>(wi + lane()) * 32;
        const int64_t rhi = R + cnt;
        const bool full = wlo >= lo_row && wlo + 32 <= hi_row && wlo >= R && wlo + 32 <= rhi;
        if (wlo < rhi && wlo + 32 > R) {
            if (full) validity[wi + lane()] = part;
            else if (part) atomicOr(&validity[wi + lane()], part);
        }
    }
}

__global__ void __launch_bounds__(256) k_fixed_req(const uint8_t* __restrict__ bytes, const DevPage* __restrict__ pages,
                                                   const DevTile* __restrict__ tiles, int ntiles, uint32_t pw,
                                                   uint32_t* __restrict__ validity, uint8_t* __restrict__ values,
                                                   DevErr* __restrict__ page_err, int32_t* __restrict__ err_any) {
    const int t = blockIdx.x * kTilesPerBlock + static_cast<int>(threadIdx.x / kWave);
    if (t >= ntiles) return;
    const DevTile T = tiles[t];
    const DevPage pg = pages[T.page];
    const uint32_t size = static_cast<uint32_t>(pg.size);
    const uint32_t r0 = static_cast<uint32_t>(T.row0), m = static_cast<uint32_t>(T.nrows);
    // ByteBuffer::check (common.hpp:162-168): the first rank whose read
    // overruns the page; its tile reports it, no tile copies past it
    const uint64_t need = static_cast<uint64_t>(max(pg.nvals, 0)) * pw;
    uint32_t mc = m;
    if (need > size) {
        const uint32_t k = size / pw;
        if (k >= r0 && k < r0 + m) set_err(page_err + T.page, err_any, PQ_ERR_BUFFER, k * pw, pw, size);
        mc = k > r0 ? min(m, k - r0) : 0u;
    }
    const int64_t R0 = pg.first_row + r0;
    const uint8_t* src = bytes + pg.off + static_cast<uint64_t>(r0) * pw;
    uint8_t* dst = values + static_cast<uint64_t>(R0) * pw;
    const uint32_t nbytes = mc * pw;
    if (((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15) == 0) {
        const uint4* s4 = reinterpret_cast<const uint4*>(src);
        uint4* d4 = reinterpret_cast<uint4*>(dst);
        const uint32_t n16 = nbytes / 16;
        for (uint32_t i = lane(); i < n16; i += kWave) d4[i] = s4[i];
        for (uint32_t i = n16 * 4 + lane(); i < nbytes / 4; i += kWave)
            reinterpret_cast<uint32_t*>(dst)[i] = reinterpret_cast<const uint32_t*>(src)[i];
    } else {
        for (uint32_t i = lane(); i < nbytes / 4; i += kWave)
            reinterpret_cast<uint32_t*>(dst)[i] = reinterpret_cast<const uint32_t*>(src)[i];
    }
    for (uint32_t j0 = 0; j0 < m; j0 += kWave) {
        const uint32_t cnt = min(64u, m - j0);
        put_valid64(validity, R0 + j0, cnt, __ballot(lane() < cnt), R0, R0 + m);
    }
}

// Exact serial form, one wavefront per page (pages the run-table form does
// not take).  tile_rank[t] = non-null rows of the page before tile t;
// page_pos[p] = the byte where the page's values start.
__device__ void levels_serial(const uint8_t* __restrict__ bytes, const DevPage* __restrict__ pages, int p,
                              const int32_t* __restrict__ page_tile0, ColumnParams cp,
                              uint32_t* __restrict__ validity, int32_t* __restrict__ tile_rank,
                              int32_t* __restrict__ page_pos, int32_t* __restrict__ page_nn,
                              DevErr* __restrict__ page_err, int32_t* __restrict__ err_any, LitRun* lits,
                              uint32_t* bits) {
    const DevPage pg = pages[p];
    const uint8_t* page = bytes + pg.off;
    const uint32_t size = static_cast<uint32_t>(pg.size);
    const uint32_t n = static_cast<uint32_t>(max(pg.nvals, 0));
    DevErr* err = page_err + p;
    const uint32_t md = static_cast<uint32_t>(cp.max_def);
    uint32_t pos = 0;
    // levels (column_reader.cpp:146-170)
    const bool has_def = cp.max_def > 0;
    SRle def;
    srle_init(def, 0, 0, 0);
    if (has_def) {
        if (pos + 4 > size) { set_err(err, err_any, PQ_ERR_BUFFER, pos, 4, size); return; }
        const uint32_t dl = suni(sload_u32(page, pos));
        pos += 4;
        if (static_cast<uint64_t>(pos) + dl > size) { set_err(err, err_any, PQ_ERR_BUFFER, pos, dl, size); return; }
        srle_init(def, pos, dl, level_bw(cp.max_def));
        pos += dl;
    }
    if (cp.max_rep > 0) {
        if (pos + 4 > size) { set_err(err, err_any, PQ_ERR_BUFFER, pos, 4, size); return; }
        const uint32_t rl = suni(sload_u32(page, pos));
        pos += 4;
        if (static_cast<uint64_t>(pos) + rl > size) { set_err(err, err_any, PQ_ERR_BUFFER, pos, rl, size); return; }
        pos += rl;
    }
    // def levels, one 512-row tile at a time (the walk state carries over)
    const int32_t t0 = page_tile0[p];
    uint32_t nn = 0;
    for (uint32_t r0 = 0; r0 < n; r0 += kTileRows) {
        const uint32_t m = min(n - r0, static_cast<uint32_t>(kTileRows));
        for (uint32_t w = lane(); w < kTileRows / 32; w += kWave) bits[w] = has_def ? 0u : ~0u;
        __builtin_amdgcn_wave_barrier();
        auto put = [&](uint32_t j, uint32_t v) {
            if (v >= md) atomicOr(&bits[j >> 5], 1u << (j & 31));
        };
        uint32_t nl = 0;
        const int rc = !has_def ? 0 : srle_walk(def, page, m, put, lits, nl, kLitCapF, [&]() {
            __builtin_amdgcn_wave_barrier();
            for (uint32_t r = 0; r < nl; r++) {
                const LitRun L = lits[r];
                const uint64_t b0 = (static_cast<uint64_t>(L.bit0_hi) << 32) | L.bit0_lo;
                for (uint32_t j = lane(); j < L.count; j += kWave) put(L.start + j, gbits(page, size, b0 + static_cast<uint64_t>(j) * def.bw, def.bw));
            }
            __builtin_amdgcn_wave_barrier();
        });
        if (rc) { set_err(err, err_any, rc, 0, 0, size); return; }
        __builtin_amdgcn_wave_barrier();
        for (uint32_t r = 0; r < nl; r++) {
            const LitRun L = lits[r];
            const uint64_t b0 = (static_cast<uint64_t>(L.bit0_hi) << 32) | L.bit0_lo;
            for (uint32_t j = lane(); j < L.count; j += kWave) put(L.start + j, gbits(page, size, b0 + static_cast<uint64_t>(j) * def.bw, def.bw));
        }
        __builtin_amdgcn_wave_barrier();
        if (lane() == 0) tile_rank[t0 + static_cast<int32_t>(r0 / kTileRows)] = static_cast<int32_t>(nn);
        const int64_t R0 = pg.first_row + r0;
        for (uint32_t j0 = 0; j0 < m; j0 += kWave) {
            const uint32_t j = j0 + lane();
            const bool v = j < m && ((bits[j >> 5] >> (j & 31)) & 1u);
            const uint64_t vm = __ballot(v);
            nn += __popcll(vm);
            put_valid64(validity, R0 + j0, min(64u, m - j0), vm, pg.first_row, pg.first_row + n);
        }
        __builtin_amdgcn_wave_barrier();
    }
    // values: ByteBuffer::check on the first overrunning rank
    const uint32_t w = static_cast<uint32_t>(cp.plain_width);
    if (static_cast<uint64_t>(pos) + static_cast<uint64_t>(nn) * w > size) {
        const uint32_t k = (size - pos) / w;
        set_err(err, err_any, PQ_ERR_BUFFER, pos + k * w, w, size);
    }
    if (lane() == 0) page_pos[p] = static_cast<int32_t>(pos);
    if (lane() == 0 && page_nn) page_nn[p] = static_cast<int32_t>(nn);
}

// The page's tiles scattered by the workgroup that decoded its levels (its
// validity words, tile ranks and value start are in HBM; the barrier orders
// them).  Nothing is read past a page whose values overrun it.
__device__ __forceinline__ void fused_scatter(const uint8_t* __restrict__ bytes, const DevPage* __restrict__ pages, int p,
                                              const int32_t* __restrict__ page_tile0, const DevTile* __restrict__ tiles,
                                              ColumnParams cp, const uint32_t* validity, const int32_t* tile_rank,
                                              const int32_t* page_pos, const DevErr* page_err,
                                              uint8_t* __restrict__ values);

// One workgroup (8 waves) per page: the page's level bytes staged in LDS,
// one lane walks the def stream into an LDS run table (run_walk.hpp), then
// the waves expand 512-row tiles in parallel (max-scan over run starts, rows
// 8l .. 8l + 7 per lane) into validity words and per-tile non-null counts.
// Pages outside that shape (long level sections, > kLvRec runs, zero-count
// runs, ...) take levels_serial on wave 0.
constexpr int kLvWaves = 8;
constexpr uint32_t kLvStage = 16384;
constexpr uint32_t kLvRec = 4096;
constexpr uint32_t kLvStageS = 8192;
constexpr uint32_t kLvRecS = 2048;
constexpr uint32_t kLvTiles = 128;
constexpr uint32_t kLvSpecMax = 4096;  // level sections up to this size: run_spec.hpp (workgroup) instead of one lane
constexpr uint32_t kLvSpecList = kLvSpecMax / 2 / kSpJump + 8;

// kScatter: the PLAIN fixed-width values too (k_fixed_scatter's work for the
// page's tiles, after its levels), one launch instead of two.  kStage / kRec:
// LDS bytes for the level section and run records (the small form, 8 KiB /
// 2,048 runs, ~35 KB per workgroup, fits four workgroups per CU instead of two;
// longer sections or more runs take the serial form).
template <bool kScatter, uint32_t kStage = kLvStage, uint32_t kRec = kLvRec>
__global__ void __launch_bounds__(kLvWaves * 64) k_fixed_levels2(const uint8_t* __restrict__ bytes,
                                                                const DevPage* __restrict__ pages,
                                                                const int32_t* __restrict__ page_tile0,
                                                                ColumnParams cp, uint32_t* __restrict__ validity,
                                                                int32_t* __restrict__ tile_rank,
                                                                int32_t* __restrict__ page_pos,
                                                                int32_t* __restrict__ page_nn,
                                                                DevErr* __restrict__ page_err,
                                                                int32_t* __restrict__ err_any,
                                                                const DevTile* __restrict__ tiles,
                                                                uint8_t* __restrict__ values) {
    __shared__ __attribute__((aligned(16))) uint32_t stage[kStage / 4 + 8];
    __shared__ uint2 rec[kRec];
    __shared__ __attribute__((aligned(16))) uint16_t mark_all[kLvWaves][kTileRows];
    __shared__ uint8_t vb_all[kLvWaves][kWave];
    __shared__ uint32_t tnn[kLvTiles];
    __shared__ uint32_t sh[4];  // status, nrec, pos
    __shared__ LitRun lits[kLitCapF];
    __shared__ uint32_t splist[kLvSpecList], spesum[kLvSpecList], ssh[4];
    const int wv = static_cast<int>(threadIdx.x / kWave);
    const int p = blockIdx.x;
    const DevPage pg = pages[p];
    const uint8_t* page = bytes + pg.off;
    const uint32_t size = static_cast<uint32_t>(max(pg.size, 0));
    const uint32_t n = static_cast<uint32_t>(max(pg.nvals, 0));
    const uint32_t md = static_cast<uint32_t>(cp.max_def), bw = level_bw(cp.max_def);
    if (wv == 0) {  // prologue (column_reader.cpp:146-164): 0 ok, 1 serial form, 2 error
        uint32_t st = 0, pos = 0, dlen = 0;
        if (cp.max_def == 0) st = 1;  // repetition levels only: the serial form
        else if (pos + 4 > size) { set_err(page_err + p, err_any, PQ_ERR_BUFFER, pos, 4, size); st = 2; }
        else {
            dlen = static_cast<uint32_t>(gld8(page, 0));
            pos = 4;
            if (static_cast<uint64_t>(pos) + dlen > size) { set_err(page_err + p, err_any, PQ_ERR_BUFFER, pos, dlen, size); st = 2; }
            else pos += dlen;
        }
        if (!st && cp.max_rep > 0) {
            if (pos + 4 > size) { set_err(page_err + p, err_any, PQ_ERR_BUFFER, pos, 4, size); st = 2; }
            else {
                const uint32_t rl = static_cast<uint32_t>(gld8(page, pos));
                pos += 4;
                if (static_cast<uint64_t>(pos) + rl > size) { set_err(page_err + p, err_any, PQ_ERR_BUFFER, pos, rl, size); st = 2; }
                else pos += rl;
            }
        }
        if (!st && (n > 65535u || 4 + dlen + 16 > kStage || n > kLvTiles * kTileRows)) st = 1;
        if (lane() == 0) { sh[0] = st; sh[1] = 0; sh[2] = pos; sh[3] = dlen; }
    }
    __syncthreads();
    if (sh[0] == 2) return;
    const uint32_t dlen = sh[3];
    if (sh[0] == 0) {  // level bytes -> LDS
        const uint4* src = reinterpret_cast<const uint4*>(page);
        uint4* dst = reinterpret_cast<uint4*>(stage);
        const uint32_t nb = (4 + dlen + 15) / 16 + 1;
        copy_blocks(dst, src, nb, threadIdx.x, blockDim.x);
    }
    __syncthreads();
    static_assert(sizeof(mark_all) >= 2 * kLvSpecMax, "jump table in mark_all");
    if (sh[0] == 0 && dlen <= kLvSpecMax) {  // the run table by the workgroup (run_spec.hpp)
        const uint32_t nr = spec_runs<kLvWaves * kWave, kLvSpecMax / (kLvWaves * kWave)>(
            stage, 4, dlen, bw, n, &mark_all[0][0], splist, spesum, kLvSpecList, rec, kRec, ssh);
        if (threadIdx.x == 0) {
            if (nr == ~0u) sh[0] = 1;
            else sh[1] = nr;
        }
    } else if (sh[0] == 0 && wv == 0) {
        RunWalk W{};
        W.alive = lane() == 0;
        W.q = 4;
        W.end = 4 + dlen;
        W.bw = bw;
        W.n = n;
        W.sbase = 0;
        W.cap = kRec;
        W.out = rec;
        W.gp = page;
        uint32_t flag = 0, nrec = 0;
        walk_runs<true>(W, stage, flag, nrec);
        if (lane() == 0) { sh[1] = nrec; if (flag) sh[0] = 1; }
    }
    __syncthreads();
    if (sh[0] == 1) {
        if (wv == 0)
            levels_serial(bytes, pages, p, page_tile0, cp, validity, tile_rank, page_pos, page_nn, page_err, err_any,
                          lits, reinterpret_cast<uint32_t*>(mark_all[1]));
        if (kScatter) fused_scatter(bytes, pages, p, page_tile0, tiles, cp, validity, tile_rank, page_pos, page_err, values);
        return;
    }
    const uint32_t nrec = sh[1];
    const uint32_t staged_bytes = 4 + dlen + 16;
    auto bits = [&](uint64_t b) -> uint32_t {
        return (b >> 3) + 8 < staged_bytes ? lds_bits(stage, staged_bytes, b, bw) : gbits(page, size, b, bw);
    };
    uint16_t* mark = mark_all[wv];
    const uint32_t ntiles = (n + kTileRows - 1) / kTileRows;
    for (uint32_t ti = static_cast<uint32_t>(wv); ti < ntiles; ti += kLvWaves) {
        const uint32_t r0 = ti * kTileRows, m = min(n - r0, static_cast<uint32_t>(kTileRows));
        // first run covering r0
        uint32_t c = 0;
        for (uint32_t k0 = 0; k0 < nrec; k0 += kWave) {
            const uint32_t k = k0 + lane();
            c += __popcll(__ballot(k < nrec && (rec[k].x & 0xFFFFu) <= r0));
        }
        const uint32_t rd0 = c - 1;
        const uint32_t l8 = lane() * 8;
        if (l8 < m) *reinterpret_cast<uint4*>(mark + l8) = make_uint4(0u, 0u, 0u, 0u);
        __builtin_amdgcn_wave_barrier();
        for (uint32_t k = rd0 + 1 + lane(); k < nrec; k += kWave) {
            const uint32_t st = rec[k].x & 0xFFFFu;
            if (st >= r0 + m) break;
            mark[st - r0] = static_cast<uint16_t>(k - rd0);
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        const uint4 mk = l8 < m ? *reinterpret_cast<const uint4*>(mark + l8) : make_uint4(0u, 0u, 0u, 0u);
        const uint32_t mw[4] = {mk.x, mk.y, mk.z, mk.w};
        uint32_t rm[8], run = 0;
#pragma unroll
        for (int k = 0; k < 8; k++) {
            run = max(run, (mw[k >> 1] >> (16 * (k & 1))) & 0xFFFFu);
            rm[k] = run;
        }
        const uint32_t ex = static_cast<uint32_t>(
            __builtin_amdgcn_update_dpp(0, static_cast<int>(wave_incl_max(run)), 0x138, 0xf, 0xf, true));
        uint32_t vb = 0;
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const uint32_t j = l8 + k;
            if (j < m) {
                const uint2 R = rec[rd0 + max(ex, rm[k])];
                uint32_t lvl = R.y & 0x7FFFFFFFu;
                if (R.y >> 31) lvl = bits((R.y & 0x7FFFFFFFu) + static_cast<uint64_t>(r0 + j - (R.x & 0xFFFFu)) * bw);
                vb |= (lvl >= md ? 1u : 0u) << k;
            }
        }
        // validity words of rows [R0, R0 + m): tile word t = vb bytes 4t .. 4t + 3
        vb_all[wv][lane()] = static_cast<uint8_t>(vb);
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        const int64_t R0 = pg.first_row + r0;
        const int64_t gfirst = R0 >> 5, glast = (R0 + m - 1) >> 5;
        const uint32_t shf = static_cast<uint32_t>(R0 & 31);
        const int64_t g = gfirst + lane();
        if (g <= glast) {
            auto tw = [&](int t) -> uint32_t {
                return (t >= 0 && t < kWave / 4) ? reinterpret_cast<const uint32_t*>(vb_all[wv])[t] : 0u;
            };
            const int t = static_cast<int>(lane());
            const uint32_t val = (tw(t) << shf) | (shf ? (tw(t - 1) >> (32 - shf)) : 0u);
            const int64_t plo = pg.first_row, phi = pg.first_row + n;
            const bool whole = g * 32 >= plo && g * 32 + 32 <= phi && g * 32 >= R0 && g * 32 + 32 <= R0 + m;
            if (whole) validity[g] = val;
            else if (val) atomicOr(&validity[g], val);
        }
        const uint32_t nn = bcast_last(wave_incl_scan(__popc(vb)));
        if (lane() == 0) tnn[ti] = nn;
        __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    if (wv == 0) {  // tile ranks, value start, PLAIN bounds check (ByteBuffer::check)
        uint32_t carry = 0;
        const int32_t t0 = page_tile0[p];
        for (uint32_t i0 = 0; i0 < ntiles; i0 += kWave) {
            const uint32_t i = i0 + lane();
            const uint32_t v = i < ntiles ? tnn[i] : 0u;
            const uint32_t inc = wave_incl_scan(v);
            if (i < ntiles) tile_rank[t0 + static_cast<int32_t>(i)] = static_cast<int32_t>(carry + inc - v);
            carry += bcast_last(inc);
        }
        const uint32_t pos = sh[2];
        const uint32_t w = static_cast<uint32_t>(cp.plain_width);
        if (static_cast<uint64_t>(pos) + static_cast<uint64_t>(carry) * w > size) {
            const uint32_t k = (size - pos) / w;
            set_err(page_err + p, err_any, PQ_ERR_BUFFER, pos + k * w, w, size);
        }
        if (lane() == 0) page_pos[p] = static_cast<int32_t>(pos);
        if (lane() == 0 && page_nn) page_nn[p] = static_cast<int32_t>(carry);
    }
    if (kScatter) fused_scatter(bytes, pages, p, page_tile0, tiles, cp, validity, tile_rank, page_pos, page_err, values);
}

// Tile t's rows: NULL rows zero, row j of rank k copies value k of the page
// (k_fixed_scatter, and the fused tail of k_fixed_levels2<.., true>).
__device__ __forceinline__ void scatter_tile(const uint8_t* __restrict__ bytes, const DevPage* __restrict__ pages,
                                             const DevTile& T, uint32_t pw, const uint32_t* __restrict__ validity_in,
                                             uint32_t rank, uint32_t pos, uint8_t* __restrict__ values) {
    const DevPage pg = pages[T.page];
    const uint8_t* src = bytes + pg.off + pos;
    const uint32_t m = static_cast<uint32_t>(T.nrows);
    const int64_t R0 = pg.first_row + T.row0;
    if ((pw == 8 || pw == 4) && m <= kTileRows) {
        // the tile's validity words in one load (lane i: word i), every row
        // group's ranks from shuffled words, then all value loads in flight
        // before any store: two memory latencies per tile, not two per 64 rows
        const int64_t wfirst = R0 >> 5, wlast = (R0 + m - 1) >> 5;
        const uint32_t sh = static_cast<uint32_t>(R0 & 31);
        const uint32_t myw = wfirst + lane() <= wlast ? validity_in[wfirst + lane()] : 0u;
        constexpr uint32_t kU = kTileRows / kWave;
        uint2 x[kU];
#pragma unroll
        for (uint32_t u = 0; u < kU; u++) {
            const uint32_t j = u * kWave + lane();
            const uint32_t b = sh + j;
            const uint32_t wd = static_cast<uint32_t>(__shfl(static_cast<int>(myw), static_cast<int>(min(b >> 5, 63u))));
            const bool v = j < m && ((wd >> (b & 31)) & 1u);
            const uint64_t vm = __ballot(v);
            const uint32_t k = rank + popc_below(vm);
            rank += __popcll(vm);
            x[u] = make_uint2(0u, 0u);
            if (v) {
                if (pw == 8) x[u] = *reinterpret_cast<const uint2*>(src + static_cast<uint64_t>(k) * 8);
                else x[u].x = *reinterpret_cast<const uint32_t*>(src + static_cast<uint64_t>(k) * 4);
            }
        }
#pragma unroll
        for (uint32_t u = 0; u < kU; u++) {
            const uint32_t j = u * kWave + lane();
            if (j < m) {
                uint8_t* o = values + static_cast<uint64_t>(R0 + j) * pw;
                if (pw == 8) *reinterpret_cast<uint2*>(o) = x[u];
                else *reinterpret_cast<uint32_t*>(o) = x[u].x;
            }
        }
        return;
    }
    for (uint32_t j0 = 0; j0 < m; j0 += kWave) {
        const uint32_t j = j0 + lane();
        const int64_t R = R0 + j;
        const bool v = j < m && ((validity_in[R >> 5] >> (R & 31)) & 1u);
        const uint64_t vm = __ballot(v);
        const uint32_t k = rank + popc_below(vm);
        rank += __popcll(vm);
        if (j < m) {
            uint8_t* o = values + static_cast<uint64_t>(R) * pw;
            const uint8_t* s = src + static_cast<uint64_t>(k) * pw;
            if (pw == 8) {
                const uint2 x = v ? *reinterpret_cast<const uint2*>(s) : make_uint2(0, 0);
                *reinterpret_cast<uint2*>(o) = x;
            } else if (pw == 4) {
                *reinterpret_cast<uint32_t*>(o) = v ? *reinterpret_cast<const uint32_t*>(s) : 0u;
            } else {
                for (uint32_t q = 0; q < pw / 4; q++)
                    reinterpret_cast<uint32_t*>(o)[q] = v ? reinterpret_cast<const uint32_t*>(s)[q] : 0u;
            }
        }
    }
}

__global__ void __launch_bounds__(256) k_fixed_scatter(const uint8_t* __restrict__ bytes,
                                                       const DevPage* __restrict__ pages,
                                                       const DevTile* __restrict__ tiles, int ntiles,
                                                       uint32_t pw, const uint32_t* __restrict__ validity_in,
                                                       const int32_t* __restrict__ tile_rank,
                                                       const int32_t* __restrict__ page_pos,
                                                       const DevErr* __restrict__ page_err,
                                                       uint8_t* __restrict__ values) {
    const int t = blockIdx.x * kTilesPerBlock + static_cast<int>(threadIdx.x / kWave);
    if (t >= ntiles) return;
    const DevTile T = tiles[t];
    if (page_err[T.page].code) return;  // the decode fails; nothing may be read past the page
    scatter_tile(bytes, pages, T, pw, validity_in, static_cast<uint32_t>(tile_rank[t]),
                 static_cast<uint32_t>(page_pos[T.page]), values);
}

__device__ __forceinline__ void fused_scatter(const uint8_t* __restrict__ bytes, const DevPage* __restrict__ pages, int p,
                                              const int32_t* __restrict__ page_tile0, const DevTile* __restrict__ tiles,
                                              ColumnParams cp, const uint32_t* validity, const int32_t* tile_rank,
                                              const int32_t* page_pos, const DevErr* page_err,
                                              uint8_t* __restrict__ values) {
    __syncthreads();  // (workgroup fence: this workgroup's validity, ranks and value start)
    if (page_err[p].code) return;
    const DevPage pg = pages[p];
    const uint32_t n = static_cast<uint32_t>(max(pg.nvals, 0));
    const int32_t t0 = page_tile0[p];
    const uint32_t nt = (n + kTileRows - 1) / kTileRows;
    const uint32_t pw = static_cast<uint32_t>(cp.plain_width);
    const uint32_t pos = static_cast<uint32_t>(page_pos[p]);
    for (uint32_t i = threadIdx.x / kWave; i < nt; i += blockDim.x / kWave) {
        const int32_t t = t0 + static_cast<int32_t>(i);
        scatter_tile(bytes, pages, tiles[t], pw, validity, static_cast<uint32_t>(tile_rank[t]), pos, values);
    }
}

}  // namespace

void launch_fixed_plain(hipStream_t s, const uint8_t* bytes, const DevPage* pages, int npages, const DevTile* tiles,
                        int ntiles, const int32_t* page_tile0, ColumnParams cp, uint32_t* validity,
                        uint8_t* values, int32_t* tile_rank, int32_t* page_pos, DevErr* page_err,
                        int32_t* err_any, bool fused, bool small) {
    if (ntiles <= 0) return;
    const uint32_t pw = static_cast<uint32_t>(cp.plain_width);
    const int tb = (ntiles + kTilesPerBlock - 1) / kTilesPerBlock;
    if (cp.max_def == 0 && cp.max_rep == 0) {
        hipLaunchKernelGGL(k_fixed_req, dim3(tb), dim3(kTilesPerBlock * kWave), 0, s, bytes, pages, tiles, ntiles, pw,
                           validity, values, page_err, err_any);
        return;
    }
    if (fused) {
        hipLaunchKernelGGL(k_fixed_levels2<true>, dim3(npages), dim3(kLvWaves * kWave), 0, s, bytes, pages, page_tile0,
                           cp, validity, tile_rank, page_pos, static_cast<int32_t*>(nullptr), page_err, err_any, tiles,
                           values);
        return;
    }
    if (small)
        hipLaunchKernelGGL((k_fixed_levels2<false, kLvStageS, kLvRecS>), dim3(npages), dim3(kLvWaves * kWave), 0, s, bytes,
                           pages, page_tile0, cp, validity, tile_rank, page_pos, static_cast<int32_t*>(nullptr), page_err,
                           err_any, static_cast<const DevTile*>(nullptr), static_cast<uint8_t*>(nullptr));
    else
        hipLaunchKernelGGL(k_fixed_levels2<false>, dim3(npages), dim3(kLvWaves * kWave), 0, s, bytes, pages, page_tile0,
                           cp, validity, tile_rank, page_pos, static_cast<int32_t*>(nullptr), page_err, err_any,
                           static_cast<const DevTile*>(nullptr), static_cast<uint8_t*>(nullptr));
    hipLaunchKernelGGL(k_fixed_scatter, dim3(tb), dim3(kTilesPerBlock * kWave), 0, s, bytes, pages, tiles, ntiles, pw,
                       validity, tile_rank, page_pos, page_err, values);
}

void launch_fixed_levels(hipStream_t s, const uint8_t* bytes, const DevPage* pages, int npages,
                         const int32_t* page_tile0, ColumnParams cp, uint32_t* validity, int32_t* tile_rank,
                         int32_t* page_pos, int32_t* page_nn, DevErr* page_err, int32_t* err_any, bool small) {
    if (npages <= 0) return;
    if (small)
        hipLaunchKernelGGL((k_fixed_levels2<false, kLvStageS, kLvRecS>), dim3(npages), dim3(kLvWaves * kWave), 0, s, bytes,
                           pages, page_tile0, cp, validity, tile_rank, page_pos, page_nn, page_err, err_any,
                           static_cast<const DevTile*>(nullptr), static_cast<uint8_t*>(nullptr));
    else
        hipLaunchKernelGGL(k_fixed_levels2<false>, dim3(npages), dim3(kLvWaves * kWave), 0, s, bytes, pages, page_tile0,
                           cp, validity, tile_rank, page_pos, page_nn, page_err, err_any,
                           static_cast<const DevTile*>(nullptr), static_cast<uint8_t*>(nullptr));
}

}  // namespace pqk
