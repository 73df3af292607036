// plain_ba.hip — PLAIN BYTE_ARRAY decode for REQUIRED chunks (SURVEY §8a
// R-PLAIN: column_reader.cpp:213-222 + read_plain_value 249-253, a u32 length
// then the bytes, per value) in two passes over windows of consecutive pages
// (one contiguous image range of at most kPWin bytes), or in one pass
// (k_plain_fused, below) when the pages' character counts are known:
//   k_plain_walk   persistent waves, one window at a time: the window is
//                  staged in LDS and each lane walks one page's length chain, writing
//                  (position in window, length) per row and the window's
//                  character count (filed under the k_plain_write workgroup
//                  that writes the window).  A chain that runs past its page
//                  is the reference's ByteBuffer error at that position.
//   k_plain_write  persistent workgroups, each wavefront a contiguous run of
//                  windows: the window is staged again, rows become int64
//                  offsets and validity words, and each lane copies its row's
//                  characters from the staged window with unaligned 16-byte
//                  moves (row_copy.hpp, as k_pipe_write does; the LDS ring of
//                  aligned blocks it replaces took 0.44 ms against 0.38 on C3:
//                  without the ring a wave needs half the LDS, so twice as many
//                  waves fit a CU).
#include <algorithm>

#include "kernels/device_common.hpp"
#include "kernels/row_copy.hpp"
#include "kernels/kernels.hpp"
#include "kernels/lane_walk.hpp"
#include "pq_gpu.h"

namespace pqk {
namespace {

using namespace dev;

constexpr int kWalkWaves = 4;
constexpr int kPWWaves = 4;

__device__ __forceinline__ uint32_t st_u32(const uint32_t* w, uint32_t a) {
    return __builtin_amdgcn_alignbyte(w[(a >> 2) + 1], w[a >> 2], a & 3);
}

// Per-lane error record (the page's own record; one lane per page).
__device__ __forceinline__ void lane_err(DevErr* e, int32_t* any, uint32_t pos, uint32_t need, uint32_t size) {
    e->code = PQ_ERR_BUFFER;
    e->pos = static_cast<int32_t>(pos);
    e->need = static_cast<int32_t>(need);
    e->size = static_cast<int32_t>(size);
    atomicOr(any, 1);
}

__global__ void __launch_bounds__(kWalkWaves * 64) k_plain_walk(PlainLaunch a) {
    __shared__ __attribute__((aligned(16))) uint32_t stage_all[kWalkWaves][kPWin / 4 + 8];
    const int wv = static_cast<int>(threadIdx.x / kWave);
    if (a.gate && *a.gate) return;
    uint32_t* stage = stage_all[wv];
    // persistent: a grid of one wave of workgroups walks the windows in a
    // grid-stride loop (one workgroup per window group was dispatch-bound)
    for (int w = static_cast<int>(blockIdx.x) * kWalkWaves + wv; w < a.nwins;
         w += static_cast<int>(gridDim.x) * kWalkWaves) {
    const DevBatch W = a.wins[w];
    {
        const uint4* src = reinterpret_cast<const uint4*>(a.bytes + W.img_lo);
        uint4* dst = reinterpret_cast<uint4*>(stage);
        const uint32_t nb = (W.img_bytes + 15) / 16 + 1;
        copy_blocks(dst, src, nb, lane(), kWave);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    uint32_t chars = 0;
    if (static_cast<int>(lane()) < W.np) {
        const int p = W.p0 + static_cast<int>(lane());
        const DevPage pg = a.pages[p];
        const uint32_t size = static_cast<uint32_t>(max(pg.size, 0));
        const uint32_t n = static_cast<uint32_t>(max(pg.nvals, 0));
        const uint32_t base = static_cast<uint32_t>(pg.off - W.img_lo);
        uint32_t* ri = a.rowinfo + pg.first_row;
        // the pages' length chains in lock step, branch-free (a divergent
        // loop with early exits spends more on exec-mask bookkeeping than on
        // the walk): one string per lane per step
        uint32_t pos = 0, k = 0;
        bool alive = n > 0, failed = false;
        while (alive) {
            const uint32_t len = st_u32(stage, base + min(pos, size));
            const bool e1 = pos + 4 > size;
            const bool e2 = !e1 && static_cast<uint64_t>(pos) + 4 + len > size;
            if (e1 | e2) {  // ByteBuffer::check (common.hpp:162-168): the reference's error position
                lane_err(a.page_err + p, a.err_any, e1 ? pos : pos + 4, e1 ? 4u : len, size);
                failed = true;
                break;
            }
            ri[k] = (base + pos + 4) | (len << 16);
            chars += len;
            pos += 4 + len;
            k++;
            alive = k < n;
        }
        if (failed)
            for (; k < n; k++) ri[k] = 0;  // a failed page: empty rows (the decode reports the error)
    }
    chars = bcast_last(wave_incl_scan(chars));
    if (lane() == 0) {
        a.wchars[w] = chars;
        if (chars) atomicAdd(&a.bsum[(w / a.per) / kPWWaves], static_cast<unsigned long long>(chars));
    }
    __builtin_amdgcn_wave_barrier();
    }
}

struct PWLds {
    uint32_t stage[kPWin / 4 + 8];
};

__global__ void __launch_bounds__(kPWWaves * 64) k_plain_write(PlainLaunch a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    if (a.gate && *a.gate) return;
    const int wv = static_cast<int>(threadIdx.x / kWave);
    PWLds& S = reinterpret_cast<PWLds*>(smem)[wv];
    const int per = a.per;
    const int ta = min(a.nwins, (static_cast<int>(blockIdx.x) * kPWWaves + wv) * per);
    const int tb = min(a.nwins, ta + per);
    __shared__ unsigned long long red[kPWWaves];
    auto wave_sum64 = [](unsigned long long v) {
        for (int d = 1; d < kWave; d <<= 1) {
            const uint32_t lo = static_cast<uint32_t>(__shfl_xor(static_cast<int>(v), d));
            const uint32_t hi = static_cast<uint32_t>(__shfl_xor(static_cast<int>(v >> 32), d));
            v += (static_cast<unsigned long long>(hi) << 32) | lo;
        }
        return v;
    };
    {
        unsigned long long acc = 0;
        for (uint32_t b = threadIdx.x; b < blockIdx.x; b += blockDim.x) acc += a.bsum[b];
        acc = wave_sum64(acc);
        if (lane() == 0) red[wv] = acc;
    }
    __syncthreads();
    int64_t G = 0;
    for (int q = 0; q < kPWWaves; q++) G += static_cast<int64_t>(red[q]);
    {
        const int tfirst = min(a.nwins, static_cast<int>(blockIdx.x * kPWWaves) * per);
        unsigned long long in = 0;
        for (int q = tfirst + static_cast<int>(lane()); q < ta; q += kWave) in += static_cast<unsigned long long>(a.wchars[q]);
        G += static_cast<int64_t>(wave_sum64(in));
    }
    for (int w = ta; w < tb; w++) {
        const DevBatch W = a.wins[w];
        const int64_t R0 = a.pages[W.p0].first_row;
        const DevPage lp = a.pages[W.p0 + W.np - 1];
        const uint32_t rows = static_cast<uint32_t>(lp.first_row + max(lp.nvals, 0) - R0);
        const int64_t G0 = G;
        const int64_t G1 = G0 + a.wchars[w];
        G = G1;
        {
            const uint4* src = reinterpret_cast<const uint4*>(a.bytes + W.img_lo);
            uint4* dst = reinterpret_cast<uint4*>(S.stage);
            const uint32_t nb = (W.img_bytes + 15) / 16 + 1;
            copy_blocks(dst, src, nb, lane(), kWave);
        }
        // validity: every row of a REQUIRED column is set (OPTIONAL: the
        // levels pass wrote it)
        if (a.validity) {
            const int64_t gfirst = R0 >> 5, glast = rows ? (R0 + rows - 1) >> 5 : gfirst - 1;
            for (int64_t g = gfirst + lane(); g <= glast; g += kWave) {
                const int64_t lo = max(g * 32, R0), hi = min(g * 32 + 32, R0 + static_cast<int64_t>(rows));
                const uint32_t nbit = static_cast<uint32_t>(hi - lo), sh = static_cast<uint32_t>(lo - g * 32);
                const uint32_t val = (nbit >= 32 ? 0xFFFFFFFFu : ((1u << nbit) - 1u)) << sh;
                if (nbit == 32) a.validity[g] = val;
                else atomicOr(&a.validity[g], val);
            }
        }
        if (R0 + rows == a.nrows_total && lane() == 0) {
            a.offsets[a.nrows_total] = G1;
            *a.total = G1;
        }
        const bool fits = G1 <= a.capacity;
        if (!fits && lane() == 0) atomicOr(a.overflow, 1);
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // rows -> int64 offsets (coalesced) and characters, each lane copying
        // its row from the staged window (row_copy.hpp)
        // (the row infos of up to 512 rows load at once: a load inside the
        // row loop would wait for the previous rows' stores, vmcnt)
        uint32_t run = 0;
        for (uint32_t kb = 0; kb < rows; kb += 8 * kWave) {
            uint32_t inf[8];
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const uint32_t r = kb + k * kWave + lane();
                inf[k] = r < rows ? a.rowinfo[R0 + r] : 0u;
            }
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const uint32_t g0 = kb + k * kWave;
                if (g0 >= rows) break;
                const uint32_t r = g0 + lane();
                const uint32_t info = inf[k];
                const uint32_t len = info >> 16, q = info & 0xFFFFu;
                const uint32_t inc = wave_incl_scan(len);
                const uint32_t s0 = run + inc - len;
                if (r < rows) a.offsets[R0 + r] = G0 + s0;
                run += bcast_last(inc);
                if (fits && r < rows && len) rc::copy_row(a.chars + G0 + s0, S.stage, q, len);
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// ── one-pass form: walk + write per window ───────────────────────────────
// For REQUIRED pages whose strings fill the page exactly (the usual layout),
// a page's characters are size - 4 * num_values, so the host knows every
// window's first output byte (PlainLaunch.wbase) and one pass can do both
// jobs: the window is staged once (the next window's bytes load into
// registers while this one is decoded), each lane walks one page's length
// chain into an LDS row list, and the rows become offsets and characters as
// in k_plain_write.  A page whose chain does not end exactly at its end (an
// error, or bytes after its last string) sets *redo, and the host decodes
// the chunk again with the two passes (which report the reference's errors).
constexpr int kPFWaves = 4;
constexpr uint32_t kPFBlocks = kPWin / 16 + 1;                       // staged 16-byte blocks per window
constexpr uint32_t kPFLoads = (kPFBlocks + kWave - 1) / kWave;       // prefetch registers per lane
struct PFLds {
    uint32_t stage[kPWin / 4 + 8];
    uint16_t list[kPWin / 4];  // window offset of each row's characters
};

__global__ void __launch_bounds__(kPFWaves * 64) k_plain_fused(PlainLaunch a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    if (a.gate && *a.gate) return;  // pseudo pages: the spec pass fell back
    if (a.wmode >= kWinOpt && *a.redo) return;  // OPTIONAL: the levels or the chains failed
    const int wv = static_cast<int>(threadIdx.x / kWave);
    PFLds& S = reinterpret_cast<PFLds*>(smem)[wv];
    const int nw = static_cast<int>(gridDim.x) * kPFWaves;
    int w = static_cast<int>(blockIdx.x) * kPFWaves + wv;
    if (w >= a.nwins) return;
    uint4 pf[kPFLoads];
    auto fetch = [&](const DevBatch& W) {
        const uint4* src = reinterpret_cast<const uint4*>(a.bytes + W.img_lo);
        const uint32_t nb = (W.img_bytes + 15) / 16 + 1;
#pragma unroll
        for (uint32_t k = 0; k < kPFLoads; k++) {
            const uint32_t b = lane() + k * kWave;
            pf[k] = b < nb ? src[b] : make_uint4(0u, 0u, 0u, 0u);
        }
    };
    DevBatch W = a.wins[w];
    fetch(W);
    for (;;) {
        const DevBatch Wc = W;
        int64_t G0 = (a.wmode == kWinBase || a.wmode == kWinPseudo) ? a.wbase[w] : 0;
#pragma unroll
        for (uint32_t k = 0; k < kPFLoads; k++) {
            const uint32_t b = lane() + k * kWave;
            if (b < kPFBlocks) reinterpret_cast<uint4*>(S.stage)[b] = pf[k];
        }
        const int wn = w + nw;
        if (wn < a.nwins) {
            W = a.wins[wn];
            fetch(W);
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // one lane per page: the length chain into the row list
        const bool act = static_cast<int>(lane()) < Wc.np;
        DevPage pg{};
        if (act) pg = a.pages[Wc.p0 + static_cast<int>(lane())];
        const uint32_t n = act ? static_cast<uint32_t>(max(pg.nvals, 0)) : 0u;
        const uint32_t rinc = wave_incl_scan(n);
        const uint32_t rows = bcast_last(rinc);
        bool misfit = act && rinc > kPWin / 4;  // more rows than 4-byte strings fit: not this form
        if (act && !misfit) {
            const uint32_t size = static_cast<uint32_t>(max(pg.size, 0));
            const uint32_t base = static_cast<uint32_t>(pg.off - Wc.img_lo);
            uint16_t* lst = S.list + (rinc - n);
            uint32_t pos = 0;
            for (uint32_t k = 0; k < n; k++) {
                if (pos + 4 > size) { misfit = true; break; }
                const uint32_t len = st_u32(S.stage, base + pos);
                if (len > size - pos - 4) { misfit = true; break; }
                lst[k] = static_cast<uint16_t>(base + pos + 4);
                pos += 4 + len;
            }
            misfit |= pos != size;
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (__ballot(misfit)) {  // the two passes redo the chunk; this window's row list is not whole
            if (lane() == 0) atomicOr(a.redo, 8);
            if (wn >= a.nwins) break;
            w = wn;
            continue;
        }
        const int64_t R0 = static_cast<int64_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(pg.first_row))) |
                           (static_cast<int64_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(pg.first_row >> 32))) << 32);
        int64_t G1;
        if (a.wmode == kWinBase) {
            G1 = a.wbase[w + 1];
        } else {
            // the window's own characters are its pages' bytes minus 4 per row
            const uint64_t sm = __ballot(act && n > 0);
            if (!sm) {  // no rows
                if (wn >= a.nwins) break;
                w = wn;
                continue;
            }
            const int fl = static_cast<int>(__builtin_ctzll(sm));
            const int64_t off = static_cast<int64_t>(__shfl(static_cast<long long>(pg.off), fl));
            const int64_t fr = static_cast<int64_t>(__shfl(static_cast<long long>(pg.first_row), fl));
            if (a.wmode == kWinPseudo) {
                // pseudo pages cut one real page whose strings fill it: the
                // characters before the window's first string are its offset
                // in the page minus 4 per earlier row
                G0 += off - 4 * fr;
            } else if (a.wmode == kWinOpt) {
                G0 = a.pbase[Wc.p0];  // value-section pages, one per real page
            } else {                  // pseudo pages of value sections
                const int rp = a.wpage[w];
                const int64_t v0 = static_cast<int64_t>(a.rpages[rp].off) + a.ppos[rp];
                G0 = a.pbase[rp] + (off - v0) - 4 * (fr - a.pdense[rp]);
            }
            const int64_t wch = act ? static_cast<int64_t>(max(pg.size, 0)) - 4 * static_cast<int64_t>(n) : 0;
            uint32_t lo = static_cast<uint32_t>(wch);
            lo = wave_incl_scan(lo);
            G1 = G0 + static_cast<int64_t>(bcast_last(lo));
        }
        // validity: every row of a REQUIRED column is set (OPTIONAL: the
        // levels pass wrote it)
        if (a.validity) {
            const int64_t gfirst = R0 >> 5, glast = rows ? (R0 + rows - 1) >> 5 : gfirst - 1;
            for (int64_t g = gfirst + lane(); g <= glast; g += kWave) {
                const int64_t lo = max(g * 32, R0), hi = min(g * 32 + 32, R0 + static_cast<int64_t>(rows));
                const uint32_t nbit = static_cast<uint32_t>(hi - lo), sh = static_cast<uint32_t>(lo - g * 32);
                const uint32_t val = (nbit >= 32 ? 0xFFFFFFFFu : ((1u << nbit) - 1u)) << sh;
                if (nbit == 32) a.validity[g] = val;
                else atomicOr(&a.validity[g], val);
            }
        }
        if (R0 + rows == a.nrows_total && lane() == 0) {
            a.offsets[a.nrows_total] = G1;
            *a.total = G1;
        }
        const bool fits = G1 <= a.capacity;
        if (!fits && lane() == 0) atomicOr(a.overflow, 1);
        uint32_t run = 0;
        for (uint32_t g0 = 0; g0 < rows; g0 += kWave) {
            const uint32_t r = g0 + lane();
            uint32_t q = 4, len = 0;
            if (r < rows) {
                q = S.list[r];
                len = st_u32(S.stage, q - 4);
            }
            const uint32_t inc = wave_incl_scan(len);
            const uint32_t s0 = run + inc - len;
            if (r < rows) a.offsets[R0 + r] = G0 + s0;
            run += bcast_last(inc);
            if (fits && r < rows && len) rc::copy_row(a.chars + G0 + s0, S.stage, q, len);
        }
        __builtin_amdgcn_wave_barrier();
        if (wn >= a.nwins) break;
        w = wn;
    }
}

// ── pages larger than a window (generic path) ─────────────────────────────
// One workgroup (16 waves) per REQUIRED PLAIN page larger than the generic
// kernel's LDS stage: 32 KiB windows of the page go to LDS; wave v walks the
// length chain of slice v speculatively from each of its first 64 byte
// offsets; one thread links the slices (the true chain enters slice v where
// slice v-1 left it) and the chosen lanes emit (len << 32 | position) row
// codes for k_ba_gather.  Entries longer than 60 bytes that straddle a slice
// edge, the string count limit and every bounds error are handled by the
// linking thread's exact walk (same error position and text as the
// reference, column_reader.cpp:249-253).
constexpr int kBigWaves = 16;
constexpr uint32_t kBigWin = 32768;
constexpr uint32_t kBigSlice = kBigWin / kBigWaves;
constexpr uint32_t kBigTiles = 256;
constexpr uint32_t kBadExit = 0xFFFFFFFFu;

__global__ void __launch_bounds__(kBigWaves * 64) k_plain_big_rows(const uint8_t* __restrict__ bytes,
                                                                  const DevPage* __restrict__ pages,
                                                                  uint32_t min_size, uint64_t* __restrict__ row_codes,
                                                                  int64_t* __restrict__ tile_chars,
                                                                  const int32_t* __restrict__ page_tile0,
                                                                  DevErr* __restrict__ page_err,
                                                                  int32_t* __restrict__ err_any) {
    __shared__ __attribute__((aligned(16))) uint32_t stage[kBigWin / 4 + 16];
    __shared__ uint32_t ex[kBigWaves * kWave], ec[kBigWaves * kWave];
    __shared__ int32_t seg_lane[kBigWaves];
    __shared__ uint32_t seg_base[kBigWaves];
    __shared__ unsigned long long tch[kBigTiles];
    __shared__ uint32_t sh[3];  // chain position, strings so far, stop
    const int p = blockIdx.x;
    const DevPage pg = pages[p];
    const uint32_t size = static_cast<uint32_t>(max(pg.size, 0));
    const uint32_t n = static_cast<uint32_t>(max(pg.nvals, 0));
    if (pg.mode != MODE_PLAIN || size <= min_size || n > kBigTiles * kTileRows) return;  // k_ba_rows' pages
    const uint8_t* page = bytes + pg.off;
    uint64_t* codes = row_codes + pg.first_row;
    const uint32_t wv = threadIdx.x / kWave;
    for (uint32_t i = threadIdx.x; i < kBigTiles; i += blockDim.x) tch[i] = 0;
    if (threadIdx.x == 0) { sh[0] = 0; sh[1] = 0; sh[2] = 0; }
    for (;;) {
        __syncthreads();
        const uint32_t wlo = sh[0], k0 = sh[1];
        if (sh[2] || k0 >= n) break;
        const uint32_t ab = wlo & ~15u;  // page byte ab sits at stage byte 0
        const uint32_t wbytes = wlo < size ? min(size - wlo, kBigWin - 16) : 0u;
        {
            const uint4* src = reinterpret_cast<const uint4*>(page + ab);
            uint4* dst = reinterpret_cast<uint4*>(stage);
            const uint32_t nb = min((wlo - ab + wbytes + 15) / 16 + 1, kBigWin / 16 + 1);
            copy_blocks(dst, src, nb, threadIdx.x, blockDim.x);
        }
        __syncthreads();
        const uint32_t wend = wlo + wbytes;
        {
            const uint32_t a0 = wlo + wv * kBigSlice, a1 = min(a0 + kBigSlice, wend);
            uint32_t q = a0 + lane(), cnt = 0;
            bool bad = q >= a1 || (wv == 0 && lane() != 0);
            while (!bad && q < a1) {
                if (q + 4 > size) { bad = true; break; }
                const uint32_t x = q - ab;
                const uint32_t len = __builtin_amdgcn_alignbyte(stage[(x >> 2) + 1], stage[x >> 2], x & 3);
                if (static_cast<uint64_t>(q) + 4 + len > size) { bad = true; break; }
                q += 4 + len;
                cnt++;
            }
            ex[threadIdx.x] = bad ? kBadExit : q;
            ec[threadIdx.x] = cnt;
        }
        __syncthreads();
        if (threadIdx.x == 0) {  // link the slices
            uint32_t t = wlo, kk = k0, stop = 0;
            for (uint32_t v = 0; v < kBigWaves; v++) {
                seg_lane[v] = -1;
                const uint32_t a0 = wlo + v * kBigSlice, a1 = min(a0 + kBigSlice, wend);
                if (stop || a0 >= wend || t >= a1 || kk >= n) continue;
                const uint32_t c = t - a0;
                if (c < kWave && ex[v * kWave + c] != kBadExit && kk + ec[v * kWave + c] <= n) {
                    seg_lane[v] = static_cast<int32_t>(c);
                    seg_base[v] = kk;
                    kk += ec[v * kWave + c];
                    t = ex[v * kWave + c];
                    continue;
                }
                while (t < a1 && kk < n) {  // exact walk
                    if (t + 4 > size) { set_err(page_err + p, err_any, PQ_ERR_BUFFER, t, 4, size); stop = 1; break; }
                    const uint32_t x = t - ab;
                    const uint32_t len = __builtin_amdgcn_alignbyte(stage[(x >> 2) + 1], stage[x >> 2], x & 3);
                    if (static_cast<uint64_t>(t) + 4 + len > size) {
                        set_err(page_err + p, err_any, PQ_ERR_BUFFER, t + 4, len, size);
                        stop = 1;
                        break;
                    }
                    codes[kk] = (static_cast<uint64_t>(len) << 32) | (t + 4);
                    tch[kk / kTileRows] += len;
                    kk++;
                    t += 4 + len;
                }
            }
            // past the window with strings left: the next window starts at t
            // (a string count reached with bytes left ends the page)
            if (!stop && kk < n && t >= size) {
                set_err(page_err + p, err_any, PQ_ERR_BUFFER, t, 4, size);
                stop = 1;
            }
            sh[0] = t;
            sh[1] = kk;
            sh[2] = stop;
        }
        __syncthreads();
        if (seg_lane[wv] == static_cast<int32_t>(lane())) {
            uint32_t q = wlo + wv * kBigSlice + lane(), kk = seg_base[wv];
            const uint32_t m = ec[threadIdx.x];
            uint32_t tsum = 0, tcur = kk / kTileRows;
            for (uint32_t j = 0; j < m; j++) {
                const uint32_t x = q - ab;
                const uint32_t len = __builtin_amdgcn_alignbyte(stage[(x >> 2) + 1], stage[x >> 2], x & 3);
                codes[kk] = (static_cast<uint64_t>(len) << 32) | (q + 4);
                if (kk / kTileRows != tcur) {
                    atomicAdd(&tch[tcur], static_cast<unsigned long long>(tsum));
                    tsum = 0;
                    tcur = kk / kTileRows;
                }
                tsum += len;
                kk++;
                q += 4 + len;
            }
            if (tsum) atomicAdd(&tch[tcur], static_cast<unsigned long long>(tsum));
        }
    }
    __syncthreads();
    const bool failed = sh[2] != 0;
    if (failed)  // rows after the error: NULL codes, nothing gathered
        for (uint32_t j = sh[1] + threadIdx.x; j < n; j += blockDim.x) codes[j] = 0xFFFFFFFFFFFFFFFFull;
    const int32_t t0 = page_tile0[p];
    for (uint32_t i = threadIdx.x; i * kTileRows < n; i += blockDim.x)
        tile_chars[t0 + static_cast<int32_t>(i)] = failed ? 0 : static_cast<int64_t>(tch[i]);
}


// ── pages larger than a window: speculative chunk chains ──────────────────
// k_plain_spec: kSpecChunks kPChunk-byte chunks per wave, kPCand lanes per
// chunk.  A string starts in a chunk's first 64 bytes (strings of <= 60
// bytes); every offset whose u32 could be a length (it and its bytes fit in
// the page) is a candidate, chunk 0's start the only one.  The first kPCand
// candidates walk the length chain (read_plain_value, column_reader.cpp:
// 249-253) until it leaves the chunk, recording where it left, how many
// strings it read and its first bounds error.  For text the false candidates
// die at once: four bytes of text are never a length that fits in the page.
// The wave first stages its chunks (kPChunk + 16 bytes each, pages sit in
// 16-byte aligned slots) in LDS with all loads in flight together, so the
// candidate tests and the chains read LDS (the chains from HBM/L2 were one
// dependent load per string: 0.16 ms on C4 c7).
constexpr int kSpecWaves = 4;
constexpr int kSpecChunks = kWave / static_cast<int>(kPCand);  // chunks per wave
constexpr uint32_t kSpecBlocks = kPChunk / 16 + 1;              // 16-byte blocks staged per chunk
constexpr uint32_t kSpecLoads = (kSpecChunks * kSpecBlocks + kWave - 1) / kWave;

__global__ void __launch_bounds__(kSpecWaves * 64) k_plain_spec(SpecLaunch a) {
    __shared__ __attribute__((aligned(16))) uint32_t stage_all[kSpecWaves][kSpecChunks * kSpecBlocks * 4 + 4];
    const int wv = static_cast<int>(threadIdx.x / kWave);
    const int cw = (static_cast<int>(blockIdx.x) * kSpecWaves + wv) * kSpecChunks;
    if (cw >= a.nchunks) return;
    uint32_t* stage = stage_all[wv];
    // lane j < 16: chunk cw + j's page offset, size, chunk start
    // d_start: where the page's chain starts (0, or after an OPTIONAL page's levels)
    uint32_t d_lo = 0, d_hi = 0, d_size = 0, d_cs = 0, d_start = 0, d_slot = 0;
    if (static_cast<int>(lane()) < kSpecChunks && cw + static_cast<int>(lane()) < a.nchunks) {
        const uint2 ch = a.chunks[cw + lane()];
        const DevPage pg = a.pages[ch.x];
        d_lo = static_cast<uint32_t>(pg.off);
        d_hi = static_cast<uint32_t>(pg.off >> 32);
        d_size = static_cast<uint32_t>(max(pg.size, 0));
        d_cs = ch.y * kPChunk;
        d_start = a.ppos ? static_cast<uint32_t>(max(a.ppos[ch.x], 0)) : 0u;
        d_slot = (d_size + 15) / 16 * 16 + 16;  // the page's slot in the image
    }
    // stage: block t of the wave's kSpecChunks x kSpecBlocks (chunk t / kSpecBlocks)
    {
        uint4 v[kSpecLoads];
#pragma unroll
        for (uint32_t u = 0; u < kSpecLoads; u++) {
            const uint32_t t = lane() + u * kWave;
            const int j = static_cast<int>(t / kSpecBlocks);
            const uint32_t blk = t - static_cast<uint32_t>(j) * kSpecBlocks;
            const int js = min(j, kSpecChunks - 1);  // shuffles with every lane active
            const uint64_t off = (static_cast<uint64_t>(static_cast<uint32_t>(__shfl(static_cast<int>(d_hi), js))) << 32) |
                                 static_cast<uint32_t>(__shfl(static_cast<int>(d_lo), js));
            const uint32_t cs = static_cast<uint32_t>(__shfl(static_cast<int>(d_cs), js));
            const uint32_t sl = static_cast<uint32_t>(__shfl(static_cast<int>(d_slot), js));
            const uint32_t b = cs + blk * 16;
            v[u] = (j < kSpecChunks && cw + j < a.nchunks && b + 16 <= sl)
                       ? *reinterpret_cast<const uint4*>(a.bytes + off + b)
                       : make_uint4(0u, 0u, 0u, 0u);
        }
#pragma unroll
        for (uint32_t u = 0; u < kSpecLoads; u++) {
            const uint32_t t = lane() + u * kWave;
            if (t < kSpecChunks * kSpecBlocks) reinterpret_cast<uint4*>(stage)[t] = v[u];
        }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // candidate offsets: lane l tests offset l of every chunk
    uint64_t mk = 0;
    const int jm = static_cast<int>(lane() / kPCand), sl = static_cast<int>(lane() % kPCand);
#pragma unroll
    for (int j = 0; j < kSpecChunks; j++) {
        const uint32_t size = __builtin_amdgcn_readlane(d_size, j);
        const uint32_t cs = __builtin_amdgcn_readlane(d_cs, j);
        const uint32_t start = __builtin_amdgcn_readlane(d_start, j);
        const uint32_t q = cs + lane(), ce = min(cs + kPChunk, size);
        const uint32_t len = q + 4 <= size ? st_u32(stage, static_cast<uint32_t>(j) * kSpecBlocks * 16 + lane()) : 0xFFFFFFFFu;
        bool plaus = q < ce && q + 4 <= size && static_cast<uint64_t>(q) + 4 + len <= size;
        if (start >= cs && start < cs + kPChunk) plaus = lane() == 0;  // the page's first string: one candidate, at start
        if (cs + kPChunk <= start) plaus = false;                      // levels, before the values
        const uint64_t m = __ballot(cw + j < a.nchunks && plaus);
        if (j == jm) mk = m;
    }
    // (shuffles with every lane active: a ds_bpermute under divergence reads
    // zeros from lanes outside exec)
    const uint32_t size = static_cast<uint32_t>(__shfl(static_cast<int>(d_size), jm));
    const uint32_t cs = static_cast<uint32_t>(__shfl(static_cast<int>(d_cs), jm));
    const uint32_t st0 = static_cast<uint32_t>(__shfl(static_cast<int>(d_start), jm));
    const int c = cw + jm;
    if (c >= a.nchunks) return;
    for (int i = 0; i < sl; i++) mk &= mk - 1;  // this lane's candidate: the sl-th set bit
    uint4 rec = make_uint4(0xFFFFFFFFu, 0u, 0u, 0u);
    if (mk) {
        const uint32_t ce = min(cs + kPChunk, size);
        const uint32_t sb = static_cast<uint32_t>(jm) * kSpecBlocks * 16 - cs;  // stage byte of page offset 0 (mod 2^32)
        const uint32_t q0 = (st0 >= cs && st0 < cs + kPChunk) ? st0 : cs + static_cast<uint32_t>(__builtin_ctzll(mk));
        uint32_t q = q0, cnt = 0, err = 0, need = 0;
        while (q < ce) {
            if (q + 4 > size) { err = 1; need = 4; break; }
            const uint32_t len = st_u32(stage, sb + q);
            if (static_cast<uint64_t>(q) + 4 + len > size) { err = 1; need = len; q += 4; break; }
            q += 4 + len;
            cnt++;
        }
        rec = make_uint4(q0 | (err << 31), q, cnt, need);
    }
    a.cand[static_cast<size_t>(c) * kPCand + sl] = rec;
}

// k_plain_link: one wave per page, rounds of kLinkStage chunks.  Each round
// first tries the speculative link (every chunk's pick from its neighbour's
// continuing candidate, checked link by link in parallel); when that does not
// hold for every chunk of the round the serial walk below decides.  Lane i takes
// chunk i of the round: its candidate records (registers) and a 64-entry
// table in LDS, entry offset -> exit (0xFFFFFFFF: no candidate there; bit 31:
// the walk hit a bounds error).  Lane 0 then follows the true chain through
// the tables, one LDS read per chunk (the entry of chunk k is where the chain
// left chunk k - 1).  Afterwards every lane turns its chunk's pick into a
// pseudo page: rows before it by a wave scan of the picked counts, cut at the
// page's value count (later bytes are never read), the page's error record at
// the first bounds error before the count (the reference's ByteBuffer
// position and size), the fallback flag for an entry that is not a candidate
// (a string longer than 60 bytes crossing a chunk edge) or a chain leaving
// its window.
constexpr uint32_t kLinkStage = 64;
constexpr uint32_t kLNone = 0xFFFFFFFFu;
constexpr uint32_t kPickHit = 1u << 16, kPickSkip = 1u << 17, kPickFail = 1u << 18, kPickNone = 1u << 19;

__global__ void __launch_bounds__(64) k_plain_link(SpecLaunch a) {
    __shared__ uint32_t tab[kLinkStage * 64];
    __shared__ uint32_t pick[kLinkStage];
    const int p = blockIdx.x;
    if (p >= a.npages) return;
    const DevPage pg = a.pages[p];
    const uint32_t size = static_cast<uint32_t>(max(pg.size, 0));
    // OPTIONAL pages: the values' count and first row come from the value
    // section page, the chain starts after the levels
    const uint32_t n = static_cast<uint32_t>(max(a.vpages ? a.vpages[p].nvals : pg.nvals, 0));
    const int64_t frow = a.vpages ? a.vpages[p].first_row : pg.first_row;
    const uint32_t pos0 = a.ppos ? static_cast<uint32_t>(max(a.ppos[p], 0)) : 0u;
    const int32_t c0 = a.chunk_base[p], c1 = a.chunk_base[p + 1];
    const uint32_t slot_end = (size + 15) / 16 * 16 + 16;
    // the chunk holding pos0 keeps its one candidate (entry pos0) in table slot 0
    auto tslot = [&](uint32_t entry, uint32_t chunk_start) {
        return (entry == pos0 && pos0 >= chunk_start && pos0 < chunk_start + kPChunk) ? 0u : entry - chunk_start;
    };
    uint32_t q = pos0, dead = 0;             // serial chain state (lane 0's values are used)
    uint32_t rows = 0, done = 0, fb = 0;     // wave-uniform: rows before the round, count reached / error, fallback
    for (int32_t cb = c0; cb < c1; cb += kLinkStage) {
        const int32_t cend = min(c1, cb + static_cast<int32_t>(kLinkStage));
        const uint32_t i = lane();
        const int32_t c = cb + static_cast<int32_t>(i);
        const bool act = c < cend;
        const uint32_t k = static_cast<uint32_t>(c - c0), chs = k * kPChunk;
        uint4 r[kPCand];
#pragma unroll
        for (uint32_t s = 0; s < kPCand; s++)
            r[s] = act ? a.cand[static_cast<size_t>(c) * kPCand + s] : make_uint4(kLNone, 0u, 0u, 0u);
        // Speculation: chunk i is entered where chunk i - 1's first candidate
        // that continues into chunk i (no bounds error, exit in chunk i's first
        // 64 bytes) left it.  When every chunk of the round holds a candidate
        // at that entry whose own exit is the one it advertised, the chain is
        // consistent link by link and equals the serial walk below (text has
        // one continuing chain per chunk); anything else takes the serial walk.
        uint32_t cexit = kLNone;
#pragma unroll
        for (int s = static_cast<int>(kPCand) - 1; s >= 0; s--)
            if (act && r[s].x != kLNone && !(r[s].x >> 31) && r[s].y >= chs + kPChunk && r[s].y < chs + kPChunk + 64)
                cexit = r[s].y;
        const uint32_t prev = static_cast<uint32_t>(__shfl_up(static_cast<int>(cexit), 1));
        const uint32_t q0 = __builtin_amdgcn_readfirstlane(q), dead0 = __builtin_amdgcn_readfirstlane(dead);
        const uint32_t e = i == 0 ? ((dead0 || q0 >= size) ? kLNone : q0) : prev;
        uint4 pr = make_uint4(kLNone, 0u, 0u, 0u);
        bool found = false;
#pragma unroll
        for (uint32_t s = 0; s < kPCand; s++)
            if (r[s].x != kLNone && (r[s].x & 0x7FFFFFFFu) == e) { pr = r[s]; found = true; }
        const bool lastc = c + 1 == cend;
        const bool ok = !act || (found && (lastc || (!(pr.x >> 31) && pr.y == cexit)));
        uint32_t pk;
        if (__ballot(!ok) == 0) {
            pk = act ? (kPickHit | (e - chs)) : kPickNone;
            const int ll = cend - cb - 1;
            const uint32_t lerr = __builtin_amdgcn_readlane(pr.x >> 31, ll);
            if (lerr) dead = 1;
            else q = __builtin_amdgcn_readlane(pr.y, ll);
        } else {
        uint4* row = reinterpret_cast<uint4*>(tab + i * 64);
#pragma unroll
        for (int w = 0; w < 16; w++) row[w] = make_uint4(kLNone, kLNone, kLNone, kLNone);
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (uint32_t s = 0; s < kPCand; s++)
            if (act && r[s].x != kLNone) tab[i * 64 + tslot(r[s].x & 0x7FFFFFFFu, chs)] = r[s].y | (r[s].x & 0x80000000u);
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (lane() == 0) {  // the chain: one LDS read per chunk
            const uint32_t nr = static_cast<uint32_t>(cend - cb);
            for (uint32_t j = 0; j < nr; j++) {
                const uint32_t js = (static_cast<uint32_t>(cb - c0) + j) * kPChunk;
                uint32_t pk;
                if (dead || q >= size) {
                    pk = kPickNone;
                    dead = 1;
                } else if (q >= js + kPChunk) {
                    pk = kPickSkip;  // a string spans this chunk
                } else if (tslot(q, js) >= 64) {
                    pk = kPickFail;
                    dead = 1;
                } else {
                    const uint32_t t = tab[j * 64 + tslot(q, js)];
                    if (t == kLNone) {
                        pk = kPickFail;
                        dead = 1;
                    } else {
                        pk = kPickHit | (q - js);
                        if (t >> 31) dead = 1;  // the chain stops at its bounds error
                        else q = t;
                    }
                }
                pick[j] = pk;
            }
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        pk = act ? pick[i] : kPickNone;
        }
        uint4 rr = make_uint4(kLNone, 0u, 0u, 0u);
        if (pk & kPickHit) {
            const uint32_t e = chs + (pk & 0xFFFFu);
#pragma unroll
            for (uint32_t s = 0; s < kPCand; s++)
                if (r[s].x != kLNone && (r[s].x & 0x7FFFFFFFu) == e) rr = r[s];
        }
        const bool hit = (pk & kPickHit) != 0;
        const uint32_t cnt = hit ? rr.z : 0u;
        const uint32_t incl = wave_incl_scan(cnt);
        const uint32_t before = rows + incl - cnt;
        const bool live = !done && before < n;             // the reference still reads values here
        const bool cend_here = live && hit && before + cnt >= n;
        const bool err_here = live && hit && !cend_here && (rr.x >> 31);
        const uint32_t g = k / kPChunkGroup;
        const bool fail_here = live && ((pk & kPickFail) || (hit && rr.y > min(g * kPChunkGroup * kPChunk + kPWin, slot_end)));
        // the first stop (count reached or bounds error) ends the page
        const uint64_t stops = __ballot(cend_here || err_here);
        const uint32_t first_stop = stops ? static_cast<uint32_t>(__builtin_ctzll(stops)) : kWave;
        const bool alive = live && i <= first_stop;
        if (err_here && i == first_stop) {
            DevErr* e = a.page_err + p;
            e->code = PQ_ERR_BUFFER;
            e->pos = static_cast<int32_t>(rr.y);
            e->need = static_cast<int32_t>(rr.w);
            e->size = static_cast<int32_t>(size);
            atomicOr(a.err_any, 1);
        }
        {
            const uint64_t fm = __ballot(fail_here && i <= first_stop);
            if (fm && !fb) {  // reason bits for diagnostics: 1 pick failed, 2 window; chunk << 8
                const uint32_t fl = static_cast<uint32_t>(__builtin_ctzll(fm));
                const uint32_t why = __builtin_amdgcn_readlane((pk & kPickFail) ? 1u : 2u, fl);
                fb = why | ((static_cast<uint32_t>(cb - c0) + fl) << 8);
            }
        }
        if (act) {
            const uint32_t take = !alive || !hit ? 0u : (cend_here ? n - before : cnt);
            const uint32_t ent = hit ? (pk & 0xFFFFu) : 0u;
            DevPage pp{};
            pp.mode = MODE_PLAIN;
            pp.dict = -1;
            pp.off = pg.off + chs + ent;
            // a chunk whose whole chain is taken: exactly its strings' bytes
            // (the one-pass kernel checks its walk ends there); a chain cut
            // at the value count: the rest of the page; no strings: empty
            const uint32_t rest = size > chs + ent ? size - chs - ent : 0u;
            pp.size = static_cast<int32_t>(take == 0 ? 0u : (take == cnt && rr.y >= chs + ent ? min(rr.y - chs - ent, rest) : rest));
            pp.nvals = static_cast<int32_t>(take);
            pp.first_row = frow + min(before, n);
            a.ppages[c] = pp;
        }
        rows += bcast_last(incl);
        if (stops) done = 1;
        q = __builtin_amdgcn_readfirstlane(q);
        dead = __builtin_amdgcn_readfirstlane(dead);
        __builtin_amdgcn_wave_barrier();
    }
    if (lane() == 0) {
        if (!fb && !done && rows < n) {  // the chain ended before the value count: the read at q fails
            DevErr* e = a.page_err + p;
            e->code = PQ_ERR_BUFFER;
            e->pos = static_cast<int32_t>(q);
            e->need = 4;
            e->size = static_cast<int32_t>(size);
            atomicOr(a.err_any, 1);
        }
        if (fb) atomicOr(a.fallback, static_cast<int32_t>(fb));
    }
}


// ── OPTIONAL chunks on the PLAIN kernels ──────────────────────────────────
// k_fixed_levels2 has decoded the def levels (validity, per-tile ranks, where
// each page's values start, non-null counts).  The value section of page p
// holds nn_p strings (column_reader.cpp:213-222 reads one per non-null row):
// it becomes a REQUIRED-shaped page of nn_p rows whose first row is the
// number of non-null rows before it, and whose characters start after the
// characters of the earlier pages (its bytes minus 4 per value, when its
// strings fill it; the one-pass kernel checks that).  A level error or a
// section too short for its values sets *redo: the host then decodes the
// chunk on the general path, which reports the reference's error.
__global__ void __launch_bounds__(256) k_opt_prep(OptLaunch o) {
    const int p = static_cast<int>(blockIdx.x * blockDim.x + threadIdx.x);
    if (p >= o.npages) return;
    const DevPage pg = o.pages[p];
    const bool bad = o.lerr[p].code != 0;
    const int64_t pos = bad ? 0 : o.page_pos[p];
    int64_t nn = bad ? 0 : o.page_nn[p];
    int64_t ch = static_cast<int64_t>(max(pg.size, 0)) - pos - 4 * nn;
    if (bad || nn < 0 || pos > pg.size || ch < 0) {
        atomicOr(o.redo, bad ? 2 : 4);
        nn = 0;
        ch = 0;
    }
    o.nnv[p] = nn;
    o.chv[p] = ch;
}

__global__ void __launch_bounds__(256) k_opt_vpages(OptLaunch o) {
    const int p = static_cast<int>(blockIdx.x * blockDim.x + threadIdx.x);
    if (p >= o.npages) return;
    const DevPage pg = o.pages[p];
    const int32_t pos = o.lerr[p].code ? 0 : max(o.page_pos[p], 0);
    DevPage v{};
    v.off = pg.off + static_cast<uint32_t>(pos);
    v.size = max(pg.size - pos, 0);
    v.nvals = static_cast<int32_t>(o.nnv[p]);
    v.first_row = o.pdense[p];
    v.mode = MODE_PLAIN;
    v.dict = -1;
    o.vpages[p] = v;
    if (p == o.npages - 1) o.doffs[o.pdense[p] + o.nnv[p]] = o.pbase[p] + o.chv[p];
}

// Def levels of small OPTIONAL pages, one lane per page (k_fixed_levels2's
// workgroup per page is for pages of thousands of rows): the lane walks the
// level stream with the reference's RleDecoder states (lane_walk.hpp) and ORs
// the validity bits, the per-tile ranks, the value section start and the
// non-null count (PLAIN: level >= max_def, column_reader.cpp:166-170).  A
// malformed section or stream sets *redo (the general path reports it).
__global__ void __launch_bounds__(256) k_opt_levels(const uint8_t* __restrict__ bytes, const DevPage* __restrict__ pages,
                                                    int npages, const int32_t* __restrict__ page_tile0, int32_t max_def,
                                                    uint32_t* __restrict__ validity, int32_t* __restrict__ tile_rank,
                                                    int32_t* __restrict__ page_pos, int32_t* __restrict__ page_nn,
                                                    DevErr* __restrict__ lerr, int32_t* __restrict__ redo) {
    const int p = static_cast<int>(blockIdx.x * blockDim.x + threadIdx.x);
    if (p >= npages) return;
    const DevPage pg = pages[p];
    const uint8_t* page = bytes + pg.off;
    const uint32_t size = static_cast<uint32_t>(max(pg.size, 0));
    const uint32_t n = static_cast<uint32_t>(max(pg.nvals, 0));
    const uint32_t md = static_cast<uint32_t>(max_def);
    auto fail = [&]() {
        lerr[p].code = PQ_ERR_UNSUPPORTED;
        atomicOr(redo, 1);
    };
    if (size < 4) return fail();
    const uint32_t dl = static_cast<uint32_t>(gld8(page, 0));
    if (static_cast<uint64_t>(dl) + 4 > size) return fail();
    const int32_t t0 = page_tile0[p];
    const int64_t R0 = pg.first_row;
    const uint32_t bw = level_bw(max_def);
    LRle r = lrle(4, dl, bw);
    auto rd8 = [&](uint32_t a) { return gld8(page, a); };
    uint32_t cur = 0, nn = 0;
    // validity bits of rows [a, a + k) of the page
    auto set_bits = [&](uint32_t a, uint32_t k) {
        int64_t lo = R0 + a;
        const int64_t hi = lo + k;
        while (lo < hi) {
            const int64_t w = lo >> 5;
            const uint32_t b0 = static_cast<uint32_t>(lo & 31);
            const uint32_t cnt = static_cast<uint32_t>(min(static_cast<int64_t>(32 - b0), hi - lo));
            atomicOr(&validity[w], (cnt == 32 ? 0xFFFFFFFFu : ((1u << cnt) - 1u)) << b0);
            lo += cnt;
        }
    };
    if (n) tile_rank[t0] = 0;
    const int rc = lane_rle(r, rd8, n, [&](uint32_t kind, uint32_t k, uint32_t arg) {
        if (kind == 0) {
            const bool v = arg >= md;
            // tile boundaries in [cur, cur + k) (the first tile's rank is 0)
            for (uint32_t b = max((cur + kTileRows - 1) / kTileRows, 1u) * kTileRows; b < cur + k && b < n; b += kTileRows)
                tile_rank[t0 + static_cast<int32_t>(b / kTileRows)] = static_cast<int32_t>(nn + (v ? b - cur : 0u));
            if (v) {
                set_bits(cur, k);
                nn += k;
            }
            cur += k;
        } else {
            uint32_t word = 0, wi = 0;
            bool have = false;
            for (uint32_t i = 0; i < k; i++, cur++) {
                if (cur % kTileRows == 0 && cur) tile_rank[t0 + static_cast<int32_t>(cur / kTileRows)] = static_cast<int32_t>(nn);
                const uint32_t lvl = gbits(page, size, static_cast<uint64_t>(arg) + static_cast<uint64_t>(i) * bw, bw);
                if (lvl >= md) {
                    const int64_t row = R0 + cur;
                    const uint32_t w = static_cast<uint32_t>(row >> 5);
                    if (have && w != wi) {
                        atomicOr(&validity[wi], word);
                        word = 0;
                    }
                    wi = w;
                    have = true;
                    word |= 1u << (row & 31);
                    nn++;
                }
            }
            if (have && word) atomicOr(&validity[wi], word);
        }
    });
    if (rc) return fail();
    page_pos[p] = static_cast<int32_t>(4 + dl);
    page_nn[p] = static_cast<int32_t>(nn);
}

// One wave per 512-row tile: row R's offset is the dense offset of its rank
// (the non-null rows before it), so a NULL row repeats the next value's start.
constexpr int kOptTiles = 4;
__global__ void __launch_bounds__(kOptTiles * 64) k_opt_offsets(const DevPage* __restrict__ pages,
                                                                const DevTile* __restrict__ tiles, int ntiles,
                                                                const int32_t* __restrict__ tile_rank,
                                                                const int64_t* __restrict__ pdense,
                                                                const uint32_t* __restrict__ validity,
                                                                const int64_t* __restrict__ doffs,
                                                                int64_t* __restrict__ offsets,
                                                                const int32_t* __restrict__ redo) {
    if (redo[0] || redo[-1]) return;  // d_flags[3] / [2]: the chunk is decoded again on the general path
    const int t = static_cast<int>(blockIdx.x) * kOptTiles + static_cast<int>(threadIdx.x / kWave);
    if (t >= ntiles) return;
    const DevTile T = tiles[t];
    const int64_t R0 = pages[T.page].first_row + T.row0;
    int64_t rank = pdense[T.page] + tile_rank[t];
    const uint32_t m = static_cast<uint32_t>(T.nrows);
    for (uint32_t j0 = 0; j0 < m; j0 += kWave) {
        const uint32_t j = j0 + lane();
        const int64_t R = R0 + j;
        const bool v = j < m && ((validity[R >> 5] >> (R & 31)) & 1u);
        const uint64_t vm = __ballot(v);
        if (j < m) offsets[R] = doffs[rank + popc_below(vm)];
        rank += __popcll(vm);
    }
}

}  // namespace

uint32_t plain_write_lds() { return kPWWaves * static_cast<uint32_t>(sizeof(PWLds)); }

static void plain_shape(const PlainLaunch& P, int* grid, int* per) {
    const int need = (P.nwins + kPWWaves - 1) / kPWWaves;
    *grid = max(1, min(need, P.grid));
    const int nw = *grid * kPWWaves;
    *per = max(1, (P.nwins + nw - 1) / nw);
}

int plain_write_blocks_per_cu() {
    return max(1, resident_blocks(reinterpret_cast<const void*>(k_plain_write), kPWWaves * kWave, plain_write_lds()));
}

void launch_plain_big_rows(hipStream_t s, const uint8_t* bytes, const DevPage* pages, int npages, uint32_t min_size,
                           uint64_t* row_codes, int64_t* tile_chars, const int32_t* page_tile0, DevErr* page_err,
                           int32_t* err_any) {
    if (npages <= 0) return;
    hipLaunchKernelGGL(k_plain_big_rows, dim3(npages), dim3(kBigWaves * kWave), 0, s, bytes, pages, min_size,
                       row_codes, tile_chars, page_tile0, page_err, err_any);
}

void launch_plain_ba(hipStream_t s, PlainLaunch P) {
    if (P.nwins <= 0) return;
    if (P.wbase || P.wmode >= kWinOpt) {  // one pass (the host re-runs the two passes if it sets *redo)
        const uint32_t lds = kPFWaves * static_cast<uint32_t>(sizeof(PFLds));
        const int fgrid = max(1, resident_blocks(reinterpret_cast<const void*>(k_plain_fused), kPFWaves * kWave, lds)) *
                          device_cus();
        const int need = (P.nwins + kPFWaves - 1) / kPFWaves;
        hipLaunchKernelGGL(k_plain_fused, dim3(std::min(need, fgrid)), dim3(kPFWaves * kWave), lds, s, P);
        return;
    }
    int grid = 0, per = 0;
    plain_shape(P, &grid, &per);
    P.per = per;
    (void)hipMemsetAsync(P.bsum, 0, static_cast<size_t>(grid) * sizeof(unsigned long long), s);
    {
        // resident workgroups of k_plain_walk on this device
        const int walk_grid = max(1, resident_blocks(reinterpret_cast<const void*>(k_plain_walk), kWalkWaves * kWave, 0)) *
                              device_cus();
        const int need = (P.nwins + kWalkWaves - 1) / kWalkWaves;
        hipLaunchKernelGGL(k_plain_walk, dim3(std::min(need, walk_grid)), dim3(kWalkWaves * kWave), 0, s, P);
    }
    hipLaunchKernelGGL(k_plain_write, dim3(grid), dim3(kPWWaves * kWave), plain_write_lds(), s, P);
}

void launch_plain_spec(hipStream_t s, const SpecLaunch& S) {
    if (S.nchunks <= 0) return;
    const int per_block = kSpecWaves * kSpecChunks;  // chunks per workgroup
    hipLaunchKernelGGL(k_plain_spec, dim3((S.nchunks + per_block - 1) / per_block), dim3(kSpecWaves * kWave), 0, s, S);
    hipLaunchKernelGGL(k_plain_link, dim3(S.npages), dim3(kWave), 0, s, S);
}

void launch_opt_pages(hipStream_t s, const OptLaunch& O) {
    if (O.npages <= 0) return;
    const int b = (O.npages + 255) / 256;
    hipLaunchKernelGGL(k_opt_prep, dim3(b), dim3(256), 0, s, O);
    launch_scan_i64(s, O.nnv, O.pdense, O.npages, O.tot_nn, O.scratch);
    launch_scan_i64(s, O.chv, O.pbase, O.npages, O.tot_ch, O.scratch);
    hipLaunchKernelGGL(k_opt_vpages, dim3(b), dim3(256), 0, s, O);
}

void launch_opt_levels(hipStream_t s, const uint8_t* bytes, const DevPage* pages, int npages,
                       const int32_t* page_tile0, int32_t max_def, uint32_t* validity, int32_t* tile_rank,
                       int32_t* page_pos, int32_t* page_nn, DevErr* lerr, int32_t* redo) {
    if (npages <= 0) return;
    hipLaunchKernelGGL(k_opt_levels, dim3((npages + 255) / 256), dim3(256), 0, s, bytes, pages, npages, page_tile0,
                       max_def, validity, tile_rank, page_pos, page_nn, lerr, redo);
}

void launch_opt_offsets(hipStream_t s, const DevPage* pages, const DevTile* tiles, int ntiles,
                        const int32_t* tile_rank, const int64_t* pdense, const uint32_t* validity,
                        const int64_t* doffs, int64_t* offsets, const int32_t* redo) {
    if (ntiles <= 0) return;
    hipLaunchKernelGGL(k_opt_offsets, dim3((ntiles + kOptTiles - 1) / kOptTiles), dim3(kOptTiles * kWave), 0, s,
                       pages, tiles, ntiles, tile_rank, pdense, validity, doffs, offsets, redo);
}

}  // namespace pqk
