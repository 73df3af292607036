// plain_ba.hip — PLAIN BYTE_ARRAY decode for REQUIRED chunks (SURVEY §8a
// R-PLAIN: column_reader.cpp:213-222 + read_plain_value 249-253, a u32 length
// then the bytes, per value) in two passes over windows of consecutive pages
// (one contiguous image range of at most kPWin bytes):
//   k_plain_walk   one wavefront per window: the window is staged in LDS and
//                  each lane walks one page's length chain, writing
//                  (position in window, length) per row and the window's
//                  character count (filed under the k_plain_write workgroup
//                  that writes the window).  A chain that runs past its page
//                  is the reference's ByteBuffer error at that position.
//   k_plain_write  persistent workgroups, each wavefront a contiguous run of
//                  windows: the window is staged again, rows become int64
//                  offsets and validity words, and the characters go through a
//                  per-wave ring aligned to 16-byte output blocks (aligned LDS
//                  moves, 16-byte stores) as in k_pipe_write.  The ring holds a
//                  whole window, so any group of rows fits.
#include "kernels/device_common.hpp"
#include "kernels/kernels.hpp"
#include "pq_gpu.h"

namespace pqk {
namespace {

using namespace dev;

constexpr int kWalkWaves = 4;
constexpr int kPWWaves = 4;
constexpr uint32_t kPRing = kPWin + 32;  // a window's characters + the carried partial block

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
    const int w = static_cast<int>(blockIdx.x) * kWalkWaves + wv;
    if (w >= a.nwins) return;
    uint32_t* stage = stage_all[wv];
    const DevBatch W = a.wins[w];
    {
        const uint4* src = reinterpret_cast<const uint4*>(a.bytes + W.img_lo);
        uint4* dst = reinterpret_cast<uint4*>(stage);
        const uint32_t nb = (W.img_bytes + 15) / 16 + 1;
        for (uint32_t i = lane(); i < nb; i += kWave) dst[i] = src[i];
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
        uint32_t pos = 0, k = 0;
        for (; k < n; k++) {
            if (pos + 4 > size) { lane_err(a.page_err + p, a.err_any, pos, 4, size); break; }
            const uint32_t len = st_u32(stage, base + pos);
            pos += 4;
            if (static_cast<uint64_t>(pos) + len > size) { lane_err(a.page_err + p, a.err_any, pos, len, size); break; }
            ri[k] = (base + pos) | (len << 16);
            chars += len;
            pos += len;
        }
        for (; k < n; k++) ri[k] = 0;  // a failed page: empty rows (the decode reports the error)
    }
    chars = bcast_last(wave_incl_scan(chars));
    if (lane() == 0) {
        a.wchars[w] = chars;
        if (chars) atomicAdd(&a.bsum[(w / a.per) / kPWWaves], static_cast<unsigned long long>(chars));
    }
}

struct PWLds {
    uint32_t stage[kPWin / 4 + 8];
    uint4 ring[kPRing / 16];
};

__global__ void __launch_bounds__(kPWWaves * 64) k_plain_write(PlainLaunch a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
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
    uint8_t* ring = reinterpret_cast<uint8_t*>(S.ring);
    const uint8_t* sb = reinterpret_cast<const uint8_t*>(S.stage);
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
            for (uint32_t i = lane(); i < nb; i += kWave) dst[i] = src[i];
        }
        // validity: every row of a REQUIRED column is set
        {
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
        int64_t RB = G0 & ~static_cast<int64_t>(15);  // output address of ring[0]
        uint32_t run = 0;
        for (uint32_t g0 = 0; g0 < rows; g0 += kWave) {
            const uint32_t r = g0 + lane();
            const uint32_t info = r < rows ? a.rowinfo[R0 + r] : 0u;
            const uint32_t len = info >> 16, q = info & 0xFFFFu;
            const uint32_t inc = wave_incl_scan(len);
            const uint32_t s0 = run + inc - len;
            if (r < rows) a.offsets[R0 + r] = G0 + s0;
            run += bcast_last(inc);
            if (!fits) continue;
            if (r < rows && len) {
                const uint32_t p = static_cast<uint32_t>(G0 + s0 - RB);
                const uint32_t h = min((4u - (p & 3u)) & 3u, len);
                {
                    const uint32_t b0 = sb[q], b1 = sb[q + 1], b2 = sb[q + 2];
                    if (h > 0) ring[p] = static_cast<uint8_t>(b0);
                    if (h > 1) ring[p + 1] = static_cast<uint8_t>(b1);
                    if (h > 2) ring[p + 2] = static_cast<uint8_t>(b2);
                }
                const uint32_t p2 = p + h, q2 = q + h, rem = len - h;
                const uint32_t nd = rem >> 2, sh = q2 & 3u;
                uint32_t* rw = reinterpret_cast<uint32_t*>(ring) + (p2 >> 2);
                const uint32_t* sw = S.stage + (q2 >> 2);
                for (uint32_t d2 = 0; d2 < nd; d2 += 4) {
                    const uint32_t s0w = sw[d2], s1 = sw[d2 + 1], s2 = sw[d2 + 2], s3 = sw[d2 + 3], s4 = sw[d2 + 4];
                    rw[d2] = __builtin_amdgcn_alignbyte(s1, s0w, sh);
                    if (d2 + 1 < nd) rw[d2 + 1] = __builtin_amdgcn_alignbyte(s2, s1, sh);
                    if (d2 + 2 < nd) rw[d2 + 2] = __builtin_amdgcn_alignbyte(s3, s2, sh);
                    if (d2 + 3 < nd) rw[d2 + 3] = __builtin_amdgcn_alignbyte(s4, s3, sh);
                }
                {
                    const uint32_t t = rem & 3u, pt = p2 + 4 * nd, qt = q2 + 4 * nd;
                    const uint32_t b0 = sb[qt], b1 = sb[qt + 1], b2 = sb[qt + 2];
                    if (t > 0) ring[pt] = static_cast<uint8_t>(b0);
                    if (t > 1) ring[pt + 1] = static_cast<uint8_t>(b1);
                    if (t > 2) ring[pt + 2] = static_cast<uint8_t>(b2);
                }
            }
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            const bool last = g0 + kWave >= rows;
            const int64_t gend = G0 + run;
            const uint32_t nfull = static_cast<uint32_t>((gend - RB) >> 4);
            const uint32_t nblk = last ? static_cast<uint32_t>((gend - RB + 15) >> 4) : nfull;
            for (uint32_t b = lane(); b < nblk; b += kWave) {
                const uint4 v = S.ring[b];
                const int64_t blk = RB + 16 * static_cast<int64_t>(b);
                if (blk >= G0 && blk + 16 <= G1) {
                    *reinterpret_cast<uint4*>(a.chars + blk) = v;
                } else {
                    const uint32_t ow[4] = {v.x, v.y, v.z, v.w};
                    const int64_t gs = max(blk, G0), ge = min(blk + 16, G1);
                    for (int64_t x = gs; x < ge; x++) {
                        const uint32_t at = static_cast<uint32_t>(x - blk);
                        a.chars[x] = static_cast<uint8_t>(ow[at >> 2] >> (8 * (at & 3)));
                    }
                }
            }
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            if (!last) {
                if (lane() == 0 && nfull) S.ring[0] = S.ring[nfull];
                RB += 16 * static_cast<int64_t>(nfull);
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            }
        }
        __builtin_amdgcn_wave_barrier();
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
    const uint32_t lds = plain_write_lds();
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_plain_write), hipFuncAttributeMaxDynamicSharedMemorySize,
                              static_cast<int>(lds));
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, reinterpret_cast<const void*>(k_plain_write),
                                                     kPWWaves * kWave, lds) != hipSuccess || occ < 1)
        occ = 1;
    return occ;
}

void launch_plain_ba(hipStream_t s, PlainLaunch P) {
    if (P.nwins <= 0) return;
    int grid = 0, per = 0;
    plain_shape(P, &grid, &per);
    P.per = per;
    (void)hipMemsetAsync(P.bsum, 0, static_cast<size_t>(grid) * sizeof(unsigned long long), s);
    hipLaunchKernelGGL(k_plain_walk, dim3((P.nwins + kWalkWaves - 1) / kWalkWaves), dim3(kWalkWaves * kWave), 0, s, P);
    hipLaunchKernelGGL(k_plain_write, dim3(grid), dim3(kPWWaves * kWave), plain_write_lds(), s, P);
}

}  // namespace pqk
