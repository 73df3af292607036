// relayout.hip — raw chunk bytes (as the file holds them, DMA'd to HBM while
// the host walks the page headers) → the 16-byte slot image every decode
// kernel reads: each payload at its slot, zeros after it to
// the slot end, zeros past EOF.  One wave per payload; each lane writes one
// aligned 16-byte block, assembled from the two aligned 16-byte source blocks
// it straddles with byte funnel shifts.  Bound: HBM, payload read + slot
// written once (C3: 2 x 310 MB ≈ 0.1 ms at 6 TB/s).
#include <algorithm>

#include "kernels/kernels.hpp"

namespace pqk {
namespace {

// d-th dword of the 8-dword pair (a, b), d in 0..7, without register-array indexing
__device__ __forceinline__ uint32_t pick(const uint4& a, const uint4& b, uint32_t d) {
    const uint32_t lo = (d & 2) ? ((d & 1) ? a.w : a.z) : ((d & 1) ? a.y : a.x);
    const uint32_t hi = (d & 2) ? ((d & 1) ? b.w : b.z) : ((d & 1) ? b.y : b.x);
    return (d & 4) ? hi : lo;
}

__global__ __launch_bounds__(256) void k_relayout(const uint8_t* __restrict__ raw, uint8_t* __restrict__ img,
                                                  const RelayoutEntry* __restrict__ ent, int32_t n) {
    const uint32_t lane = __lane_id();
    const int32_t waves = static_cast<int32_t>(gridDim.x * (blockDim.x / kWave));
    for (int32_t i = static_cast<int32_t>(blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave); i < n;
         i += waves) {
        const RelayoutEntry e = ent[i];
        uint4* dst = reinterpret_cast<uint4*>(img + e.dst);
        const uint32_t nblk = e.slot / 16;
        for (uint32_t k = lane; k < nblk; k += kWave) {
            const uint32_t b0 = k * 16;  // first payload byte of this block
            uint4 v = make_uint4(0, 0, 0, 0);
            if (b0 < e.avail) {
                const uint64_t s = e.src + b0;
                const uint4* q = reinterpret_cast<const uint4*>(raw + (s & ~15ull));
                const uint4 a = q[0], b = q[1];  // raw has >= 32 readable bytes past any payload
                const uint32_t sh = static_cast<uint32_t>(s & 15), d = sh >> 2, bs = sh & 3;
                const uint32_t w0 = pick(a, b, d), w1 = pick(a, b, d + 1), w2 = pick(a, b, d + 2),
                               w3 = pick(a, b, d + 3), w4 = pick(a, b, d + 4);
                v = make_uint4(__builtin_amdgcn_alignbyte(w1, w0, bs), __builtin_amdgcn_alignbyte(w2, w1, bs),
                               __builtin_amdgcn_alignbyte(w3, w2, bs), __builtin_amdgcn_alignbyte(w4, w3, bs));
                if (b0 + 16 > e.avail) {  // last partial block: bytes past the payload are zero
                    const uint32_t keep = e.avail - b0;  // 1..15
                    uint32_t* x = reinterpret_cast<uint32_t*>(&v);
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        const int32_t kb = static_cast<int32_t>(keep) - 4 * j;
                        x[j] &= kb >= 4 ? 0xFFFFFFFFu : (kb <= 0 ? 0u : ((1u << (8 * kb)) - 1u));
                    }
                }
            }
            dst[k] = v;
        }
    }
}

}  // namespace

void launch_relayout(hipStream_t s, const uint8_t* raw, uint8_t* img, const RelayoutEntry* ent, int32_t n) {
    if (n <= 0) return;
    const int per_block = 4;  // waves
    const int blocks = std::min((n + per_block - 1) / per_block, 256 * 32);
    hipLaunchKernelGGL(k_relayout, dim3(blocks), dim3(per_block * kWave), 0, s, raw, img, ent, n);
}

}  // namespace pqk
