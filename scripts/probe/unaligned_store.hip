// Probe: HBM store throughput of the row-copy patterns k_pipe_write can use.
// Rows of 8..39 bytes (C2's dictionary lengths) packed back to back; lane l of
// each 64-row group owns row l.  Variants:
//   aligned16   the same bytes as aligned 16-byte blocks (ring layout)
//   row16       per row: unaligned 16-byte moves, last one overlapping
//   row16pair   as row16, rows < 16 bytes as two overlapping 8/4/2-byte moves
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
struct __attribute__((packed, aligned(1))) U16B { uint32_t x, y, z, w; };
struct __attribute__((packed, aligned(1))) U8B { uint32_t x, y; };
struct __attribute__((packed, aligned(1))) U4B { uint32_t x; };
struct __attribute__((packed, aligned(1))) U2B { uint16_t x; };

__global__ void k_aligned(uint4* out, size_t n16) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
        out[i] = make_uint4(i, 0, 1, 2);
}
template <bool kPair>
__global__ void k_rows(uint8_t* out, const uint32_t* off, size_t nrows) {
    for (size_t r = blockIdx.x * (size_t)blockDim.x + threadIdx.x; r < nrows; r += (size_t)gridDim.x * blockDim.x) {
        const uint32_t s0 = off[r], ln = off[r + 1] - s0;
        uint8_t* d = out + s0;
        const U16B z{ln, s0, 1u, 2u};
        if (ln >= 16) {
            for (uint32_t x = 0; x + 16 < ln; x += 16) *reinterpret_cast<U16B*>(d + x) = z;
            *reinterpret_cast<U16B*>(d + ln - 16) = z;
        } else if (kPair) {
            if (ln >= 8) {
                *reinterpret_cast<U8B*>(d) = U8B{ln, s0};
                *reinterpret_cast<U8B*>(d + ln - 8) = U8B{ln, s0};
            } else if (ln >= 4) {
                *reinterpret_cast<U4B*>(d) = U4B{ln};
                *reinterpret_cast<U4B*>(d + ln - 4) = U4B{ln};
            } else if (ln) {
                d[0] = 1;
            }
        } else {
            uint32_t x = 0;
            if (ln & 8u) { *reinterpret_cast<U8B*>(d) = U8B{ln, s0}; x = 8; }
            if (ln & 4u) { *reinterpret_cast<U4B*>(d + x) = U4B{ln}; x += 4; }
            if (ln & 2u) { *reinterpret_cast<U2B*>(d + x) = U2B{1}; x += 2; }
            if (ln & 1u) d[x] = 1;
        }
    }
}
int main() {
    const size_t nrows = 9500000;
    std::vector<uint32_t> off(nrows + 1);
    uint64_t s = 12345;
    off[0] = 0;
    for (size_t i = 0; i < nrows; i++) {
        s = s * 6364136223846793005ull + 1442695040888963407ull;
        off[i + 1] = off[i] + 8 + static_cast<uint32_t>((s >> 33) % 32);
    }
    const size_t bytes = off[nrows];
    uint8_t* d;
    uint32_t* doff;
    hipMalloc(&d, bytes + 64);
    hipMalloc(&doff, off.size() * 4);
    hipMemcpy(doff, off.data(), off.size() * 4, hipMemcpyHostToDevice);
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    auto timeit = [&](const char* name, auto launch) {
        launch();
        hipEventRecord(a);
        for (int it = 0; it < 10; it++) launch();
        hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        printf("%-12s %.1f us  %.2f TB/s\n", name, ms * 100, bytes / (ms / 10 * 1e-3) / 1e12);
    };
    printf("rows %zu, bytes %zu\n", nrows, bytes);
    timeit("aligned16", [&] { hipLaunchKernelGGL(k_aligned, dim3(4096), dim3(256), 0, 0, (uint4*)d, bytes / 16); });
    timeit("row16", [&] { hipLaunchKernelGGL(k_rows<false>, dim3(4096), dim3(256), 0, 0, d, doff, nrows); });
    timeit("row16pair", [&] { hipLaunchKernelGGL(k_rows<true>, dim3(4096), dim3(256), 0, 0, d, doff, nrows); });
    return 0;
}
