// Probe: HBM write rate when one kernel writes two output streams tile by tile
// (k_pipe_write: 4 KiB of int64 offsets + ~11 KiB of characters per 512-row
// tile), against each stream alone and the two streams in separate kernels.
// Aligned 16-byte stores, one 1 KiB wave-instruction at a time.
// build: hipcc --offload-arch=gfx950 -O3 two_stream.hip -o two_stream.bin
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr size_t kTiles = 19531, kA = 4096, kB = 11184;  // bytes per tile (C2: 80 MB + 218 MB)

// lane-contiguous: each lane writes its own run of consecutive blocks of the
// tile's character range (the layout a lane assembling its own rows would use)
__global__ void __launch_bounds__(640) k_lanes(uint4* B) {
    const size_t nw = (size_t)gridDim.x * (blockDim.x / 64);
    const size_t w = blockIdx.x * (size_t)(blockDim.x / 64) + threadIdx.x / 64;
    const uint32_t l = threadIdx.x & 63;
    constexpr uint32_t nb = kB / 16, per = (nb + 63) / 64;
    for (size_t t = w; t < kTiles; t += nw)
        for (uint32_t i = 0; i < per; i++) {
            const uint32_t b = l * per + i;
            if (b < nb) B[t * nb + b] = make_uint4(t, b, 5, 6);
        }
}

__global__ void __launch_bounds__(640) k_two(uint4* A, uint4* B, int wa, int wb) {
    const size_t nw = (size_t)gridDim.x * (blockDim.x / 64);
    const size_t w = blockIdx.x * (size_t)(blockDim.x / 64) + threadIdx.x / 64;
    const uint32_t l = threadIdx.x & 63;
    for (size_t t = w; t < kTiles; t += nw) {
        if (wa)
            for (size_t i = l; i < kA / 16; i += 64) A[t * (kA / 16) + i] = make_uint4(t, i, 1, 2);
        if (wb)
            for (size_t i = l; i < kB / 16; i += 64) B[t * (kB / 16) + i] = make_uint4(t, i, 3, 4);
    }
}

int main() {
    uint4 *A, *B;
    hipMalloc(&A, kTiles * kA);
    hipMalloc(&B, kTiles * kB);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int grid = 256 * 2;
    auto run = [&](const char* name, int mode) {
        for (int rep = 0; rep < 2; rep++) {
            const int n = 20;
            hipEventRecord(e0);
            for (int i = 0; i < n; i++) {
                if (mode == 0) hipLaunchKernelGGL(k_two, dim3(grid), dim3(640), 0, 0, A, B, 1, 1);
                if (mode == 1) hipLaunchKernelGGL(k_two, dim3(grid), dim3(640), 0, 0, A, B, 1, 0);
                if (mode == 2) hipLaunchKernelGGL(k_two, dim3(grid), dim3(640), 0, 0, A, B, 0, 1);
                if (mode == 4) hipLaunchKernelGGL(k_lanes, dim3(grid), dim3(640), 0, 0, B);
                if (mode == 3) {
                    hipLaunchKernelGGL(k_two, dim3(grid), dim3(640), 0, 0, A, B, 1, 0);
                    hipLaunchKernelGGL(k_two, dim3(grid), dim3(640), 0, 0, A, B, 0, 1);
                }
            }
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            const double bytes = (mode == 1 ? kA : (mode == 2 || mode == 4) ? kB : kA + kB) * (double)kTiles;
            if (rep) printf("%-28s %8.1f us  %6.2f TB/s\n", name, ms / n * 1e3, bytes / (ms / n * 1e-3) / 1e12);
        }
    };
    run("both streams, one kernel", 0);
    run("offsets only", 1);
    run("characters only", 2);
    run("offsets kernel + chars kernel", 3);
    run("characters, lane-contiguous", 4);
    return 0;
}
