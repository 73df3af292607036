// Write-pattern probe for k_pipe_write's layout question: 300 MB written
// (a) grid-stride 16-byte stores over the whole buffer (a fill),
// (b) each wave a contiguous region of `per` tiles of 16 KiB (k_pipe_write's
//     persistent contiguous tile ranges),
// (c) tiles dealt round-robin to the waves (tile t -> wave t mod W).
// Timed with HIP events, 10 launches each.  hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void k_flat(uint4* out, size_t n16) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
        out[i] = make_uint4((uint32_t)i, 0, 1, 2);
}
// one wave per `wave` index; tiles of t16 16-byte blocks
__global__ void k_tiles(uint4* out, size_t t16, size_t ntiles, int contiguous) {
    const size_t w = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) / 64;
    const uint32_t l = threadIdx.x & 63;
    const size_t W = (size_t)gridDim.x * blockDim.x / 64;
    const size_t per = (ntiles + W - 1) / W;
    for (size_t k = 0; k < per; k++) {
        const size_t t = contiguous ? w * per + k : k * W + w;
        if (t >= ntiles) break;
        uint4* o = out + t * t16;
        for (size_t i = l; i < t16; i += 64) o[i] = make_uint4((uint32_t)i, (uint32_t)t, 1, 2);
    }
}
int main() {
    const size_t bytes = 300ull * 1000 * 1000 / 16384 * 16384;
    uint4* d;
    if (hipMalloc(&d, bytes) != hipSuccess) return 1;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const size_t n16 = bytes / 16, t16 = 16384 / 16, ntiles = bytes / 16384;
    auto run = [&](const char* name, auto launch) {
        for (int i = 0; i < 3; i++) launch();
        hipEventRecord(a);
        for (int i = 0; i < 10; i++) launch();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        ms /= 10;
        printf("%-34s %8.1f us %6.2f TB/s\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e12);
    };
    for (int grid : {1024, 4096}) {
        char nm[64];
        snprintf(nm, sizeof nm, "flat grid %d x 256", grid);
        run(nm, [&] { hipLaunchKernelGGL(k_flat, dim3(grid), dim3(256), 0, 0, d, n16); });
    }
    for (int waves_per_cu : {10, 20, 40}) {
        const int grid = 256 * waves_per_cu / 10;  // 640-thread workgroups
        char nm[64];
        snprintf(nm, sizeof nm, "tiles contiguous %d waves/CU", waves_per_cu);
        run(nm, [&] { hipLaunchKernelGGL(k_tiles, dim3(grid), dim3(640), 0, 0, d, t16, ntiles, 1); });
        snprintf(nm, sizeof nm, "tiles round-robin %d waves/CU", waves_per_cu);
        run(nm, [&] { hipLaunchKernelGGL(k_tiles, dim3(grid), dim3(640), 0, 0, d, t16, ntiles, 0); });
    }
    return 0;
}
