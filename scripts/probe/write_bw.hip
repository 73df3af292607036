// Probe: HBM store bandwidth for the character-writer pattern — each wave
// writes one contiguous chunk (uint4 per lane), chunks back to back.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k_chunks(uint4* out, size_t chunk16, size_t nchunks) {
    const size_t w = (blockIdx.x * blockDim.x + threadIdx.x) / 64;
    const uint32_t l = threadIdx.x & 63;
    const size_t nw = gridDim.x * blockDim.x / 64;
    for (size_t c = w; c < nchunks; c += nw) {
        uint4* o = out + c * chunk16;
        for (size_t i = l; i < chunk16; i += 64) o[i] = make_uint4(i, c, 1, 2);
    }
}
__global__ void k_flat(uint4* out, size_t n16) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
        out[i] = make_uint4(i, 0, 1, 2);
}
int main() {
    const size_t bytes = 218ull << 20;
    uint4* d;
    hipMalloc(&d, bytes);
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    const size_t n16 = bytes / 16;
    for (int rep = 0; rep < 2; rep++) {
        for (int grid : {1024, 2048, 4096, 8192}) {
            hipEventRecord(a);
            for (int it = 0; it < 10; it++) hipLaunchKernelGGL(k_flat, dim3(grid), dim3(256), 0, 0, d, n16);
            hipEventRecord(b); hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b);
            if (rep) printf("flat grid %5d: %.1f us  %.2f TB/s\n", grid, ms * 100, bytes / (ms / 10 * 1e-3) / 1e12);
        }
        for (size_t chunk : {size_t(720), size_t(2048)}) {
            hipEventRecord(a);
            for (int it = 0; it < 10; it++) hipLaunchKernelGGL(k_chunks, dim3(512), dim3(384), 0, 0, d, chunk, n16 / chunk);
            hipEventRecord(b); hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b);
            if (rep) printf("chunks of %zu blocks (512x6 waves): %.1f us  %.2f TB/s\n", chunk, ms * 100, bytes / (ms / 10 * 1e-3) / 1e12);
        }
        hipEventRecord(a);
        for (int it = 0; it < 10; it++) hipMemsetAsync(d, 1, bytes);
        hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        if (rep) printf("hipMemset: %.1f us  %.2f TB/s\n", ms * 100, bytes / (ms / 10 * 1e-3) / 1e12);
    }
    return 0;
}
