// Probe: unaligned 16-byte LDS reads/writes (ds_read_b128 / ds_write_b128 at
// byte addresses) return the same bytes as a byte-wise copy on this GPU.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
struct __attribute__((packed, aligned(1))) U4 { uint32_t x, y, z, w; };
__global__ void k(const uint32_t* in, uint32_t* out) {
    __shared__ uint32_t s[1024];
    __shared__ uint32_t d[1024];
    for (int i = threadIdx.x; i < 1024; i += blockDim.x) { s[i] = in[i]; d[i] = 0; }
    __syncthreads();
    const uint8_t* b = reinterpret_cast<const uint8_t*>(s) + threadIdx.x * 7 + 3;
    U4 v = *reinterpret_cast<const U4*>(b);
    uint8_t* w = reinterpret_cast<uint8_t*>(d) + threadIdx.x * 13 + 1;
    *reinterpret_cast<U4*>(w) = v;  // overlapping writes across lanes are not compared
    __syncthreads();
    out[threadIdx.x * 4 + 0] = v.x; out[threadIdx.x * 4 + 1] = v.y;
    out[threadIdx.x * 4 + 2] = v.z; out[threadIdx.x * 4 + 3] = v.w;
}
int main() {
    uint32_t h[1024], o[1024];
    for (int i = 0; i < 1024; i++) h[i] = 0x01010101u * (i & 0xff) ^ (i * 2654435761u);
    uint32_t *di, *dout;
    hipMalloc(&di, sizeof h); hipMalloc(&dout, sizeof o);
    hipMemcpy(di, h, sizeof h, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(256), 0, 0, di, dout);
    hipMemcpy(o, dout, sizeof o, hipMemcpyDeviceToHost);
    const uint8_t* hb = reinterpret_cast<const uint8_t*>(h);
    int bad = 0;
    for (int t = 0; t < 256; t++) {
        const uint8_t* ob = reinterpret_cast<const uint8_t*>(o + t * 4);
        for (int j = 0; j < 16; j++) bad += ob[j] != hb[t * 7 + 3 + j];
    }
    printf("unaligned ds_read_b128: %s (%d bad bytes)\n", bad ? "MISMATCH" : "ok", bad);
    return bad ? 1 : 0;
}
