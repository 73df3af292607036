// window.hpp — wave-uniform byte reader over a register-resident window.
//
// The serial parts of Parquet decode (hybrid-stream run headers,
// rle_decoder.hpp:37-53/76-95; BYTE_ARRAY u32 length chains,
// column_reader.cpp:249-253) advance a single, wave-uniform cursor.  Keeping
// 1 KiB of the stream in four VGPRs (lane l holds dwords l, 64+l, 128+l,
// 192+l) lets the cursor read bytes with v_readlane_b32 into SGPRs instead of
// a dependent LDS or HBM round trip per byte.  A second window is prefetched
// so that a long chain (dictionary pages) never waits on a reload.
#pragma once
#include "kernels/device_common.hpp"

namespace pqk {
namespace dev {

__device__ __forceinline__ uint32_t uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }

struct Win {
    uint32_t v0, v1, v2, v3;  // current window (dword wbase + 64k + lane)
    uint32_t n0, n1, n2, n3;  // prefetched next window (dword wbase + 256 + ...)
    uint32_t wbase;           // uniform dword index of the current window
    const uint32_t* src;      // aligned source words (global or LDS)
    uint32_t nwords;          // words readable from src (zero beyond)
};

__device__ __forceinline__ uint32_t wload(const uint32_t* src, uint32_t nwords, uint32_t i) {
    return i < nwords ? src[i] : 0u;
}

__device__ __forceinline__ void win_fill(Win& w, uint32_t wbase) {
    w.wbase = uni(wbase);
    const uint32_t i = w.wbase + lane();
    w.v0 = wload(w.src, w.nwords, i);
    w.v1 = wload(w.src, w.nwords, i + 64);
    w.v2 = wload(w.src, w.nwords, i + 128);
    w.v3 = wload(w.src, w.nwords, i + 192);
    w.n0 = wload(w.src, w.nwords, i + 256);
    w.n1 = wload(w.src, w.nwords, i + 320);
    w.n2 = wload(w.src, w.nwords, i + 384);
    w.n3 = wload(w.src, w.nwords, i + 448);
}

__device__ __forceinline__ void win_init(Win& w, const uint32_t* src, uint32_t nwords) {
    w.src = src;
    w.nwords = nwords;
    win_fill(w, 0);
}

// Slide forward by 256 dwords (the prefetched half becomes current).
__device__ __forceinline__ void win_slide(Win& w) {
    w.v0 = w.n0; w.v1 = w.n1; w.v2 = w.n2; w.v3 = w.n3;
    w.wbase = uni(w.wbase + 256);
    const uint32_t i = w.wbase + 256 + lane();
    w.n0 = wload(w.src, w.nwords, i);
    w.n1 = wload(w.src, w.nwords, i + 64);
    w.n2 = wload(w.src, w.nwords, i + 128);
    w.n3 = wload(w.src, w.nwords, i + 192);
}

// Make dwords [d, d + 4] addressable (d uniform, absolute dword index):
// afterwards wbase <= d < wbase + 256, so d + 4 < wbase + 512.
__device__ __forceinline__ void win_ensure(Win& w, uint32_t d) {
    if (d < w.wbase || d >= w.wbase + 512) {
        win_fill(w, d);
    } else if (d >= w.wbase + 256) {
        win_slide(w);
    }
}

__device__ __forceinline__ uint32_t rl(uint32_t v, uint32_t l) { return __builtin_amdgcn_readlane(v, l); }

// Dword d (absolute, uniform) from the window; win_ensure(d) must hold.
__device__ __forceinline__ uint32_t win_dword(const Win& w, uint32_t d) {
    uint32_t r = uni(d - w.wbase);
    uint32_t l = r & 63;
    switch (r >> 6) {
        case 0: return rl(w.v0, l);
        case 1: return rl(w.v1, l);
        case 2: return rl(w.v2, l);
        case 3: return rl(w.v3, l);
        case 4: return rl(w.n0, l);
        case 5: return rl(w.n1, l);
        case 6: return rl(w.n2, l);
        default: return rl(w.n3, l);
    }
}

// 64 bits starting at byte p (uniform).
__device__ __forceinline__ uint64_t win_u64(Win& w, uint32_t p) {
    uint32_t d = p >> 2;
    win_ensure(w, d);
    uint64_t a = (static_cast<uint64_t>(win_dword(w, d + 1)) << 32) | win_dword(w, d);
    uint64_t b = win_dword(w, d + 2);
    uint32_t s = (p & 3) * 8;
    return s ? ((a >> s) | (b << (64 - s))) : a;
}
__device__ __forceinline__ uint32_t win_u32(Win& w, uint32_t p) {
    return static_cast<uint32_t>(win_u64(w, p));
}

}  // namespace dev
}  // namespace pqk
