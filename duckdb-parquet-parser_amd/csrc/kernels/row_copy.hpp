// row_copy.hpp — one row's characters from an LDS byte image to HBM, as
// k_pipe_write copies dictionary entries: unaligned 16-byte moves, the last
// one overlapping the row's own earlier bytes, rows under 16 bytes as two
// overlapping 8/4/2-byte moves, so no store leaves the row and neighbouring
// lanes' rows (consecutive in the output) fill the lines between them.
// Source bytes come from dword-aligned LDS reads + v_alignbyte (byte-unaligned
// ds_read_b128 is much slower).
#pragma once
#include "kernels/device_common.hpp"

namespace pqk {
namespace dev {
namespace rc {

struct __attribute__((packed, aligned(1))) B16 { uint32_t x, y, z, w; };
struct __attribute__((packed, aligned(1))) B8 { uint32_t x, y; };
struct __attribute__((packed, aligned(1))) B4 { uint32_t x; };
struct __attribute__((packed, aligned(1))) B2 { uint16_t x; };

// 16 bytes at LDS byte address A of a dword array (20 readable bytes past A).
__device__ __forceinline__ uint4 lds16(const uint32_t* w, uint32_t A) {
    const uint32_t i = A >> 2, sh = A & 3u;
    const uint32_t w0 = w[i], w1 = w[i + 1], w2 = w[i + 2], w3 = w[i + 3], w4 = w[i + 4];
    return make_uint4(__builtin_amdgcn_alignbyte(w1, w0, sh), __builtin_amdgcn_alignbyte(w2, w1, sh),
                      __builtin_amdgcn_alignbyte(w3, w2, sh), __builtin_amdgcn_alignbyte(w4, w3, sh));
}

// Bytes [sa, sa + ln) of the LDS image `w` to d[0 .. ln).
__device__ __forceinline__ void copy_row(uint8_t* d, const uint32_t* w, uint32_t sa, uint32_t ln) {
    if (ln >= 16) {
        for (uint32_t x = 0; x + 16 < ln; x += 16) {
            const uint4 v = lds16(w, sa + x);
            *reinterpret_cast<B16*>(d + x) = B16{v.x, v.y, v.z, v.w};
        }
        const uint4 v = lds16(w, sa + ln - 16);
        *reinterpret_cast<B16*>(d + ln - 16) = B16{v.x, v.y, v.z, v.w};
    } else if (ln) {
        const uint4 v = lds16(w, sa);  // bytes 0 .. 15 of the row's source
        const uint32_t t = ln >= 8 ? ln - 8 : (ln >= 4 ? ln - 4 : (ln >= 2 ? ln - 2 : 0u));
        const uint4 u = lds16(w, sa + t);  // bytes t .. t + 15
        if (ln >= 8) {
            *reinterpret_cast<B8*>(d) = B8{v.x, v.y};
            *reinterpret_cast<B8*>(d + t) = B8{u.x, u.y};
        } else if (ln >= 4) {
            *reinterpret_cast<B4*>(d) = B4{v.x};
            *reinterpret_cast<B4*>(d + t) = B4{u.x};
        } else if (ln >= 2) {
            *reinterpret_cast<B2*>(d) = B2{static_cast<uint16_t>(v.x)};
            *reinterpret_cast<B2*>(d + t) = B2{static_cast<uint16_t>(u.x)};
        } else {
            d[0] = static_cast<uint8_t>(v.x);
        }
    }
}

// Bytes s[0 .. ln) (global memory, any alignment, >= 16 readable bytes past
// the row: image slots are zero padded) to d[0 .. ln), the same move shapes.
__device__ __forceinline__ void copy_row_g(uint8_t* d, const uint8_t* s, uint32_t ln) {
    if (ln >= 16) {
        for (uint32_t x = 0; x + 16 < ln; x += 16) *reinterpret_cast<B16*>(d + x) = *reinterpret_cast<const B16*>(s + x);
        *reinterpret_cast<B16*>(d + ln - 16) = *reinterpret_cast<const B16*>(s + ln - 16);
    } else if (ln >= 8) {
        const B8 a = *reinterpret_cast<const B8*>(s), b = *reinterpret_cast<const B8*>(s + ln - 8);
        *reinterpret_cast<B8*>(d) = a;
        *reinterpret_cast<B8*>(d + ln - 8) = b;
    } else if (ln >= 4) {
        const B4 a = *reinterpret_cast<const B4*>(s), b = *reinterpret_cast<const B4*>(s + ln - 4);
        *reinterpret_cast<B4*>(d) = a;
        *reinterpret_cast<B4*>(d + ln - 4) = b;
    } else if (ln >= 2) {
        const B2 a = *reinterpret_cast<const B2*>(s), b = *reinterpret_cast<const B2*>(s + ln - 2);
        *reinterpret_cast<B2*>(d) = a;
        *reinterpret_cast<B2*>(d + ln - 2) = b;
    } else if (ln) {
        d[0] = s[0];
    }
}

}  // namespace rc
}  // namespace dev
}  // namespace pqk
