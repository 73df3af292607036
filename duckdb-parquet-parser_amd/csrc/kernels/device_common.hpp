// device_common.hpp — device helpers shared by the decode and regex kernels:
// the page byte source (LDS-staged words or the HBM image, zero past the page
// end) and the hybrid RLE/bit-packed stream state machine, a restatement of
// the reference's RleDecoder (include/reader/rle_decoder.hpp:6-108).
#pragma once
#include "kernels/kernels.hpp"
#include "pq_gpu.h"

namespace pqk {
namespace dev {

// Timing ablations and diagnostics (the `fused_debug` / `regex_debug` option
// bits that scripts/ab_opts.py and scripts/regex_ablate.py set) exist only in
// the probe build (`make PROBES=1 OBJDIR=... LIB=...`, loaded through AB_PKG):
// in the shipped library kProbes is false and every such branch folds away.
#ifndef PQ_PROBES
#define PQ_PROBES 0
#endif
constexpr bool kProbes = PQ_PROBES != 0;
__device__ __forceinline__ bool probe(int debug, int bits) { return kProbes && (debug & bits) != 0; }

__device__ __forceinline__ uint32_t lane() { return __lane_id(); }

// ── page byte source: LDS-staged words, or the HBM image (zero past end) ──
struct Src {
    const uint32_t* lds;  // staged payload words, or nullptr
    const uint8_t* g;     // payload start in the device byte image
    uint32_t size;        // payload bytes
};

__device__ __forceinline__ uint32_t gword(const uint8_t* g, uint64_t b) {
    uintptr_t a = reinterpret_cast<uintptr_t>(g) + b;
    const uint32_t* ap = reinterpret_cast<const uint32_t*>(a & ~static_cast<uintptr_t>(3));
    return __builtin_amdgcn_alignbyte(ap[1], ap[0], static_cast<uint32_t>(a & 3));
}

__device__ __forceinline__ uint32_t src_word(const Src& s, uint64_t wi) {
    uint64_t b = wi * 4;
    if (b >= s.size) return 0u;
    uint32_t w = s.lds ? s.lds[wi] : gword(s.g, b);
    uint64_t rem = s.size - b;
    if (rem < 4) w &= (1u << (8 * rem)) - 1u;
    return w;
}
__device__ __forceinline__ uint32_t src_byte(const Src& s, uint32_t p) {
    return (src_word(s, p >> 2) >> ((p & 3) * 8)) & 0xFFu;
}
__device__ __forceinline__ uint32_t src_u32(const Src& s, uint32_t p) {
    uint32_t lo = src_word(s, p >> 2), hi = src_word(s, (p >> 2) + 1);
    return __builtin_amdgcn_alignbyte(hi, lo, p & 3);
}
// low min(bw, 32) bits of the bit field starting at page bit `b`
__device__ __forceinline__ uint32_t src_bits(const Src& s, uint64_t b, uint32_t bw) {
    uint64_t wi = b >> 5;
    uint64_t v = (static_cast<uint64_t>(src_word(s, wi + 1)) << 32) | src_word(s, wi);
    uint32_t x = static_cast<uint32_t>(v >> (b & 31));
    return bw >= 32 ? x : (x & ((1u << bw) - 1u));
}

// LDS-only readers (no generic-pointer branch, so they always lower to DS ops).
// `words` holds `size` bytes of a page; bytes past `size` read as zero.
__device__ __forceinline__ uint32_t lds_word(const uint32_t* words, uint32_t size, uint64_t wi) {
    uint64_t b = wi * 4;
    if (b >= size) return 0u;
    uint32_t w = words[wi];
    uint64_t rem = size - b;
    if (rem < 4) w &= (1u << (8 * rem)) - 1u;
    return w;
}
__device__ __forceinline__ uint32_t lds_bits(const uint32_t* words, uint32_t size, uint64_t b, uint32_t bw) {
    uint64_t wi = b >> 5;
    uint64_t v = (static_cast<uint64_t>(lds_word(words, size, wi + 1)) << 32) | lds_word(words, size, wi);
    uint32_t x = static_cast<uint32_t>(v >> (b & 31));
    return bw >= 32 ? x : (x & ((1u << bw) - 1u));
}

// 8 bytes at LDS byte address a (the staged page has >= 16 readable bytes
// past its end).
__device__ __forceinline__ uint64_t lds_u64(const uint32_t* w, uint32_t a) {
    const uint32_t i = a >> 2, sh = a & 3;
    const uint32_t d0 = w[i], d1 = w[i + 1], d2 = w[i + 2];
    const uint32_t lo = __builtin_amdgcn_alignbyte(d1, d0, sh);
    const uint32_t hi = __builtin_amdgcn_alignbyte(d2, d1, sh);
    return (static_cast<uint64_t>(hi) << 32) | lo;
}

// Stage a page's payload into this wave's LDS words (zero-filled tail word).
__device__ inline void stage_page(uint32_t* lds, const uint8_t* g, uint32_t size) {
    uint32_t nw = (size + 3) / 4;
    for (uint32_t i = lane(); i < nw; i += kWave) {
        uint32_t w = gword(g, static_cast<uint64_t>(i) * 4);
        uint32_t rem = size - i * 4;
        if (rem < 4) w &= (1u << (8 * rem)) - 1u;
        lds[i] = w;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
}

// ── bulk copies: kU loads in flight per thread ────────────────────────────
// dst[i] = f(src[i]) for i = t, t + nt, ... < n.  A plain strided loop makes
// each iteration wait for its own load before the next is issued (one HBM
// latency per iteration, vmcnt(0) before the LDS store); batching kU loads
// before their stores pays one latency per batch.
template <int kU = 8, class D, class S, class F>
__device__ __forceinline__ void copy_map(D* __restrict__ dst, const S* __restrict__ src, uint32_t n, uint32_t t,
                                         uint32_t nt, F&& f) {
    for (uint32_t i0 = t; i0 < n; i0 += kU * nt) {
        S v[kU];
#pragma unroll
        for (int u = 0; u < kU; u++) {
            const uint32_t i = i0 + static_cast<uint32_t>(u) * nt;
            if (i < n) v[u] = src[i];
        }
#pragma unroll
        for (int u = 0; u < kU; u++) {
            const uint32_t i = i0 + static_cast<uint32_t>(u) * nt;
            if (i < n) dst[i] = f(v[u]);
        }
    }
}
template <int kU = 8, class T>
__device__ __forceinline__ void copy_blocks(T* __restrict__ dst, const T* __restrict__ src, uint32_t n, uint32_t t,
                                            uint32_t nt) {
    copy_map<kU>(dst, src, n, t, nt, [](const T& x) { return x; });
}

// ── hybrid RLE / bit-packed decoder: rle_decoder.hpp state machine ─────────
struct Rle {
    uint32_t base;      // stream start (page byte offset)
    uint32_t size;      // size_
    uint32_t pos;       // pos_
    uint32_t bw;        // bit_width_
    uint32_t repeat;    // repeat_count_
    uint32_t literal;   // literal_count_ (u32 wrap kept)
    uint32_t value;     // low 32 bits of current_value_
    uint32_t lit_start; // literal_pos_ - data_
    uint32_t lit_bit;   // literal_bit_offset_
    uint32_t lit_valid; // literal_pos_ != nullptr
};

__device__ __forceinline__ void rle_init(Rle& r, uint32_t base, uint32_t size, uint32_t bw) {
    r.base = base; r.size = size; r.pos = 0; r.bw = bw; r.repeat = 0; r.literal = 0;
    r.value = 0; r.lit_start = 0; r.lit_bit = 0; r.lit_valid = 0;
}

// Produce the next n values of the stream; out(j, v) for j in [0, n) spread
// over the lanes.  Wave-uniform control flow.
template <class F>
__device__ int rle_decode(Rle& r, const Src& s, uint32_t n, F&& out) {
    uint32_t done = 0;
    while (done < n) {
        if (r.repeat == 0 && r.literal == 0) {
            if (r.pos >= r.size) {  // exhausted: zero-fill (rle_decoder.hpp:20-23)
                for (uint32_t j = done + lane(); j < n; j += kWave) out(j, 0u);
                return 0;
            }
            uint32_t ind = 0, shift = 0;  // read_varint32 (76-86)
            while (r.pos < r.size) {
                uint32_t b = src_byte(s, r.base + r.pos);
                r.pos++;
                if (shift < 32) ind |= (b & 0x7Fu) << shift;
                if (!(b & 0x80u)) break;
                shift += 7;
            }
            if (ind & 1u) {  // literal run (41-46)
                r.literal = (ind >> 1) * 8u;
                r.lit_start = r.pos;
                r.lit_valid = 1;
                r.lit_bit = 0;
            } else {  // repeated run (48-50, read_fixed_width_value 88-95)
                r.repeat = ind >> 1;
                uint32_t nb = (r.bw + 7) / 8, v = 0;
                for (uint32_t i = 0; i < nb && r.pos < r.size; i++) {
                    uint32_t b = src_byte(s, r.base + r.pos);
                    r.pos++;
                    if (i < 4) v |= b << (8 * i);
                }
                r.value = v;
            }
        }
        if (r.bw > 64) return PQ_ERR_UNSUPPORTED;
        if (r.repeat > 0) {
            uint32_t k = min(r.repeat, n - done);
            for (uint32_t j = lane(); j < k; j += kWave) out(done + j, r.value);
            r.repeat -= k;
            done += k;
        } else {
            // literal_count_ == 0 here means a zero-count run: the reference's
            // counter wraps and every later value is read from the literal cursor.
            if (r.bw > 0 && !r.lit_valid) return PQ_ERR_UNSUPPORTED;
            bool wrapped = r.literal == 0;
            uint32_t k = wrapped ? n - done : min(r.literal, n - done);
            uint64_t bit0 = static_cast<uint64_t>(r.base + r.lit_start) * 8u + r.lit_bit;
            for (uint32_t j = lane(); j < k; j += kWave)
                out(done + j, r.bw ? src_bits(s, bit0 + static_cast<uint64_t>(j) * r.bw, r.bw) : 0u);
            bool finishes = !wrapped && k == r.literal;
            r.lit_bit += k * r.bw;
            r.literal -= k;
            if (finishes && r.bw > 0) r.pos = r.lit_start + (r.lit_bit + 7) / 8;  // 66-72
            done += k;
        }
    }
    return 0;
}

__device__ __forceinline__ uint32_t level_bw(int32_t m) {  // column_reader.cpp:270-276
    uint32_t bw = 0;
    while (m > 0) { bw++; m >>= 1; }
    return bw;
}

__device__ __forceinline__ void set_err(DevErr* e, int32_t* any, int code, uint32_t pos, uint32_t need,
                                        uint32_t size) {
    if (lane() == 0) {
        e->code = code;
        e->pos = static_cast<int32_t>(pos);
        e->need = static_cast<int32_t>(need);
        e->size = static_cast<int32_t>(size);
        atomicOr(any, 1);
    }
}


// ── wave primitives on DPP (no LDS round trip; gfx9 row_bcast15/31) ───────
template <int kCtrl, int kRowMask = 0xf>
__device__ __forceinline__ uint32_t dpp0(uint32_t v) {
    return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), kCtrl, kRowMask, 0xf, true));
}

// Inclusive wave prefix sum / max of a u32 (all 64 lanes active).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    v += dpp0<0x111>(v);        // row_shr:1
    v += dpp0<0x112>(v);        // row_shr:2
    v += dpp0<0x114>(v);        // row_shr:4
    v += dpp0<0x118>(v);        // row_shr:8
    v += dpp0<0x142, 0xa>(v);   // row_bcast:15 -> rows 1, 3
    v += dpp0<0x143, 0xc>(v);   // row_bcast:31 -> rows 2, 3
    return v;
}
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t v) {
    v = max(v, dpp0<0x111>(v));
    v = max(v, dpp0<0x112>(v));
    v = max(v, dpp0<0x114>(v));
    v = max(v, dpp0<0x118>(v));
    v = max(v, dpp0<0x142, 0xa>(v));
    v = max(v, dpp0<0x143, 0xc>(v));
    return v;
}
__device__ __forceinline__ uint32_t bcast_last(uint32_t v) {
    return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), kWave - 1));
}
__device__ __forceinline__ uint32_t popc_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(m >> 32),
                                     __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(m), 0u));
}

}  // namespace dev
}  // namespace pqk
