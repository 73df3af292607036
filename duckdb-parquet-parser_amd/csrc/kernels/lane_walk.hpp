// lane_walk.hpp — one lane walks one page's hybrid RLE/bit-packed stream.
//
// The reference's RleDecoder state machine (include/reader/rle_decoder.hpp:
// 6-108) restated as plain per-thread code, so that a wavefront advances 64
// pages' streams with each instruction (dict_batch.hip, regex.hip).  Exact
// semantics, including the zero-count-run wrap of literal_count_, zero fill on
// exhaustion and pos_ advancing only at the end of a literal run.
#pragma once
#include "kernels/device_common.hpp"

namespace pqk {
namespace dev {

// Stream at page bytes [base, base + size); rd8(a) returns the 8 page bytes
// starting at page byte a (bytes past the stream are masked here).
struct LRle {
    uint32_t base, size, pos, bw, repeat, literal, value, lit_start, lit_bit, lit_valid;
};

__device__ __forceinline__ LRle lrle(uint32_t base, uint32_t size, uint32_t bw) {
    return LRle{base, size, 0, bw, 0, 0, 0, 0, 0, 0};
}

// Produces `need` values as segments emit(kind, count, arg): kind 0 = `count`
// copies of value `arg`; kind 1 = `count` bit-packed values starting at page
// bit `arg`.  Returns 0 or PQ_ERR_UNSUPPORTED (bw > 64, or a zero-count run
// before any literal run: outside the parity scope).
template <class Rd8, class F>
__device__ int lane_rle(LRle& r, Rd8&& rd8, uint32_t need, F&& emit) {
    uint32_t done = 0;
    while (done < need) {
        if (r.repeat == 0 && r.literal == 0) {
            if (r.pos >= r.size) {  // exhausted: zeros (rle_decoder.hpp:20-23)
                emit(0u, need - done, 0u);
                return 0;
            }
            uint32_t ind = 0, shift = 0;  // read_varint32 (76-86), bounded by the stream
            for (;;) {
                const uint64_t x = rd8(r.base + r.pos);
                const uint32_t avail = min(8u, r.size - r.pos);
                uint32_t i = 0;
                bool end = false;
                for (; i < avail; i++) {
                    const uint32_t b = static_cast<uint32_t>(x >> (8 * i)) & 0xFFu;
                    if (shift < 32) ind |= (b & 0x7Fu) << shift;
                    shift += 7;
                    if (!(b & 0x80u)) { end = true; i++; break; }
                }
                r.pos += i;
                if (end || r.pos >= r.size) break;
            }
            if (ind & 1u) {  // literal run (41-46)
                r.literal = (ind >> 1) * 8u;
                r.lit_start = r.pos;
                r.lit_valid = 1;
                r.lit_bit = 0;
            } else {  // repeated run (48-50, 88-95)
                r.repeat = ind >> 1;
                const uint32_t nb = min((r.bw + 7) / 8, r.size - r.pos);
                uint32_t v = nb ? static_cast<uint32_t>(rd8(r.base + r.pos)) : 0u;
                if (nb < 4) v &= (1u << (8 * nb)) - 1u;
                r.value = v;
                r.pos += nb;
            }
        }
        if (r.bw > 64) return PQ_ERR_UNSUPPORTED;
        if (r.repeat > 0) {
            const uint32_t k = min(r.repeat, need - done);
            emit(0u, k, r.value);
            r.repeat -= k;
            done += k;
        } else {
            // literal_count_ == 0: a zero-count run; the reference's counter
            // wraps and every later value comes from the literal cursor
            if (r.bw > 0 && !r.lit_valid) return PQ_ERR_UNSUPPORTED;
            const bool wrapped = r.literal == 0;
            const uint32_t k = wrapped ? need - done : min(r.literal, need - done);
            if (r.bw == 0) emit(0u, k, 0u);
            else emit(1u, k, (r.base + r.lit_start) * 8u + r.lit_bit);
            const bool finishes = !wrapped && k == r.literal;
            r.lit_bit += k * r.bw;
            r.literal -= k;
            if (finishes && r.bw > 0) r.pos = r.lit_start + (r.lit_bit + 7) / 8;  // 66-72
            done += k;
        }
    }
    return 0;
}

// 8 bytes at page byte a of a 16-byte aligned page slot in global memory
// (slots carry >= 16 zero bytes after the payload, capi.hip).
__device__ __forceinline__ uint64_t gld8(const uint8_t* page, uint32_t a) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(page) + (a >> 2);
    const uint32_t d0 = w[0], d1 = w[1], d2 = w[2], sh = a & 3;
    return (static_cast<uint64_t>(__builtin_amdgcn_alignbyte(d2, d1, sh)) << 32) | __builtin_amdgcn_alignbyte(d1, d0, sh);
}
// low min(bw, 32) bits at page bit b of a page of `size` bytes (zero past it)
__device__ __forceinline__ uint32_t gbits(const uint8_t* page, uint32_t size, uint64_t b, uint32_t bw) {
    const uint32_t a = static_cast<uint32_t>(b >> 3);
    if (a >= size) return 0u;
    uint64_t x = gld8(page, a);
    if (size - a < 8) x &= (1ull << (8 * (size - a))) - 1ull;
    const uint32_t v = static_cast<uint32_t>(x >> (b & 7));
    return bw >= 32 ? v : (v & ((1u << bw) - 1u));
}

}  // namespace dev
}  // namespace pqk
