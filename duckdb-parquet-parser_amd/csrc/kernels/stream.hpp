// stream.hpp — the serial parts of Parquet page decode on the scalar unit.
//
// Run headers of the hybrid RLE/bit-packed stream (rle_decoder.hpp:37-53,
// 76-95) and u32 length chains of PLAIN BYTE_ARRAY values
// (column_reader.cpp:249-253) form a serial dependency through a wave-uniform
// cursor.  Reading the page through the constant address space makes the
// compiler use SMEM (s_load_dword*) with the cursor in SGPRs: one scalar
// load and a handful of SALU ops per run header, no vector memory round trip
// and no vmcnt waits on the critical path.  Payloads sit 16-byte aligned in
// the device image with at least 16 zero bytes after them (capi.hip), so the
// 12-byte scalar reads never leave the allocation.
//
// RLE runs are expanded into LDS immediately (stores only, nothing waits on
// them); bit-packed runs are recorded and expanded afterwards, one value per
// lane, from the LDS copy of the page.
#pragma once
#include "kernels/device_common.hpp"

namespace pqk {
namespace dev {

typedef __attribute__((address_space(4))) const uint32_t cu32;

__device__ __forceinline__ uint32_t suni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }

// 8 bytes starting at byte `pos` of a 4-byte aligned buffer (pos uniform).
__device__ __forceinline__ uint64_t sload8(const uint8_t* base, uint32_t pos) {
    cu32* p = reinterpret_cast<cu32*>(reinterpret_cast<uintptr_t>(base)) + (pos >> 2);
    uint32_t a = p[0], b = p[1];
    uint64_t lo = (static_cast<uint64_t>(b) << 32) | a;
    uint32_t s = (pos & 3) * 8;
    if (s == 0) return lo;
    uint32_t c = p[2];
    return (lo >> s) | (static_cast<uint64_t>(c) << (64 - s));
}
__device__ __forceinline__ uint32_t sload_u32(const uint8_t* base, uint32_t pos) {
    return static_cast<uint32_t>(sload8(base, pos));
}

// A recorded bit-packed run: `count` values of `bw` bits starting at page
// bit `bit0`, for output slots [start, start + count).
struct LitRun {
    uint32_t start, count, bit0_lo, bit0_hi;
};

// Scalar state of one hybrid stream (rle_decoder.hpp member for member).
struct SRle {
    uint32_t base, size, pos, bw, repeat, literal, value, lit_start, lit_bit, lit_valid;
};

__device__ __forceinline__ void srle_init(SRle& r, uint32_t base, uint32_t size, uint32_t bw) {
    r.base = base; r.size = size; r.pos = 0; r.bw = bw; r.repeat = 0; r.literal = 0;
    r.value = 0; r.lit_start = 0; r.lit_bit = 0; r.lit_valid = 0;
}

// Walk the next `n` values of the stream.  RLE values go out through
// rle_out(j, v) (lanes j = lane, lane+64, ...); literal runs are appended to
// lits[] (LDS, uniform count nlits).  `flush` is called when lits is full.
// Returns 0 or PQ_ERR_UNSUPPORTED (outside the parity scope, see oracle).
template <class RleOut, class Flush>
__device__ int srle_walk(SRle& r, const uint8_t* page, uint32_t n, RleOut&& rle_out, LitRun* lits,
                         uint32_t& nlits, uint32_t lit_cap, Flush&& flush) {
    uint32_t done = 0;
    while (done < n) {
        if (r.repeat == 0 && r.literal == 0) {
            if (r.pos >= r.size) {  // exhausted: zero-fill (rle_decoder.hpp:20-23)
                for (uint32_t j = done + lane(); j < n; j += kWave) rle_out(j, 0u);
                return 0;
            }
            // read_varint32 (76-86): bounded by the stream size
            uint32_t ind = 0, shift = 0;
            for (;;) {
                uint64_t x = sload8(page, r.base + r.pos);
                uint32_t avail = min(8u, r.size - r.pos);
                uint32_t i = 0;
                bool end = false;
                for (; i < avail; i++) {
                    uint32_t b = static_cast<uint32_t>(x >> (8 * i)) & 0xFFu;
                    if (shift < 32) ind |= (b & 0x7Fu) << shift;
                    shift += 7;
                    if (!(b & 0x80u)) { end = true; i++; break; }
                }
                r.pos += i;
                if (end || r.pos >= r.size) break;
            }
            ind = suni(ind);
            if (ind & 1u) {  // literal run (41-46)
                r.literal = (ind >> 1) * 8u;
                r.lit_start = r.pos;
                r.lit_valid = 1;
                r.lit_bit = 0;
            } else {  // repeated run (48-50, 88-95)
                r.repeat = ind >> 1;
                uint32_t nb = min((r.bw + 7) / 8, r.size - r.pos);
                uint32_t v = nb ? static_cast<uint32_t>(sload8(page, r.base + r.pos)) : 0u;
                if (nb < 4) v &= (1u << (8 * nb)) - 1u;
                r.value = suni(v);
                r.pos += nb;
            }
        }
        if (r.bw > 64) return PQ_ERR_UNSUPPORTED;
        if (r.repeat > 0) {
            uint32_t k = min(r.repeat, n - done);
            for (uint32_t j = lane(); j < k; j += kWave) rle_out(done + j, r.value);
            r.repeat -= k;
            done += k;
        } else {
            // literal_count_ == 0 here is a zero-count run: the reference's
            // counter wraps and every later value comes from the literal cursor
            if (r.bw > 0 && !r.lit_valid) return PQ_ERR_UNSUPPORTED;
            bool wrapped = r.literal == 0;
            uint32_t k = wrapped ? n - done : min(r.literal, n - done);
            if (r.bw == 0) {
                for (uint32_t j = lane(); j < k; j += kWave) rle_out(done + j, 0u);
            } else {
                if (nlits == lit_cap) { flush(); nlits = 0; }
                uint64_t bit0 = static_cast<uint64_t>(r.base + r.lit_start) * 8u + r.lit_bit;
                if (lane() == 0)
                    lits[nlits] = LitRun{done, k, static_cast<uint32_t>(bit0), static_cast<uint32_t>(bit0 >> 32)};
                nlits++;
            }
            bool finishes = !wrapped && k == r.literal;
            r.lit_bit += k * r.bw;
            r.literal -= k;
            if (finishes && r.bw > 0) r.pos = r.lit_start + (r.lit_bit + 7) / 8;  // 66-72
            done += k;
        }
    }
    return 0;
}

// Expand recorded literal runs: out(slot, value) from the LDS page copy.
template <class Out>
__device__ __forceinline__ void expand_lits(const LitRun* lits, uint32_t nlits, const uint32_t* words,
                                            uint32_t size, uint32_t bw, Out&& out) {
    __builtin_amdgcn_wave_barrier();
    for (uint32_t r = 0; r < nlits; r++) {
        const LitRun L = lits[r];
        const uint64_t bit0 = (static_cast<uint64_t>(L.bit0_hi) << 32) | L.bit0_lo;
        for (uint32_t j = lane(); j < L.count; j += kWave)
            out(L.start + j, lds_bits(words, size, bit0 + static_cast<uint64_t>(j) * bw, bw));
    }
    __builtin_amdgcn_wave_barrier();
}

}  // namespace dev
}  // namespace pqk
