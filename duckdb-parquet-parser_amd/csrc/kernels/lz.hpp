// lz.hpp — the SNAPPY and LZ4 command-stream parsers of the codec pass
// (SURVEY §8f rank 4 widening; outside the reference's parity scope: the
// reference rejects every codec, column_reader.cpp:13-15).
//
// Written once over four small interfaces, like zstd.hpp, so that the same
// parse runs in k_codec (a wavefront, wave-uniformly) and in the host harness
// the sanitizer tests drive (tools/lz_check.cpp):
//   I     the page input: ensure(p, k) (bytes [p, p + k) readable), byte(p),
//         u32be(p)
//   Win   command headers: Win{&I}; need(p, k), byte(q), u16le(q), u32le(q),
//         and Win::uni(v), the wave-uniform copy of a value (k_codec's TagWin:
//         256 input bytes in a register, v_readfirstlane)
//   O     the output: st, op, vbase, lit(I, p, n) (input bytes [p, p + n)),
//         copy(d, n) (n bytes from distance d); O checks room and distance
//         and sets st (k_codec's QSink / Out; the harness restates QSink's)
//   status ST_OK / ST_CORRUPT / ST_SIZE, as k_codec's
//   SNAPPY   format_description.txt of google/snappy: a varint length, then
//            tagged literals and copies (1-, 2- and 4-byte offsets)
//   LZ4      one block (LZ4_RAW, codec 7), or Hadoop framing (codec 5):
//            [u32 BE raw][u32 BE packed][block] repeated
#pragma once
#include <cstdint>

#ifndef LZ_HD
#define LZ_HD __device__ __forceinline__
#endif
#ifndef PQ_CODEC_PARSE_ONLY  // timing probe: the command stream parsed, nothing executed
#define PQ_CODEC_PARSE_ONLY 0
#endif

namespace pqlz {

enum : uint32_t { ST_OK = 0, ST_CORRUPT = 1, ST_SIZE = 2 };

template <class Win, class InX, class OutT>
LZ_HD void snappy(InX& I, OutT& O, uint32_t p, uint32_t end, uint32_t expect) {
    uint32_t ulen = 0;
    I.ensure(p, 8);
    for (uint32_t k = 0;; k++) {
        if (k == 5 || p >= end) { O.st = ST_CORRUPT; return; }
        const uint32_t b = I.byte(p++);
        ulen |= (b & 0x7Fu) << (7 * k);
        if (!(b & 0x80u)) break;
    }
    if (ulen != expect) { O.st = ST_SIZE; return; }
    Win T{&I};
    while (p < end && O.st == ST_OK) {
        T.need(p, 5);  // the longest header: a tag and four bytes
        const uint32_t t = T.byte(p);
        const uint32_t ty = t & 3u;
        if (ty == 0) {
            uint32_t n = (t >> 2) + 1;
            p += 1;
            if (n > 60) {
                const uint32_t nb = n - 60;
                const uint32_t x = T.u32le(p);
                n = (nb == 4 ? x : (x & ((1u << (8 * nb)) - 1u))) + 1;
                p += nb;
            }
            n = Win::uni(n);
            if (p > end || n > end - p || n == 0) { O.st = ST_CORRUPT; return; }
#if PQ_CODEC_PARSE_ONLY
            O.op += n;
#else
            O.lit(I, p, n);
#endif
            p += n;
        } else {
            uint32_t n, d;
            if (ty == 1) {
                n = 4 + ((t >> 2) & 7u);
                d = ((t >> 5) << 8) | T.byte(p + 1);
                p += 2;
            } else if (ty == 2) {
                n = (t >> 2) + 1;
                d = T.u16le(p + 1);
                p += 3;
            } else {
                n = (t >> 2) + 1;
                d = T.u32le(p + 1);
                p += 5;
            }
            if (p > end) { O.st = ST_CORRUPT; return; }
#if PQ_CODEC_PARSE_ONLY
            O.op += Win::uni(n);
#else
            O.copy(Win::uni(d), Win::uni(n));
#endif
        }
    }
    if (O.st == ST_OK && O.op - O.vbase != expect) O.st = ST_SIZE;
}

template <class Win, class InX, class OutT>
LZ_HD void lz4_block(InX& I, OutT& O, uint32_t p, uint32_t end) {
    Win T{&I};
    for (;;) {
        if (p >= end) { O.st = ST_CORRUPT; return; }
        T.need(p, 1);
        const uint32_t tok = T.byte(p++);
        uint32_t n = tok >> 4;
        if (n == 15) {
            uint32_t b;
            do {
                if (p >= end) { O.st = ST_CORRUPT; return; }
                T.need(p, 1);
                b = T.byte(p++);
                n += b;
            } while (b == 255);
        }
        n = Win::uni(n);
        if (n > end - p) { O.st = ST_CORRUPT; return; }
        if (n) O.lit(I, p, n);
        if (O.st != ST_OK) return;
        p += n;
        if (p == end) return;  // the last sequence holds literals only
        if (end - p < 2) { O.st = ST_CORRUPT; return; }
        T.need(p, 2);
        const uint32_t d = T.u16le(p);
        p += 2;
        uint32_t m = tok & 15u;
        if (m == 15) {
            uint32_t b;
            do {
                if (p >= end) { O.st = ST_CORRUPT; return; }
                T.need(p, 1);
                b = T.byte(p++);
                m += b;
            } while (b == 255);
        }
        m = Win::uni(m);
        O.copy(d, m + 4);
        if (O.st != ST_OK) return;
    }
}

template <class Win, class InX, class OutT>
LZ_HD void lz4_hadoop(InX& I, OutT& O, uint32_t p, uint32_t end) {
    while (p < end && O.st == ST_OK) {
        if (end - p < 8) { O.st = ST_CORRUPT; return; }
        I.ensure(p, 8);
        const uint32_t raw = Win::uni(I.u32be(p)), packed = Win::uni(I.u32be(p + 4));
        p += 8;
        if (packed > end - p) { O.st = ST_CORRUPT; return; }
        const uint32_t o0 = O.op;
        lz4_block<Win>(I, O, p, p + packed);
        if (O.st == ST_OK && O.op - o0 != raw) O.st = ST_SIZE;
        p += packed;
    }
}

}  // namespace pqlz
