// deflate.hpp — DEFLATE (RFC 1951) in GZIP members (RFC 1952) or one zlib
// stream (RFC 1950) for the codec pass (SURVEY §8f rank 4 widening; outside
// the reference's parity scope: the reference rejects every codec,
// column_reader.cpp:13-15).
//
// Written once, like zstd.hpp and lz.hpp, so that the same decoder runs in
// k_codec (one wavefront per page: table builds spread over the lanes, symbol
// decode wave-uniform) and in the host harness the sanitizer tests drive
// (tools/gzip_check.cpp).  Template parameters:
//   W     the wave: W::lane(), W::kWave, W::sync() (a wave barrier with LDS
//         ordering), W::uni(v) (the wave-uniform copy), W::bitrev(v); the host
//         harness runs one lane (lane 0, kWave 1)
//   LdsT  the tables: lens[320], sym[320], code[320], cnt[2][16], nxt[16],
//         offs[16], scratch[4], lt / dt[1 << kFast]
//   InX   the input: ensure(p, k), byte(p), u16le(p), u32le(p)
//   OutT  the output: st, op, put1(b), lit(I, p, n), copy(d, n), the running
//         CRC-32 of GZIP members (crc_on, crc, crc_pos, crc_keep(),
//         crc_upto(to), kCrcSlack)
// Huffman symbols decode through kFast-bit lookup tables, longer codes by the
// canonical bit-serial walk.
#pragma once
#include <cstdint>

#ifndef DF_HD
#define DF_HD __device__ __forceinline__
#endif
#ifndef DF_CONST
#define DF_CONST __constant__
#endif

namespace pqinf {

enum : uint32_t { ST_OK = 0, ST_CORRUPT = 1, ST_SIZE = 2 };
constexpr uint32_t kFast = 10;  // Huffman lookup bits

DF_CONST uint16_t kLBase[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31,
                                    35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
DF_CONST uint8_t kLExt[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
DF_CONST uint16_t kDBase[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129,
                                    193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
DF_CONST uint8_t kDExt[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
DF_CONST uint8_t kClOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

template <class InX>
struct Bits {
    uint64_t buf;
    uint32_t cnt, p, end;
    uint32_t pad;  // zero bytes supplied past the input end (a valid stream never consumes them)
    DF_HD void need(InX& I, uint32_t n) {
        while (cnt < n) {
            if (p >= end) {
                pad++;
                cnt += 8;
                continue;
            }
            I.ensure(p, 4);
            const uint32_t k = end - p < 4u ? end - p : 4u;
            uint32_t v = I.u32le(p);
            if (k < 4) v &= (1u << (8 * k)) - 1u;
            buf |= static_cast<uint64_t>(v) << cnt;
            cnt += 8 * k;
            p += k;
        }
    }
    DF_HD uint32_t peek(uint32_t n) const { return static_cast<uint32_t>(buf) & ((1u << n) - 1u); }
    DF_HD void drop(uint32_t n) { buf >>= n; cnt -= n; }
    DF_HD uint32_t take(InX& I, uint32_t n) {
        if (n == 0) return 0;
        need(I, n);
        const uint32_t v = peek(n);
        drop(n);
        return v;
    }
    // bits consumed past the input end
    DF_HD bool overrun() const {
        return 8ull * (static_cast<uint64_t>(p) + pad) - cnt > 8ull * end;
    }
    // byte position of the next unread bit (after dropping to a byte
    // boundary); > end when the stream consumed bits it does not have
    DF_HD uint32_t align_byte() {
        drop(cnt & 7u);
        const uint32_t q = p + pad - cnt / 8;
        buf = 0;
        cnt = 0;
        pad = 0;
        p = q;
        return q;
    }
};

// Canonical Huffman code over lens[base, base + n): counts, codes, symbols
// in code order, and the kFast-bit lookup table.  Returns false for an
// over-subscribed code.
template <class W, class LdsT>
DF_HD bool build_code(LdsT& L, int which, uint32_t base, uint32_t n, uint16_t* table) {
    uint16_t* cnt = L.cnt[which];
    for (uint32_t i = W::lane(); i < 16; i += W::kWave) cnt[i] = 0;
    W::sync();
    if (W::lane() == 0) {
        for (uint32_t s = 0; s < n; s++) cnt[L.lens[base + s]]++;
        cnt[0] = 0;
        uint16_t* next = L.nxt;
        uint16_t* offs = L.offs;
        int32_t left = 1;
        uint32_t code = 0, idx = 0;
        bool bad = false;
        for (uint32_t l = 1; l < 16; l++) {
            left = left * 2 - cnt[l];  // (a multiply: left may be negative, and a left shift of it is undefined)
            bad |= left < 0;
            code = (code + (l > 1 ? cnt[l - 1] : 0u)) << 1;
            next[l] = static_cast<uint16_t>(code);
            offs[l] = static_cast<uint16_t>(idx);
            idx += cnt[l];
        }
        for (uint32_t s = 0; s < n; s++) {
            const uint32_t l = L.lens[base + s];
            if (l) {
                L.code[base + s] = next[l]++;
                L.sym[base + offs[l]++] = static_cast<uint16_t>(s);
            }
        }
        L.scratch[which] = bad ? 1u : 0u;
    }
    for (uint32_t i = W::lane(); i < (1u << kFast); i += W::kWave) table[i] = 0;
    W::sync();
    for (uint32_t s = W::lane(); s < n; s += W::kWave) {
        const uint32_t l = L.lens[base + s];
        if (l == 0 || l > kFast) continue;
        const uint32_t rev = W::bitrev(L.code[base + s]) >> (32 - l);
        const uint16_t e = static_cast<uint16_t>((s << 4) | l);
        for (uint32_t k = 0; k < (1u << (kFast - l)); k++) table[rev | (k << l)] = e;
    }
    W::sync();
    return W::uni(L.scratch[which]) == 0;
}

// One Huffman symbol: the lookup table, else the canonical bit-serial walk.
template <class W, class LdsT, class InX>
DF_HD int32_t decode_sym(LdsT& L, InX& I, Bits<InX>& B, const uint16_t* table, int which, uint32_t base) {
    B.need(I, 15);
    const uint32_t e = W::uni(table[B.peek(kFast)]);
    if (e & 15u) {
        B.drop(e & 15u);
        return static_cast<int32_t>(e >> 4);
    }
    const uint16_t* cnt = L.cnt[which];
    int32_t code = 0, first = 0, index = 0;
    for (uint32_t l = 1; l < 16; l++) {
        code |= static_cast<int32_t>(B.peek(1));
        B.drop(1);
        const int32_t c = cnt[l];
        if (code - c < first) return static_cast<int32_t>(W::uni(L.sym[base + static_cast<uint32_t>(index + code - first)]));
        index += c;
        first = (first + c) << 1;
        code <<= 1;
    }
    return -1;
}

template <class W, class LdsT, class InX, class OutT>
DF_HD void inflate(LdsT& L, InX& I, OutT& O, Bits<InX>& B) {
    for (;;) {
        const uint32_t fin = B.take(I, 1);
        const uint32_t ty = B.take(I, 2);
        if (ty == 0) {  // stored
            uint32_t q = B.align_byte();
            if (q > B.end || B.end - q < 4) { O.st = ST_CORRUPT; return; }
            I.ensure(q, 4);
            const uint32_t n = W::uni(I.u16le(q)), nn = W::uni(I.u16le(q + 2));
            q += 4;
            if ((n ^ 0xFFFFu) != nn || n > B.end - q) { O.st = ST_CORRUPT; return; }
            for (uint32_t d = 0; d < n; d += O.kCrcSlack) {  // pieces of <= kCrcSlack bytes, CRC kept up
                O.crc_keep();
                O.lit(I, q + d, n - d < O.kCrcSlack ? n - d : O.kCrcSlack);
                if (O.st != ST_OK) return;
            }
            B.p = q + n;
        } else if (ty == 1 || ty == 2) {
            uint32_t nl = 288, nd = 30;
            if (ty == 1) {
                for (uint32_t s = W::lane(); s < 320; s += W::kWave)
                    L.lens[s] = s < 144 ? 8 : (s < 256 ? 9 : (s < 280 ? 7 : (s < 288 ? 8 : 5)));
                W::sync();
            } else {
                nl = B.take(I, 5) + 257;
                nd = B.take(I, 5) + 1;
                const uint32_t nc = B.take(I, 4) + 4;
                if (nl > 286 || nd > 30) { O.st = ST_CORRUPT; return; }
                // code-length code (lengths in kClOrder), built in the distance slots
                for (uint32_t s = W::lane(); s < 19; s += W::kWave) L.lens[288 + s] = 0;
                W::sync();
                for (uint32_t k = 0; k < nc; k++) {
                    const uint32_t v = B.take(I, 3);
                    if (W::lane() == 0) L.lens[288 + kClOrder[k]] = static_cast<uint8_t>(v);
                }
                W::sync();
                if (!build_code<W>(L, 1, 288, 19, L.dt)) { O.st = ST_CORRUPT; return; }
                uint32_t i = 0, prev = 0;
                while (i < nl + nd) {
                    const int32_t sy = decode_sym<W>(L, I, B, L.dt, 1, 288);
                    uint32_t rep = 1, val = 0;
                    if (sy < 0) { O.st = ST_CORRUPT; return; }
                    // code 16 repeats the last length WRITTEN, zeros of a 17/18 run
                    // included (RFC 1951 3.2.7; zlib's lens[have - 1])
                    if (sy < 16) {
                        val = static_cast<uint32_t>(sy);
                    } else if (sy == 16) {
                        if (i == 0) { O.st = ST_CORRUPT; return; }
                        val = prev;
                        rep = 3 + B.take(I, 2);
                    } else if (sy == 17) {
                        rep = 3 + B.take(I, 3);
                    } else {
                        rep = 11 + B.take(I, 7);
                    }
                    prev = val;
                    if (i + rep > nl + nd) { O.st = ST_CORRUPT; return; }
                    // lengths i .. i + rep: litlen [0, nl) -> lens[0 ..], dist -> lens[288 ..] (after the
                    // code-length table is no longer needed: written into a staging copy first)
                    for (uint32_t k = W::lane(); k < rep; k += W::kWave) {
                        const uint32_t j = i + k;
                        // the code-length code lives in lens[288, 307): distance lengths go to
                        // sym[] (free until build_code) and are moved after the loop
                        if (j < nl) L.lens[j] = static_cast<uint8_t>(val);
                        else L.sym[j - nl] = static_cast<uint16_t>(val);
                    }
                    W::sync();
                    i += rep;
                }
                for (uint32_t s = W::lane(); s < 288; s += W::kWave)
                    if (s >= nl) L.lens[s] = 0;
                for (uint32_t s = W::lane(); s < 32; s += W::kWave) L.lens[288 + s] = s < nd ? static_cast<uint8_t>(L.sym[s]) : 0;
                W::sync();
                if (L.lens[256] == 0) { O.st = ST_CORRUPT; return; }
            }
            if (!build_code<W>(L, 0, 0, 288, L.lt) || !build_code<W>(L, 1, 288, 32, L.dt)) {
                O.st = ST_CORRUPT;
                return;
            }
            for (;;) {
                O.crc_keep();  // a symbol adds <= 258 bytes
                const int32_t sy = decode_sym<W>(L, I, B, L.lt, 0, 0);
                if (sy < 0 || sy > 285) { O.st = ST_CORRUPT; return; }
                if (sy < 256) {
                    O.put1(static_cast<uint32_t>(sy));
                } else if (sy == 256) {
                    break;
                } else {
                    const uint32_t li = static_cast<uint32_t>(sy) - 257;
                    const uint32_t n = kLBase[li] + B.take(I, kLExt[li]);
                    const int32_t ds = decode_sym<W>(L, I, B, L.dt, 1, 288);
                    if (ds < 0 || ds > 29) { O.st = ST_CORRUPT; return; }
                    const uint32_t d = kDBase[ds] + B.take(I, kDExt[ds]);
                    W::sync();
                    O.copy(W::uni(d), W::uni(n));
                }
                if (O.st != ST_OK || B.overrun()) {
                    if (O.st == ST_OK) O.st = ST_CORRUPT;
                    return;
                }
            }
            W::sync();
        } else {
            O.st = ST_CORRUPT;
            return;
        }
        if (O.st != ST_OK || B.overrun()) {
            if (O.st == ST_OK) O.st = ST_CORRUPT;
            return;
        }
        if (fin) return;
    }
}

// GZIP members (RFC 1952) or one zlib stream (RFC 1950).
template <class W, class LdsT, class InX, class OutT>
DF_HD void gzip(LdsT& L, InX& I, OutT& O, uint32_t p, uint32_t end) {
    bool first = true;
    while (O.st == ST_OK && (first || p < end)) {
        if (end - p < 2) { O.st = ST_CORRUPT; return; }
        I.ensure(p, 16);
        const uint32_t b0 = I.byte(p), b1 = I.byte(p + 1);
        const uint32_t o0 = O.op;
        bool zlib = false;
        if (b0 == 0x1f && b1 == 0x8b) {
            if (end - p < 18 || I.byte(p + 2) != 8) { O.st = ST_CORRUPT; return; }
            const uint32_t flg = I.byte(p + 3);
            p += 10;
            if (flg & 4) {
                I.ensure(p, 2);
                p += 2 + I.u16le(p);
            }
            for (uint32_t f = 8; f <= 16; f <<= 1) {
                if (!(flg & f)) continue;
                for (;;) {  // zero-terminated name / comment
                    if (p >= end) { O.st = ST_CORRUPT; return; }
                    I.ensure(p, 1);
                    if (I.byte(p++) == 0) break;
                }
            }
            if (flg & 2) p += 2;
        } else if (first && (b0 & 0x0f) == 8 && ((b0 << 8) | b1) % 31 == 0 && !(b1 & 0x20)) {
            zlib = true;
            p += 2;
        } else {
            O.st = ST_CORRUPT;
            return;
        }
        if (p > end) { O.st = ST_CORRUPT; return; }
        Bits<InX> B{0ull, 0u, p, end, 0u};
        O.crc_on = !zlib;  // zlib streams end in an Adler-32 (not checked)
        O.crc = 0;
        O.crc_pos = O.op;
        inflate<W>(L, I, O, B);
        if (O.st != ST_OK) return;
        p = B.align_byte();
        const uint32_t tail = zlib ? 4u : 8u;
        if (p > end || end - p < tail) { O.st = ST_CORRUPT; return; }
        if (!zlib) {
            I.ensure(p, 8);
            if (I.u32le(p + 4) != O.op - o0) { O.st = ST_SIZE; return; }
            O.crc_upto(O.op);  // the member's last bytes (still in the ring)
            if (I.u32le(p) != O.crc) { O.st = ST_CORRUPT; return; }
            O.crc_on = false;
        }
        p += tail;
        first = false;
        if (zlib) break;
    }
}

}  // namespace pqinf
