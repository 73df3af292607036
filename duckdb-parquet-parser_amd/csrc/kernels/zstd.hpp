// zstd.hpp — Zstandard frame decoding (RFC 8878) for the codec pass
// (SURVEY §8f rank 4 widening; outside the reference's parity scope: the
// reference rejects every codec, column_reader.cpp:13-15).  Parquet's ZSTD
// pages (codec 6) are one or more zstd frames each.
//
// The decoder is written once over three small interfaces so that the same
// code runs in k_codec (a wavefront executing it wave-uniformly: every lane
// computes the same scalar values, the output stage spreads copies over the
// lanes) and in the host harness the tests use to pin it against pyarrow's
// zstd (tools/zstd_check.cpp):
//   src.byte(p)   input byte p (0 past the end)
//   out           lit_begin(n) / lit_at(k, b) / lit_done(): the block's literals;
//                 lits(n), raw(p, n), rle(b, n), copy(offset, n): the output
//   ZTables       FSE and Huffman decode tables (LDS on the device)
// Literals decoded by Huffman go to a literal buffer the output stage owns
// (out.lit_at / out.lit_done); sequences then copy from it.
// Not supported (status ZS_UNSUPPORTED): dictionaries (a frame naming a
// dictionary id).  The content checksum is skipped, not verified.
#pragma once
#include <cstdint>

#ifndef ZS_HD
#define ZS_HD __host__ __device__ __forceinline__
#endif

namespace zs {

enum : uint32_t { ZS_OK = 0, ZS_CORRUPT = 1, ZS_SIZE = 2, ZS_UNSUPPORTED = 3 };

struct FseEnt {  // one decode-table entry
    uint16_t base;   // next state's baseline
    uint8_t sym;
    uint8_t bits;
};
struct HufEnt {
    uint8_t sym;
    uint8_t bits;
};

constexpr int kLLMax = 35, kMLMax = 52, kOFMax = 31;
constexpr int kLLLog = 9, kMLLog = 9, kOFLog = 8, kHufMaxBits = 11;

struct ZTables {
    FseEnt ll[1 << kLLLog];
    FseEnt ml[1 << kMLLog];
    FseEnt of[1 << kOFLog];
    HufEnt huf[1 << kHufMaxBits];
    FseEnt wt[1 << 6];           // Huffman weights' FSE table
    int16_t norm[64];            // normalized counts (build scratch)
    uint16_t next[64];           // symbolNext (build scratch)
    uint8_t weights[256];
    uint32_t llc[36], mlc[53];   // code -> baseline | extra bits << 24 (filled by decompress)
    uint32_t ll_log, ml_log, of_log, huf_bits;
    uint32_t have_ll, have_ml, have_of, have_huf;  // repeat modes: a table from an earlier block
};

ZS_HD uint32_t highbit(uint32_t v) { return 31u - static_cast<uint32_t>(__builtin_clz(v)); }  // v > 0

// bits [lo, lo + n) of the little-endian bit array held by src bytes
// [base, base + len) (n <= 32; bits outside read 0)
template <class Src>
ZS_HD uint32_t bits_at(const Src& src, uint32_t base, uint32_t len, int64_t lo, uint32_t n) {
    if (n == 0) return 0u;
    uint64_t v = 0;
    const int64_t b0 = lo >> 3;  // (arithmetic shift: lo may be < 0)
    for (int k = 0; k < 5; k++) {
        const int64_t b = b0 + k;
        const uint32_t x = (b >= 0 && b < static_cast<int64_t>(len)) ? src.byte(base + static_cast<uint32_t>(b)) : 0u;
        v |= static_cast<uint64_t>(x) << (8 * k);
    }
    const uint32_t sh = static_cast<uint32_t>(lo - (b0 << 3));
    return static_cast<uint32_t>((v >> sh) & ((n == 32) ? 0xFFFFFFFFull : ((1ull << n) - 1ull)));
}

// Backward bit stream (zstd's BIT_DStream): bits are read from the end of
// [base, base + len); the last byte's highest set bit is the start marker.
template <class Src>
struct BitB {
    const Src* src;
    uint32_t base, len;
    int64_t pos;   // bits left above bit 0 (negative: read past the start)
    uint64_t cont; // bits [clo, clo + 64) of the stream (0 outside it)
    int64_t clo;
    ZS_HD bool init(const Src& s, uint32_t b, uint32_t l) {
        src = &s;
        base = b;
        len = l;
        if (l == 0) return false;
        const uint32_t last = s.byte(b + l - 1);
        if (last == 0) return false;
        pos = static_cast<int64_t>(8 * (l - 1) + highbit(last));
        fill(pos);
        return true;
    }
    // the 8 bytes that end with the byte holding bit e - 1 (a reader moving
    // down the stream refills about once per 7 bytes)
    ZS_HD void fill(int64_t e) {
        const int64_t bend = (e + 7) >> 3;  // exclusive byte end
        uint64_t v = 0;
        for (int k = 0; k < 8; k++) {
            const int64_t b = bend - 8 + k;
            const uint32_t x = (b >= 0 && b < static_cast<int64_t>(len)) ? src->byte(base + static_cast<uint32_t>(b)) : 0u;
            v |= static_cast<uint64_t>(x) << (8 * k);
        }
        cont = v;
        clo = (bend - 8) * 8;
    }
    ZS_HD uint32_t get(int64_t lo, uint32_t n) {  // n <= 32
        if (n == 0) return 0u;
        if (lo < clo || lo + n > clo + 64) fill(lo + n);
        return static_cast<uint32_t>((cont >> (lo - clo)) & ((n == 32) ? 0xFFFFFFFFull : ((1ull << n) - 1ull)));
    }
    ZS_HD uint32_t read(uint32_t n) {
        pos -= n;
        return get(pos, n);
    }
    ZS_HD uint32_t peek(uint32_t n) { return get(pos - n, n); }
};

// FSE table description (forward bit stream at src[p ..], at most `end`):
// normalized counts into T.norm, returns bytes used (0: corrupt)
template <class Src>
ZS_HD uint32_t read_norm(const Src& src, uint32_t p, uint32_t end, int max_sym, uint32_t max_log, ZTables& T,
                         uint32_t& log, int& nsym) {
    if (p >= end) return 0;
    const uint32_t len = end - p;
    int64_t bp = 0;  // bit position
    log = (bits_at(src, p, len, bp, 4)) + 5;
    bp += 4;
    if (log > max_log) return 0;
    if (max_sym > 63) max_sym = 63;  // T.norm / T.next hold 64 symbols; no zstd alphabet is larger
    int32_t remaining = (1 << log) + 1;
    int32_t threshold = 1 << log;
    uint32_t nb = log + 1;
    int s = 0;
    bool prev0 = false;
    for (int k = 0; k < 64; k++) T.norm[k] = 0;
    while (remaining > 1 && s <= max_sym) {
        if (prev0) {
            for (;;) {
                const uint32_t r = bits_at(src, p, len, bp, 2);
                bp += 2;
                s += static_cast<int>(r);
                if (r != 3) break;
            }
            if (s > max_sym) return 0;
            prev0 = false;
            if (bp > static_cast<int64_t>(8) * len) return 0;
            continue;
        }
        const int32_t maxv = (2 * threshold - 1) - remaining;
        int32_t count;
        const uint32_t low = bits_at(src, p, len, bp, nb - 1);
        if (static_cast<int32_t>(low) < maxv) {
            count = static_cast<int32_t>(low);
            bp += nb - 1;
        } else {
            count = static_cast<int32_t>(bits_at(src, p, len, bp, nb));
            if (count >= threshold) count -= maxv;
            bp += nb;
        }
        count--;  // -1: probability "less than 1"
        remaining -= count < 0 ? -count : count;
        T.norm[s++] = static_cast<int16_t>(count);
        prev0 = count == 0;
        while (remaining < threshold && nb > 1) {
            nb--;
            threshold >>= 1;
        }
        if (bp > static_cast<int64_t>(8) * len) return 0;
    }
    if (remaining != 1) return 0;
    nsym = s;
    return static_cast<uint32_t>((bp + 7) >> 3);
}

// decode table from T.norm[0 .. nsym) at accuracy log `log`
ZS_HD bool build_fse(ZTables& T, FseEnt* tab, uint32_t log, int nsym) {
    const uint32_t size = 1u << log;
    uint32_t high = size - 1;
    for (int s = 0; s < nsym; s++) {
        if (T.norm[s] == -1) {
            tab[high].sym = static_cast<uint8_t>(s);
            if (high == 0) return false;
            high--;
            T.next[s] = 1;
        } else {
            T.next[s] = static_cast<uint16_t>(T.norm[s] < 0 ? 0 : T.norm[s]);
        }
    }
    const uint32_t step = (size >> 1) + (size >> 3) + 3, mask = size - 1;
    uint32_t pos = 0;
    for (int s = 0; s < nsym; s++) {
        for (int i = 0; i < T.norm[s]; i++) {
            tab[pos].sym = static_cast<uint8_t>(s);
            do pos = (pos + step) & mask;
            while (pos > high);
        }
    }
    if (pos != 0) return false;
    for (uint32_t u = 0; u < size; u++) {
        const uint32_t s = tab[u].sym;
        const uint32_t ns = T.next[s]++;
        if (ns == 0) return false;
        const uint32_t b = log - highbit(ns);
        tab[u].bits = static_cast<uint8_t>(b);
        tab[u].base = static_cast<uint16_t>((ns << b) - size);
    }
    return true;
}

ZS_HD void build_rle(FseEnt* tab, uint32_t sym) {
    tab[0].sym = static_cast<uint8_t>(sym);
    tab[0].bits = 0;
    tab[0].base = 0;
}

// predefined distributions (RFC 8878 3.1.1.3.2.2)
ZS_HD int16_t ll_default(int s) {
    constexpr int16_t t[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                               2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
    return t[s];
}
ZS_HD int16_t ml_default(int s) {
    constexpr int16_t t[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                               1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
    return t[s];
}
ZS_HD int16_t of_default(int s) {
    constexpr int16_t t[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1,
                               1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};
    return t[s];
}
ZS_HD uint32_t ll_base(uint32_t c) {
    constexpr uint32_t t[36] = {0,  1,  2,  3,  4,  5,  6,   7,   8,   9,   10,   11,   12,   13,   14,    15,    16,   18,
                                20, 22, 24, 28, 32, 40, 48, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536};
    return t[c];
}
ZS_HD uint32_t ll_bits(uint32_t c) {
    constexpr uint8_t t[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,  0,  1,  1,
                               1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
    return t[c];
}
ZS_HD uint32_t ml_base(uint32_t c) {
    constexpr uint32_t t[53] = {3,  4,  5,  6,  7,  8,  9,  10, 11, 12,  13,  14,  15,   16,   17,   18,   19,   20,
                                21, 22, 23, 24, 25, 26, 27, 28, 29, 30,  31,  32,  33,   34,   35,   37,   39,   41,
                                43, 47, 51, 59, 67, 83, 99, 131, 259, 515, 1027, 2051, 4099, 8195, 16387, 32771, 65539};
    return t[c];
}
ZS_HD uint32_t ml_bits(uint32_t c) {
    constexpr uint8_t t[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                               0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
    return t[c];
}

// One symbol table of the sequences section by its mode; returns bytes used
// (mode 2) or 0 / 1 (predefined, repeat / RLE), or -1: corrupt.
template <class Src>
ZS_HD int32_t seq_table(const Src& src, uint32_t p, uint32_t end, uint32_t mode, int which, ZTables& T) {
    FseEnt* tab = which == 0 ? T.ll : (which == 1 ? T.of : T.ml);
    uint32_t* lg = which == 0 ? &T.ll_log : (which == 1 ? &T.of_log : &T.ml_log);
    uint32_t* have = which == 0 ? &T.have_ll : (which == 1 ? &T.have_of : &T.have_ml);
    const int maxs = which == 0 ? kLLMax : (which == 1 ? kOFMax : kMLMax);
    const uint32_t maxlog = which == 0 ? kLLLog : (which == 1 ? kOFLog : kMLLog);
    if (mode == 0) {
        const int n = which == 0 ? 36 : (which == 1 ? 29 : 53);
        for (int s = 0; s < n; s++) T.norm[s] = which == 0 ? ll_default(s) : (which == 1 ? of_default(s) : ml_default(s));
        const uint32_t l = which == 1 ? 5u : 6u;
        if (!build_fse(T, tab, l, n)) return -1;
        *lg = l;
        *have = 1;
        return 0;
    }
    if (mode == 1) {
        if (p >= end) return -1;
        const uint32_t s = src.byte(p);
        if (static_cast<int>(s) > maxs) return -1;
        build_rle(tab, s);
        *lg = 0;
        *have = 1;
        return 1;
    }
    if (mode == 2) {
        uint32_t l = 0;
        int n = 0;
        const uint32_t used = read_norm(src, p, end, maxs, maxlog, T, l, n);
        if (used == 0 || !build_fse(T, tab, l, n)) return -1;
        *lg = l;
        *have = 1;
        return static_cast<int32_t>(used);
    }
    return *have ? 0 : -1;  // repeat
}

// Huffman tree description at src[p ..]; returns bytes used (0: corrupt)
template <class Src>
ZS_HD uint32_t read_huf(const Src& src, uint32_t p, uint32_t end, ZTables& T) {
    if (p >= end) return 0;
    const uint32_t hb = src.byte(p);
    uint32_t nw = 0, used = 0;
    if (hb >= 128) {  // direct: 4-bit weights
        nw = hb - 127;
        used = 1 + (nw + 1) / 2;
        if (p + used > end) return 0;
        for (uint32_t i = 0; i < nw; i++) {
            const uint32_t b = src.byte(p + 1 + i / 2);
            T.weights[i] = static_cast<uint8_t>((i & 1) ? (b & 15u) : (b >> 4));
        }
    } else {  // FSE-compressed weights (two interleaved states)
        if (hb == 0 || p + 1 + hb > end) return 0;
        uint32_t lg = 0;
        int ns = 0;
        const uint32_t d = read_norm(src, p + 1, p + 1 + hb, 12, 6, T, lg, ns);  // weights 0..12 (RFC 8878 4.2.1.2)
        if (d == 0 || d >= hb || !build_fse(T, T.wt, lg, ns)) return 0;
        BitB<Src> bs;
        if (!bs.init(src, p + 1 + d, hb - d)) return 0;
        uint32_t s1 = bs.read(lg), s2 = bs.read(lg);
        for (;;) {
            if (nw >= 255) return 0;
            T.weights[nw++] = T.wt[s1].sym;
            s1 = T.wt[s1].base + bs.read(T.wt[s1].bits);
            if (bs.pos < 0) {
                if (nw >= 255) return 0;
                T.weights[nw++] = T.wt[s2].sym;
                break;
            }
            if (nw >= 255) return 0;
            T.weights[nw++] = T.wt[s2].sym;
            s2 = T.wt[s2].base + bs.read(T.wt[s2].bits);
            if (bs.pos < 0) {
                if (nw >= 255) return 0;
                T.weights[nw++] = T.wt[s1].sym;
                break;
            }
        }
        used = 1 + hb;
    }
    // the last weight is implied: the total of 2^(w-1) rounds up to a power of two
    uint32_t total = 0;
    for (uint32_t i = 0; i < nw; i++) {
        if (T.weights[i] > kHufMaxBits) return 0;
        if (T.weights[i]) total += 1u << (T.weights[i] - 1);
    }
    if (total == 0) return 0;
    const uint32_t maxb = highbit(total) + 1;
    if (maxb > kHufMaxBits) return 0;
    const uint32_t rest = (1u << maxb) - total;
    if (rest & (rest - 1)) return 0;
    if (nw >= 256) return 0;
    T.weights[nw++] = static_cast<uint8_t>(highbit(rest) + 1);
    // table: weights 1 .. maxb in order, each symbol 2^(w-1) entries
    uint32_t at = 0;
    for (uint32_t w = 1; w <= maxb; w++) {
        for (uint32_t s = 0; s < nw; s++) {
            if (T.weights[s] != w) continue;
            const uint32_t n = 1u << (w - 1);
            for (uint32_t k = 0; k < n; k++) {
                T.huf[at + k].sym = static_cast<uint8_t>(s);
                T.huf[at + k].bits = static_cast<uint8_t>(maxb + 1 - w);
            }
            at += n;
        }
    }
    if (at != (1u << maxb)) return 0;
    T.huf_bits = maxb;
    T.have_huf = 1;
    return used;
}

// One Huffman stream of n symbols at src[p, p + len) into the output stage's
// literal buffer from index k0.
template <class Src, class Out>
ZS_HD bool huf_stream(const Src& src, uint32_t p, uint32_t len, uint32_t n, uint32_t k0, const ZTables& T, Out& out) {
    BitB<Src> bs;
    if (!bs.init(src, p, len)) return false;
    const uint32_t mb = T.huf_bits;
    for (uint32_t i = 0; i < n; i++) {
        const HufEnt e = T.huf[bs.peek(mb)];
        bs.pos -= e.bits;
        out.lit_at(k0 + i, e.sym);
    }
    return bs.pos == 0;
}

// One compressed block src[p, p + bsize).
template <class Src, class Out>
ZS_HD uint32_t block(const Src& src, uint32_t p, uint32_t bsize, ZTables& T, Out& out, uint32_t rep[3]) {
    const uint32_t end = p + bsize;
    // literals section
    const uint32_t b0 = src.byte(p);
    const uint32_t lt = b0 & 3u, sf = (b0 >> 2) & 3u;
    uint32_t regen = 0, csize = 0, hl = 0;
    bool four = false;
    if (lt < 2) {
        if (sf == 0 || sf == 2) { regen = b0 >> 3; hl = 1; }
        else if (sf == 1) { regen = (b0 >> 4) + (src.byte(p + 1) << 4); hl = 2; }
        else { regen = (b0 >> 4) + (src.byte(p + 1) << 4) + (src.byte(p + 2) << 12); hl = 3; }
    } else {
        const uint32_t x = b0 | (src.byte(p + 1) << 8) | (src.byte(p + 2) << 16) | (src.byte(p + 3) << 24);
        if (sf < 2) {
            hl = 3;
            regen = (x >> 4) & 0x3FFu;
            csize = (x >> 14) & 0x3FFu;
            four = sf == 1;
        } else if (sf == 2) {
            hl = 4;
            regen = (x >> 4) & 0x3FFFu;
            csize = (x >> 18) & 0x3FFFu;
            four = true;
        } else {
            hl = 5;
            const uint64_t y = static_cast<uint64_t>(x) | (static_cast<uint64_t>(src.byte(p + 4)) << 32);
            regen = static_cast<uint32_t>((y >> 4) & 0x3FFFFu);
            csize = static_cast<uint32_t>((y >> 22) & 0x3FFFFu);
            four = true;
        }
    }
    if (regen > (128u << 10)) return ZS_CORRUPT;
    uint32_t q = p + hl;
    if (q > end) return ZS_CORRUPT;
    if (!out.lit_begin(regen)) return ZS_SIZE;
    if (lt == 0) {  // raw
        if (q + regen > end) return ZS_CORRUPT;
        for (uint32_t i = 0; i < regen; i++) out.lit_at(i, src.byte(q + i));
        q += regen;
    } else if (lt == 1) {  // RLE
        if (q + 1 > end) return ZS_CORRUPT;
        const uint32_t b = src.byte(q);
        for (uint32_t i = 0; i < regen; i++) out.lit_at(i, b);
        q += 1;
    } else {
        if (q + csize > end) return ZS_CORRUPT;
        uint32_t h = 0;
        if (lt == 2) {
            h = read_huf(src, q, q + csize, T);
            if (h == 0) return ZS_CORRUPT;
        } else if (!T.have_huf) {
            return ZS_CORRUPT;
        }
        const uint32_t s0 = q + h, slen = csize - h;
        if (!four) {
            if (!huf_stream(src, s0, slen, regen, 0, T, out)) return ZS_CORRUPT;
        } else {
            if (slen < 6) return ZS_CORRUPT;
            const uint32_t l1 = src.byte(s0) | (src.byte(s0 + 1) << 8), l2 = src.byte(s0 + 2) | (src.byte(s0 + 3) << 8),
                           l3 = src.byte(s0 + 4) | (src.byte(s0 + 5) << 8);
            if (6u + l1 + l2 + l3 > slen) return ZS_CORRUPT;
            const uint32_t l4 = slen - 6 - l1 - l2 - l3;
            const uint32_t per = (regen + 3) / 4;
            if (regen < 3 * per) return ZS_CORRUPT;
            uint32_t a = s0 + 6;
            if (!huf_stream(src, a, l1, per, 0, T, out)) return ZS_CORRUPT;
            a += l1;
            if (!huf_stream(src, a, l2, per, per, T, out)) return ZS_CORRUPT;
            a += l2;
            if (!huf_stream(src, a, l3, per, 2 * per, T, out)) return ZS_CORRUPT;
            a += l3;
            if (!huf_stream(src, a, l4, regen - 3 * per, 3 * per, T, out)) return ZS_CORRUPT;
        }
        q += csize;
    }
    out.lit_done();
    // sequences section
    if (q >= end) {  // no sequences header byte: literals only
        if (q > end) return ZS_CORRUPT;
        return out.lits(regen) ? ZS_OK : ZS_SIZE;
    }
    uint32_t nseq = src.byte(q++);
    if (nseq >= 128) {
        if (nseq < 255) {
            if (q >= end) return ZS_CORRUPT;
            nseq = ((nseq - 128) << 8) + src.byte(q++);
        } else {
            if (q + 2 > end) return ZS_CORRUPT;
            nseq = src.byte(q) + (src.byte(q + 1) << 8) + 0x7F00u;
            q += 2;
        }
    }
    if (nseq == 0) {
        if (q != end) return ZS_CORRUPT;
        return out.lits(regen) ? ZS_OK : ZS_SIZE;
    }
    if (q >= end) return ZS_CORRUPT;
    const uint32_t modes = src.byte(q++);
    if (modes & 3u) return ZS_CORRUPT;
    const uint32_t mll = modes >> 6, mof = (modes >> 4) & 3u, mml = (modes >> 2) & 3u;
    int32_t u = seq_table(src, q, end, mll, 0, T);
    if (u < 0) return ZS_CORRUPT;
    q += static_cast<uint32_t>(u);
    u = seq_table(src, q, end, mof, 1, T);
    if (u < 0) return ZS_CORRUPT;
    q += static_cast<uint32_t>(u);
    u = seq_table(src, q, end, mml, 2, T);
    if (u < 0) return ZS_CORRUPT;
    q += static_cast<uint32_t>(u);
    if (q >= end) return ZS_CORRUPT;
    BitB<Src> bs;
    if (!bs.init(src, q, end - q)) return ZS_CORRUPT;
    uint32_t sll = bs.read(T.ll_log), sof = bs.read(T.of_log), sml = bs.read(T.ml_log);
    uint32_t lused = 0;
    for (uint32_t i = 0; i < nseq; i++) {
        const FseEnt eo = T.of[sof], em = T.ml[sml], el = T.ll[sll];
        const uint32_t oc = eo.sym, mc = em.sym, lc = el.sym;
        if (oc > 31 || mc > kMLMax || lc > kLLMax) return ZS_CORRUPT;
        uint32_t ofv = oc < 32 ? (1u << oc) : 0u;
        ofv += bs.read(oc);
        const uint32_t mlx = T.mlc[mc], llx = T.llc[lc];
        const uint32_t mlv = (mlx & 0xFFFFFFu) + bs.read(mlx >> 24);
        const uint32_t llv = (llx & 0xFFFFFFu) + bs.read(llx >> 24);
        if (i + 1 < nseq) {
            sll = el.base + bs.read(el.bits);
            sml = em.base + bs.read(em.bits);
            sof = eo.base + bs.read(eo.bits);
        }
        uint32_t off;
        if (ofv > 3) {
            off = ofv - 3;
            rep[2] = rep[1];
            rep[1] = rep[0];
            rep[0] = off;
        } else {
            uint32_t idx = ofv - 1 + (llv == 0 ? 1u : 0u);
            if (idx == 0) {
                off = rep[0];
            } else {
                off = idx == 3 ? rep[0] - 1 : rep[idx];
                if (idx >= 2) rep[2] = rep[1];
                rep[1] = rep[0];
                rep[0] = off;
            }
        }
        if (llv > regen - lused) return ZS_CORRUPT;
        if (llv && !out.lits(llv)) return ZS_SIZE;
        lused += llv;
        if (off == 0) return ZS_CORRUPT;
        const uint32_t st = out.copy(off, mlv);
        if (st != ZS_OK) return st;
    }
    if (bs.pos != 0) return ZS_CORRUPT;
    if (lused < regen && !out.lits(regen - lused)) return ZS_SIZE;
    return ZS_OK;
}

// Every frame of src[0, len): the page's payload.
template <class Src, class Out>
ZS_HD uint32_t decompress(const Src& src, uint32_t len, ZTables& T, Out& out) {
    uint32_t p = 0;
    if (len == 0) return ZS_CORRUPT;
    for (uint32_t c = 0; c < 36; c++) T.llc[c] = ll_base(c) | (ll_bits(c) << 24);
    for (uint32_t c = 0; c < 53; c++) T.mlc[c] = ml_base(c) | (ml_bits(c) << 24);
    while (p < len) {
        if (p + 4 > len) return ZS_CORRUPT;
        const uint32_t magic = src.byte(p) | (src.byte(p + 1) << 8) | (src.byte(p + 2) << 16) | (src.byte(p + 3) << 24);
        p += 4;
        if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {  // skippable frame
            if (p + 4 > len) return ZS_CORRUPT;
            const uint32_t n = src.byte(p) | (src.byte(p + 1) << 8) | (src.byte(p + 2) << 16) | (src.byte(p + 3) << 24);
            p += 4;
            if (n > len - p) return ZS_CORRUPT;
            p += n;
            continue;
        }
        if (magic != 0xFD2FB528u) return ZS_CORRUPT;
        if (p >= len) return ZS_CORRUPT;
        const uint32_t fhd = src.byte(p++);
        const uint32_t fcs_flag = fhd >> 6, single = (fhd >> 5) & 1u, cksum = (fhd >> 2) & 1u, did = fhd & 3u;
        if (fhd & 8u) return ZS_CORRUPT;  // reserved bit
        if (!single) p += 1;              // window descriptor (the output is the page: no window limit needed)
        const uint32_t dsz = did == 0 ? 0u : (did == 1 ? 1u : (did == 2 ? 2u : 4u));
        uint32_t dict = 0;
        for (uint32_t k = 0; k < dsz; k++) dict |= src.byte(p + k) << (8 * k);
        p += dsz;
        if (dict) return ZS_UNSUPPORTED;
        const uint32_t fsz = fcs_flag == 0 ? (single ? 1u : 0u) : (fcs_flag == 1 ? 2u : (fcs_flag == 2 ? 4u : 8u));
        p += fsz;  // (content size: the slot's size is checked by the caller)
        if (p > len) return ZS_CORRUPT;
        uint32_t rep[3] = {1, 4, 8};
        T.have_ll = T.have_ml = T.have_of = T.have_huf = 0;
        for (;;) {
            if (p + 3 > len) return ZS_CORRUPT;
            const uint32_t bh = src.byte(p) | (src.byte(p + 1) << 8) | (src.byte(p + 2) << 16);
            p += 3;
            const uint32_t last = bh & 1u, bt = (bh >> 1) & 3u, bs = bh >> 3;
            if (bt == 0) {
                if (bs > len - p) return ZS_CORRUPT;
                if (!out.raw(p, bs)) return ZS_SIZE;
                p += bs;
            } else if (bt == 1) {
                if (p + 1 > len) return ZS_CORRUPT;
                if (!out.rle(src.byte(p), bs)) return ZS_SIZE;
                p += 1;
            } else if (bt == 2) {
                if (bs > len - p || bs == 0 || bs > (128u << 10)) return ZS_CORRUPT;
                const uint32_t st = block(src, p, bs, T, out, rep);
                if (st != ZS_OK) return st;
                p += bs;
            } else {
                return ZS_CORRUPT;
            }
            if (last) break;
        }
        if (cksum) p += 4;  // content checksum: skipped
        if (p > len) return ZS_CORRUPT;
    }
    return ZS_OK;
}

}  // namespace zs
