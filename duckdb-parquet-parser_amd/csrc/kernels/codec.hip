// codec.hip — compressed pages and DATA_PAGE_V2 pages on the GPU (SURVEY §8f
// rank 4; outside the reference's parity scope: the reference rejects any
// codec, column_reader.cpp:13-15, and does not decode V2 pages, 56-67).
//
// Each entry turns one page payload, as the file holds it (raw chunk bytes in
// HBM), into the payload the decode kernels read, written to the page's slot
// in the chunk image (capi.hip `slot`):
//   V1 page, codec C:  decompress(payload)
//   V2 page:           [u32 def_len][def levels] (max_def > 0)
//                      [u32 rep_len][rep levels] (max_rep > 0)
//                      values (decompressed when the page says is_compressed)
// i.e. the V1 layout in the order the reference reads it (column_reader.cpp:
// 146-170), so every decode and regex kernel runs unchanged on the result.
//
// One wavefront per page (persistent grid-stride loop).  The compressed input
// is staged through an 8 KiB LDS window; the output goes through a 64 KiB LDS
// ring that holds the whole back-reference history (SNAPPY and LZ4 offsets
// are < 2^16, DEFLATE's < 2^15) and is flushed to HBM 1 KiB at a time as
// aligned 16-byte stores.  The command stream (literal runs and copies) is
// parsed wave-uniformly; each command is executed 64 bytes per step by the
// whole wave.  A copy's byte j reads the ring at c0 - d + (j mod d) for
// overlapping copies (d < 64) or c0 - d + j, relative to the step's first
// output byte c0: bytes before c0 are final, and a step's LDS reads issue
// before its writes, so one step never reads its own output.
//   SNAPPY   (codec 1): format_description.txt of google/snappy
//   GZIP     (codec 2): RFC 1952 members holding RFC 1951 DEFLATE (zlib RFC
//                       1950 framing also accepted); Huffman symbols decoded
//                       through 10-bit LDS lookup tables, longer codes by the
//                       canonical bit-serial walk
//   LZ4      (codec 5): Hadoop framing ([u32 BE raw][u32 BE packed] blocks)
//   LZ4_RAW  (codec 7): one LZ4 block
//   ZSTD     (codec 6): RFC 8878 frames (zstd.hpp, the decoder the host tests
//                       pin against pyarrow's zstd); Huffman literals go to
//                       the slot's tail (at or past every byte still to be
//                       written) and are copied out by the sequences; matches
//                       farther back than the ring read the flushed output
#include <algorithm>
#include <cstddef>

#include "kernels/device_common.hpp"
#include "kernels/kernels.hpp"
#include "kernels/deflate.hpp"
#include "kernels/lz.hpp"
#include "kernels/zstd.hpp"
#include "pq_gpu.h"

#ifndef PQ_CODEC_EXEC_SKIP  // timing probe: the executor drains the command queue without running it
#define PQ_CODEC_EXEC_SKIP 0
#endif
#ifndef PQ_CODEC_PUSH_SKIP
#define PQ_CODEC_PUSH_SKIP 0
#endif
#ifndef PQ_CODEC_CHECK_SKIP
#define PQ_CODEC_CHECK_SKIP 0
#endif

namespace pqk {
namespace {

using dev::lane;

constexpr uint32_t kRing = 65536;
constexpr uint32_t kRingMask = kRing - 1;
constexpr uint32_t kInWin = 8192;  // staged input bytes (+16 slack)
constexpr uint32_t kFlush = 1024;  // output bytes per flush step (16 per lane)
constexpr uint32_t kFast = pqinf::kFast;  // Huffman lookup bits (deflate.hpp)

struct CodecLds {
    uint8_t ring[kRing];
    uint8_t in[kInWin + 32];
    uint16_t lt[1 << kFast];  // litlen: sym << 4 | len (0 = longer code)
    uint16_t dt[1 << kFast];  // distance
    uint16_t sym[320];        // symbols in canonical order: litlen [0, 288), dist [288, 320)
    uint16_t code[320];       // canonical code per symbol
    uint16_t cnt[2][16];      // code count per length
    uint8_t lens[320];        // code lengths: litlen [0, 288), dist [288, 320)
    uint16_t nxt[16], offs[16];  // build_code: next code / next symbol slot per length
    uint32_t scratch[4];
    uint32_t crc_tab[256];    // CRC-32 (gzip trailers): byte table
};

// LDS pointers keep their address space (a generic pointer held in a struct
// compiles to flat accesses, which also count in the vector memory counter)
using lds8 = __attribute__((address_space(3))) uint8_t;
using lds16 = __attribute__((address_space(3))) uint16_t;
using lds32 = __attribute__((address_space(3))) uint32_t;

__device__ __forceinline__ void lds_put16(lds8* base, uint32_t off, const uint4& v) {
    lds32* d = reinterpret_cast<lds32*>(base + off);
    d[0] = v.x;
    d[1] = v.y;
    d[2] = v.z;
    d[3] = v.w;
}
__device__ __forceinline__ uint4 lds_get16(const lds8* base, uint32_t off) {
    const lds32* d = reinterpret_cast<const lds32*>(base + off);
    return make_uint4(d[0], d[1], d[2], d[3]);
}

__device__ __forceinline__ void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// ── staged input ───────────────────────────────────────────────────────────
// kWin: staged input bytes (kInWin; kSWin in the small-page instantiations)
template <uint32_t kWin>
struct InT {
    static constexpr uint32_t kWindow = kWin;
    const uint8_t* g;  // page input in HBM
    uint32_t len;      // input bytes
    uint32_t wlo;      // input byte held at in[sh]
    uint32_t sh;
    lds8* w;
    __device__ __forceinline__ void refill(uint32_t p) {
        const uintptr_t a = reinterpret_cast<uintptr_t>(g) + p;
        wlo = p;
        sh = static_cast<uint32_t>(a & 15u);
        // (derived from g, so the loads stay global: a pointer made from an
        // integer would compile to flat loads)
        const uint4* src = reinterpret_cast<const uint4*>(g + p - sh);  // (g + p) - sh: never below g's buffer
        constexpr uint32_t nb = kWin / 16;
        static_assert(nb % kWave == 0, "one block per lane per step");
        const uint32_t nvalid = (sh + len > p ? (sh + len - p + 15) / 16 : 0u);  // blocks holding input bytes
        uint4 v[nb / kWave];
#pragma unroll
        for (uint32_t k = 0; k < nb / kWave; k++) {
            const uint32_t b = lane() + k * kWave;
            const uint4 x = src[min(b, nvalid ? nvalid - 1 : 0u)];
            v[k] = b < nvalid ? x : make_uint4(0u, 0u, 0u, 0u);
        }
#pragma unroll
        for (uint32_t k = 0; k < nb / kWave; k++) lds_put16(w, 16 * (lane() + k * kWave), v[k]);
        if (lane() < 2) lds_put16(w, 16 * (nb + lane()), make_uint4(0u, 0u, 0u, 0u));
        wsync();
    }
    // bytes [p, p + k) staged (k <= 16)
    __device__ __forceinline__ void ensure(uint32_t p, uint32_t k) {
        if (p < wlo || p + k + sh > wlo + kWin) refill(p);
    }
    __device__ __forceinline__ uint32_t at(uint32_t p) const { return min(p - wlo + sh, kWin + 16u); }
    __device__ __forceinline__ uint32_t byte(uint32_t p) const { return w[at(p)]; }
    __device__ __forceinline__ uint32_t u16le(uint32_t p) const { return byte(p) | (byte(p + 1) << 8); }
    __device__ __forceinline__ uint32_t u32le(uint32_t p) const {
        return byte(p) | (byte(p + 1) << 8) | (byte(p + 2) << 16) | (byte(p + 3) << 24);
    }
    __device__ __forceinline__ uint32_t u32be(uint32_t p) const {
        return (byte(p) << 24) | (byte(p + 1) << 16) | (byte(p + 2) << 8) | byte(p + 3);
    }
};

using In = InT<kInWin>;
// Pages whose payload is under kSRing bytes decode in the small-page
// instantiations: an 8 KiB history that holds the whole page and a 1 KiB
// input window, ~9 KiB of LDS per wavefront instead of 72, so a CU holds as
// many decoding pages as its registers allow (16) instead of two
constexpr uint32_t kSRing = 8192;
constexpr uint32_t kSWin = 1024;
using InS = InT<kSWin>;

enum : uint32_t { ST_OK = 0, ST_CORRUPT = 1, ST_SIZE = 2, ST_UNSUPPORTED = 3 };

// ── CRC-32 of GZIP members (RFC 1952; reflected polynomial 0xEDB88320) ─────
constexpr uint32_t kCrcPoly = 0xEDB88320u;
// a(x) * b(x) mod P(x) in the reflected representation (zlib's multmodp),
// branch-free: 32 steps
__device__ __forceinline__ uint32_t crc_mulmod(uint32_t a, uint32_t b) {
    uint32_t p = 0;
#pragma unroll
    for (int k = 31; k >= 0; k--) {
        p ^= (0u - ((a >> k) & 1u)) & b;
        b = (b >> 1) ^ ((0u - (b & 1u)) & kCrcPoly);
    }
    return p;
}
// x^(8 * nbytes) mod P (x2nmodp(nbytes, 3)): the shift crc32_combine applies
__device__ __forceinline__ uint32_t crc_xpow8(uint32_t nbytes) {
    uint32_t p = 1u << 31, sq = 1u << 23;  // x^0; x^(8 * 2^0) = x^8
    while (nbytes) {
        if (nbytes & 1u) p = crc_mulmod(sq, p);
        sq = crc_mulmod(sq, sq);
        nbytes >>= 1;
    }
    return p;
}

// CRC-32 of ring bytes [from, to) folded into crc (finalized form): 64
// lane segments, a crc32_combine tree over the lanes, a byte-wise tail
__device__ __attribute__((noinline)) uint32_t crc_fold(const lds8* ring, const lds32* crc_tab, uint32_t crc,
                                                      uint32_t from, uint32_t to) {
    const uint32_t len = uni(to - from), s = len / kWave;  // 64 segments of s bytes, then a tail
    if (s) {
        uint32_t c = 0xFFFFFFFFu;
        const uint32_t b0 = from + lane() * s;
        for (uint32_t j = 0; j < s; j++) c = crc_tab[(c ^ ring[(b0 + j) & kRingMask]) & 0xFFu] ^ (c >> 8);
        c = ~c;
        // tree of crc32_combine over the lanes: round r joins lanes i, i + 2^r
        uint32_t pw = crc_xpow8(s);  // shift by 2^r segments
#pragma unroll
        for (int r = 0; r < 6; r++) {
            const uint32_t other = static_cast<uint32_t>(__shfl_down(static_cast<int>(c), 1 << r));
            const uint32_t joined = crc_mulmod(c, pw) ^ other;
            c = (lane() & ((2u << r) - 1u)) == 0 ? joined : c;
            pw = crc_mulmod(pw, pw);
        }
        // pw: shift by 64 segments; fold the block (lane 0) into the running value
        crc = uni(crc_mulmod(crc, pw) ^ static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(c)));
        from += kWave * s;
    }
    if (from < to) {  // the tail (< 64 bytes): every lane, byte by byte (uniform result)
        uint32_t c = ~crc;
        for (uint32_t q = from; q < to; q++) c = crc_tab[(c ^ ring[q & kRingMask]) & 0xFFu] ^ (c >> 8);
        crc = uni(~c);
    }
    return crc;
}

// ── output ring ────────────────────────────────────────────────────────────
// kCrc: the GZIP kernel only.  The CRC fold in flush() would otherwise sit,
// inlined, in every codec's hot loop (147 VGPRs and 64 B/lane of scratch
// with it in round 3, against 111 VGPRs and none without): the non-GZIP
// kernel compiles it out.
template <bool kCrc, uint32_t kRingB = kRing>
struct Out {
    static constexpr uint32_t kRingSize = kRingB, kMask = kRingB - 1;
    lds8* ring;
    uint8_t* dst;   // the page slot (16-byte aligned)
    uint32_t op;    // bytes produced
    uint32_t fl;    // bytes flushed to dst (multiple of 16 until the end)
    uint32_t cap;   // bytes the slot's payload holds
    uint32_t vbase; // first byte of the decompressed stream (after a V2 prologue)
    uint32_t st;    // ST_*
    // running CRC-32 of the output since crc_pos0 (GZIP members): bytes
    // [crc_pos0, crc_pos) are in `crc` (finalized form); they are folded in
    // from the ring before it can be overwritten: inflate calls crc_keep()
    // once per symbol (a scalar compare; the fold runs about once per 63 KiB
    // of output) and folds before each piece of a stored block, so the fold
    // is out of flush() and out of the per-byte paths
    bool crc_on = false;
    uint32_t crc = 0, crc_pos = 0;
    const lds32* crc_tab = nullptr;
    // (the fold is a separate function taking values, not `this`: a call
    // through `this` puts the whole Out object in scratch)
    __device__ __forceinline__ void crc_upto(uint32_t to) {
        if constexpr (!kCrc) return;
        if (!crc_on || to <= crc_pos) return;
        crc = crc_fold(ring, crc_tab, crc, crc_pos, to);
        crc_pos = to;
    }
    // fold before the ring can wrap over bytes not yet in the CRC (the
    // caller then adds at most kCrcSlack bytes)
    static constexpr uint32_t kCrcSlack = 1024;
    __device__ __forceinline__ void crc_keep() {
        if constexpr (kCrc)
            if (crc_on && op - crc_pos > kRingB - kCrcSlack) crc_upto(op);
    }
    __device__ __forceinline__ void flush(bool final) {
        while (op - fl >= kFlush || (final && fl < op)) {
            const uint32_t n = min(kFlush, op - fl);
            const uint32_t b = fl + 16u * lane();
            if (b < fl + n) {
                uint4 v = lds_get16(ring, b & kMask);
                if (b + 16 > op) {  // bytes past the payload stay zero (slot padding)
                    const int32_t keep = static_cast<int32_t>(op - b);
                    auto mk = [&](int j) -> uint32_t {
                        const int32_t kb = keep - 4 * j;
                        return kb >= 4 ? 0xFFFFFFFFu : (kb <= 0 ? 0u : ((1u << (8 * kb)) - 1u));
                    };
                    v = make_uint4(v.x & mk(0), v.y & mk(1), v.z & mk(2), v.w & mk(3));
                }
                *reinterpret_cast<uint4*>(dst + b) = v;
            }
            fl += n;
            wsync();
        }
    }
    __device__ __forceinline__ bool room(uint32_t n) {
        if (op + n > cap || op + n < op) { st = ST_SIZE; return false; }
        return true;
    }
    // literal bytes [p, p + n) of the input
    template <class InX>
    __device__ __forceinline__ void lit(InX& I, uint32_t p, uint32_t n) {
        if (!room(n)) return;
        if (n <= static_cast<uint32_t>(kWave)) {  // one step (most literals): no loop
            I.ensure(p, n);
            if (lane() < n) ring[(op + lane()) & kMask] = static_cast<uint8_t>(I.byte(p + lane()));
            op += n;
            wsync();
            if (op - fl >= kFlush) flush(false);
            return;
        }
        for (uint32_t d = 0; d < n; d += kWave) {
            I.ensure(p + d, kWave);
            const uint32_t m = min(static_cast<uint32_t>(kWave), n - d);
            if (lane() < m) ring[(op + lane()) & kMask] = static_cast<uint8_t>(I.byte(p + d + lane()));
            op += m;
            wsync();
            if (op - fl >= kFlush) flush(false);
        }
    }
    // copy of n bytes from distance d: 64 bytes per step, byte c0 + j of a
    // step from c0 - d + (j mod d) (d < 64) or c0 - d + j: before c0, final
    __device__ __forceinline__ void copy(uint32_t d, uint32_t n) {
        if (d == 0 || d > op - vbase || d > kRingB - 1) { st = ST_CORRUPT; return; }
        if (!room(n)) return;
        if (n <= static_cast<uint32_t>(kWave) && d >= n) {  // one step, no overlap (most copies): no loop, no lane % d
            if (lane() < n) ring[(op + lane()) & kMask] = ring[(op - d + lane()) & kMask];
            op += n;
            wsync();
            if (op - fl >= kFlush) flush(false);
            return;
        }
        const uint32_t r = d >= static_cast<uint32_t>(kWave) ? lane() : lane() % d;
        for (uint32_t k = 0; k < n; k += kWave) {
            const uint32_t m = min(static_cast<uint32_t>(kWave), n - k);
            if (lane() < m) {
                const uint32_t v = ring[(op - d + r) & kMask];
                ring[(op + lane()) & kMask] = static_cast<uint8_t>(v);
            }
            op += m;
            wsync();
            if (op - fl >= kFlush) flush(false);
        }
    }
    __device__ __forceinline__ void put1(uint32_t b) {
        if (!room(1)) return;
        if (lane() == 0) ring[op & kMask] = static_cast<uint8_t>(b);
        op++;
        if (op - fl >= kFlush) {
            wsync();
            flush(false);
        }
    }
    __device__ __forceinline__ void put_u32(uint32_t v) {
        if (!room(4)) return;
        if (lane() < 4) ring[(op + lane()) & kMask] = static_cast<uint8_t>(v >> (8 * lane()));
        wsync();
        op += 4;
        flush(false);
    }
};

// ── command headers from registers ─────────────────────────────────────────
// The SNAPPY / LZ4 command stream is parsed wave-uniformly, one command after
// the other.  Reading each header byte from the staged input costs an LDS
// round trip on that serial chain; instead 256 input bytes sit in one VGPR
// (4 per lane) and a header byte is a v_readlane, so a command's only LDS
// round trip is its own execution (the ring read before the ring write).
template <class InX>
struct TagWin {
    InX* I;
    uint32_t base = 1u, lim = 0u, w = 0u;  // bytes [base, lim) held (empty at first)
    __device__ __forceinline__ void load(uint32_t p) {
        I->ensure(p, 16);
        base = p & ~3u;
        const uint32_t q = base + 4 * lane();
        w = I->byte(q) | (I->byte(q + 1) << 8) | (I->byte(q + 2) << 16) | (I->byte(q + 3) << 24);
        // the staged window's bytes only (past it the LDS holds others)
        lim = uni(min(base + 4 * static_cast<uint32_t>(kWave), I->wlo + InX::kWindow - I->sh));
        base = uni(base);
    }
    // bytes [p, p + k) held, loading them when they are not (k <= 16)
    __device__ __forceinline__ void need(uint32_t p, uint32_t k) {
        if (p < base || p + k > lim) load(p);
    }
    __device__ __forceinline__ uint32_t byte(uint32_t q) const {
        const uint32_t o = q - base;
        return (static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(w), static_cast<int>(o >> 2))) >>
                (8 * (o & 3u))) & 0xFFu;
    }
    __device__ __forceinline__ uint32_t u16le(uint32_t q) const { return byte(q) | (byte(q + 1) << 8); }
    __device__ __forceinline__ uint32_t u32le(uint32_t q) const {
        return byte(q) | (byte(q + 1) << 8) | (byte(q + 2) << 16) | (byte(q + 3) << 24);
    }
    static __device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
};

// ── SNAPPY / LZ4 parsers (lz.hpp), headers through TagWin ─────────────────
static_assert(pqlz::ST_OK == ST_OK && pqlz::ST_CORRUPT == ST_CORRUPT && pqlz::ST_SIZE == ST_SIZE, "status codes");
template <class InX, class OutT>
__device__ __forceinline__ void snappy(InX& I, OutT& O, uint32_t p, uint32_t end, uint32_t expect) {
    pqlz::snappy<TagWin<InX>>(I, O, p, end, expect);
}
template <class InX, class OutT>
__device__ __forceinline__ void lz4_block(InX& I, OutT& O, uint32_t p, uint32_t end) {
    pqlz::lz4_block<TagWin<InX>>(I, O, p, end);
}
template <class InX, class OutT>
__device__ __forceinline__ void lz4_hadoop(InX& I, OutT& O, uint32_t p, uint32_t end) {
    pqlz::lz4_hadoop<TagWin<InX>>(I, O, p, end);
}

// ── SNAPPY / LZ4: parse and execute on two waves ───────────────────────────
// One wave alone is issue-bound on a page (one instruction per four clocks
// and per wave, about half of them the serial parse: PQ_CODEC_PARSE_ONLY),
// and a chunk of 1 MiB pages has a few hundred pages for 1,024 SIMDs.  So
// the kind-0 kernel runs two waves per page: wave 0 parses the command
// stream (snappy / lz4_block with a QSink as their output: the same checks
// as Out's, on its own copy of the input) into a queue of command groups in
// LDS, wave 1 executes them on the ring (Out::lit / Out::copy) as they come.
constexpr uint32_t kQGroups = 4;              // groups of kWave commands in the queue
constexpr uint32_t kSpinCap = 1u << 22;       // polls before a wave gives up (ST_CORRUPT): no hang
enum : uint32_t { Q_PUB = 0, Q_DONE = 1, Q_END = 2, Q_ST = 3, Q_STOP = 4, Q_CTL = 8 };
// record word 0: bytes | kCmdCopy | kCmdSlow; word 1: input position (literal) / distance (copy)
constexpr uint32_t kCmdCopy = 1u << 31;
constexpr uint32_t kCmdSlow = 1u << 30;       // longer than a wave step, or a copy overlapping itself
constexpr uint32_t kCmdBytes = kCmdSlow - 1u;

__device__ __forceinline__ uint32_t vload(const lds32* a) { return *reinterpret_cast<const volatile lds32*>(a); }
__device__ __forceinline__ void vstore(lds32* a, uint32_t v) { *reinterpret_cast<volatile lds32*>(a) = v; }
__device__ __forceinline__ void wg_release() { __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup"); }
__device__ __forceinline__ void wg_acquire() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup"); }

// The parser's output: Out's interface (st, op, vbase, lit, copy) with
// Out's checks, each command appended to the open group (lane k holds
// command k), a full group published to the queue.
struct QSink {
    lds32* rec;       // kQGroups * kWave records of two words
    lds32* ctl;
    uint32_t ring;    // the executor's ring bytes (copies reach at most ring - 1 back)
    uint32_t st = ST_OK;
    uint32_t op, vbase, cap;
    uint32_t k = 0, g = 0;  // commands in the open group; groups published
    uint32_t rn = 0, rs = 0;
    __device__ __forceinline__ bool publish() {
        for (uint32_t spins = 0; g - vload(ctl + Q_DONE) >= kQGroups;) {
            if (vload(ctl + Q_STOP) || ++spins > kSpinCap) return false;
            __builtin_amdgcn_s_sleep(1);
        }
        wg_acquire();
        const uint32_t slot = (g % kQGroups) * kWave + lane();
        rec[2 * slot] = lane() < k ? rn : 0u;  // 0: no command (the group's end)
        rec[2 * slot + 1] = rs;
        wg_release();
        g++;
        if (lane() == 0) vstore(ctl + Q_PUB, g);
        k = 0;
        return true;
    }
    __device__ __forceinline__ void push(uint32_t w0, uint32_t w1) {
#if PQ_CODEC_PUSH_SKIP  // timing probe: commands checked, not queued
        return;
#endif
        // (selects, not a branch on the lane: no exec-mask round trip through
        // the scalar unit; v_writelane through M0 measured the same, r6t)
        const bool mine = lane() == k;
        rn = mine ? w0 : rn;
        rs = mine ? w1 : rs;
        if (++k == kWave && !publish()) st = ST_CORRUPT;
    }
    // (op <= cap holds throughout, so each check is one compare)
    template <class InX>
    __device__ __forceinline__ void lit(InX&, uint32_t p, uint32_t n) {
#if PQ_CODEC_CHECK_SKIP  // timing probe: commands counted only
        op += n;
        return;
#endif
        if (n > cap - op) { st = ST_SIZE; return; }
        push(n | (n > static_cast<uint32_t>(kWave) ? kCmdSlow : 0u), p);
        op += n;
    }
    __device__ __forceinline__ void copy(uint32_t d, uint32_t n) {
#if PQ_CODEC_CHECK_SKIP
        op += n;
        return;
#endif
        if (d - 1u >= min(op - vbase, ring - 1)) { st = ST_CORRUPT; return; }  // d in [1, min(history, ring - 1)]
        if (n > cap - op) { st = ST_SIZE; return; }
        if (n == 0) return;
        push(n | kCmdCopy | (n > static_cast<uint32_t>(kWave) || d < n ? kCmdSlow : 0u), d);
        op += n;
    }
    // the last group and the parse's status; Q_END after them
    __device__ __forceinline__ void finish() {
        if (k && !publish() && st == ST_OK) st = ST_CORRUPT;
        if (lane() == 0) {
            vstore(ctl + Q_ST, st);
            wg_release();
            vstore(ctl + Q_END, 1u);
        }
    }
};

// The executor: every published group, in order, until Q_END.
template <class InX, class OutT>
__device__ __forceinline__ void lz_execute(InX& I, OutT& O, const lds32* rec, lds32* ctl) {
    uint32_t g = 0, spins = 0;
    for (;;) {
        const uint32_t pub = vload(ctl + Q_PUB);
        if (g == pub) {
            if (vload(ctl + Q_END)) {
                wg_acquire();
                if (vload(ctl + Q_PUB) == g) break;
                continue;
            }
            if (++spins > kSpinCap) {
                O.st = ST_CORRUPT;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        spins = 0;
        wg_acquire();
        const uint32_t slot = (g % kQGroups) * kWave + lane();
        const uint32_t rn = rec[2 * slot], rs = rec[2 * slot + 1];
        // The parser has checked every command against the same counts (QSink
        // keeps Out's op), so a short command runs without checks and without
        // a branch on its kind: one source address per lane (ring or staged
        // input), one LDS read, one LDS write.
        const uint32_t ring0 = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(O.ring));
        const uint32_t in0 = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(I.w));
        for (uint32_t j = 0; j < (PQ_CODEC_EXEC_SKIP ? 0u : static_cast<uint32_t>(kWave)) && O.st == ST_OK; j++) {
            const uint32_t w = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(rn), static_cast<int>(j)));
            if (w == 0) break;
            const uint32_t a = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(rs), static_cast<int>(j)));
            const uint32_t n = w & kCmdBytes;
            if (w & kCmdSlow) {
                if (w & kCmdCopy) O.copy(a, n);
                else O.lit(I, a, n);
                continue;
            }
            const bool cp = (w & kCmdCopy) != 0;
            if (!cp) I.ensure(a, n);
            const uint32_t src = cp ? ring0 + ((O.op - a + lane()) & OutT::kMask) : in0 + (a + lane() - I.wlo + I.sh);
            if (lane() < n) O.ring[(O.op + lane()) & OutT::kMask] = *reinterpret_cast<const lds8*>(static_cast<uintptr_t>(src));
            O.op += n;
            if (O.op - O.fl >= kFlush) {
                wsync();
                O.flush(false);
            }
        }
        wsync();
        g++;
        if (lane() == 0) {
            if (O.st != ST_OK) vstore(ctl + Q_STOP, 1u);
            vstore(ctl + Q_DONE, g);
        }
    }
#if PQ_CODEC_EXEC_SKIP
    O.op = O.cap;  // (the size check passes; the output is not written)
#endif
    if (lane() == 0) vstore(ctl + Q_STOP, 1u);  // (a parser still waiting for room stops)
    const uint32_t ps = vload(ctl + Q_ST);
    if (O.st == ST_OK && vload(ctl + Q_END) && ps != ST_OK) O.st = ps;
}

// ── DEFLATE (deflate.hpp) on one wavefront ─────────────────────────────────
static_assert(pqinf::ST_OK == ST_OK && pqinf::ST_CORRUPT == ST_CORRUPT && pqinf::ST_SIZE == ST_SIZE, "status codes");
struct DevWave {
    static constexpr uint32_t kWave = static_cast<uint32_t>(pqk::kWave);
    static __device__ __forceinline__ uint32_t lane() { return dev::lane(); }
    static __device__ __forceinline__ void sync() { wsync(); }
    static __device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
    static __device__ __forceinline__ uint32_t bitrev(uint32_t v) { return __builtin_bitreverse32(v); }
};
__device__ __forceinline__ void gzip(CodecLds& L, In& I, Out<true>& O, uint32_t p, uint32_t end) {
    pqinf::gzip<DevWave>(L, I, O, p, end);
}

// ZSTD's LDS (k_codec<2>): a 32 KiB ring (matches farther back read the
// flushed slot), the staged input and the decode tables, 59 KiB in all, so
// two pages share a CU (CodecLds with the tables: 91 KiB, one)
constexpr uint32_t kZRing = 32768;
template <uint32_t kRingB, uint32_t kWin>
struct ZCodecLdsT {
    uint8_t ring[kRingB];
    uint8_t in[kWin + 32];
    uint8_t zstage[64];
    zs::ZTables T;
};
using ZCodecLds = ZCodecLdsT<kZRing, kInWin>;
// the small-page layouts (pages under kSRing bytes)
struct SCodecLds {
    uint8_t ring[kSRing];
    uint8_t in[kSWin + 32];
};
using ZSCodecLds = ZCodecLdsT<kSRing, kSWin>;

// ── ZSTD adapters (zstd.hpp's source and output over In and the ring) ────
template <class InX>
struct ZSrc {
    InX* I;
    uint32_t base, len;  // the zstd stream: input bytes [base, base + len)
    __device__ __forceinline__ uint32_t byte(uint32_t q) const {
        if (q >= len) return 0u;
        const uint32_t p = base + q;
        // the decoder reads forward (headers, raw blocks) and backward (bit
        // streams): refill with p mid-window
        constexpr uint32_t w = InX::kWindow;
        if (p < I->wlo || p + 1 + I->sh > I->wlo + w) I->refill(p > w / 2 ? p - w / 2 : 0u);
        return I->byte(p);
    }
};

template <class OutT, class InX>
struct ZOut {
    OutT* O;
    InX* I;
    uint32_t base;         // input offset of the zstd stream (raw blocks)
    lds8* stage;           // 64 literal bytes on their way to the slot
    uint32_t litbase = 0;  // slot offset of the block's literals: its tail, past every byte still to be written
    uint32_t nlit = 0, lp = 0, lk0 = 0, ln = 0;
    __device__ __forceinline__ bool lit_begin(uint32_t n) {
        if (O->st != ST_OK || n > O->cap - O->op) return false;
        litbase = O->cap - n;
        nlit = n;
        lp = 0;
        ln = 0;
        return true;
    }
    __device__ __forceinline__ void lit_flush() {
        wsync();
        if (lane() < ln) O->dst[litbase + lk0 + lane()] = stage[lane()];
        ln = 0;
        wsync();
    }
    __device__ __forceinline__ void lit_at(uint32_t k, uint32_t b) {
        if (ln && k != lk0 + ln) lit_flush();
        if (ln == 0) lk0 = k;
        if (lane() == 0) stage[ln] = static_cast<uint8_t>(b);
        ln++;
        if (ln == kWave) lit_flush();
    }
    __device__ __forceinline__ void visible() {  // this wave's global stores -> its later global loads
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __device__ __forceinline__ void lit_done() {
        if (ln) lit_flush();
        visible();
    }
    __device__ __forceinline__ bool lits(uint32_t n) {
        if (lp + n > nlit || !O->room(n)) return false;
        for (uint32_t d = 0; d < n; d += kWave) {
            const uint32_t m = min(static_cast<uint32_t>(kWave), n - d);
            if (lane() < m) O->ring[(O->op + lane()) & OutT::kMask] = O->dst[litbase + lp + d + lane()];
            O->op += m;
            wsync();
            if (O->op - O->fl >= kFlush) O->flush(false);
        }
        lp += n;
        return O->st == ST_OK;
    }
    __device__ __forceinline__ bool raw(uint32_t p, uint32_t n) {
        O->lit(*I, base + p, n);
        return O->st == ST_OK;
    }
    __device__ __forceinline__ bool rle(uint32_t b, uint32_t n) {
        if (!O->room(n)) return false;
        for (uint32_t d = 0; d < n; d += kWave) {
            const uint32_t m = min(static_cast<uint32_t>(kWave), n - d);
            if (lane() < m) O->ring[(O->op + lane()) & OutT::kMask] = static_cast<uint8_t>(b);
            O->op += m;
            wsync();
            if (O->op - O->fl >= kFlush) O->flush(false);
        }
        return true;
    }
    __device__ __forceinline__ uint32_t copy(uint32_t off, uint32_t n) {
        if (off == 0 || off > O->op - O->vbase) return zs::ZS_CORRUPT;
        if (off < OutT::kRingSize - 2 * kFlush) {  // from the ring
            O->copy(off, n);
            return O->st == ST_OK ? zs::ZS_OK : (O->st == ST_SIZE ? zs::ZS_SIZE : zs::ZS_CORRUPT);
        }
        // farther back than the ring: every source byte is flushed (the ring
        // keeps < kFlush unflushed bytes), read from the slot
        if (!O->room(n)) return zs::ZS_SIZE;
        for (uint32_t d = 0; d < n; d += kWave) {
            visible();
            const uint32_t m = min(static_cast<uint32_t>(kWave), n - d);
            if (lane() < m) O->ring[(O->op + lane()) & OutT::kMask] = O->dst[O->op + lane() - off];
            O->op += m;
            wsync();
            if (O->op - O->fl >= kFlush) O->flush(false);
        }
        return zs::ZS_OK;
    }
};

// kGzip: the GZIP instantiation (CRC-32 on, DEFLATE); the other one takes
// every other codec and the V2 rebuild.  A chunk has one codec, so one
// launch takes one instantiation (launch_codec).  kSmall: the small-page
// layout (SCodecLds / ZSCodecLds), over the entries whose payload is under
// kSRing bytes; the full layout takes the rest (each launch skips the others).
// The kind-0 layouts: the executor's ring and window where CodecLds /
// SCodecLds have them, then the parser's window and the command queue.
template <uint32_t kRingB, uint32_t kWinB, uint32_t kPWinB>
struct LzLdsT {
    uint8_t ring[kRingB];
    uint8_t in[kWinB + 32];
    uint8_t pin[kPWinB + 32];
    uint32_t rec[2 * kQGroups * kWave];
    uint32_t ctl[Q_CTL];
};
constexpr uint32_t kPWin = 2048;  // the parser's staged input (full layout): headers only
using LzLds = LzLdsT<kRing, kInWin, kPWin>;
using LzSLds = LzLdsT<kSRing, kSWin, kSWin>;
static_assert(offsetof(LzLds, in) == offsetof(CodecLds, in) && offsetof(LzSLds, in) == offsetof(SCodecLds, in),
              "kind 0 keeps the ring and window offsets");
static_assert(offsetof(LzLds, rec) % 8 == 0 && offsetof(LzSLds, rec) % 8 == 0, "record alignment");
static_assert(offsetof(LzLds, rec) - offsetof(LzLds, pin) == kPWin + 32 &&
              offsetof(LzSLds, rec) - offsetof(LzSLds, pin) == kSWin + 32, "the parser's window and its staging size");

template <int kKind>
constexpr int codec_threads() { return kKind == 0 ? 2 * kWave : kWave; }

template <int kKind, bool kSmall>
__global__ void __launch_bounds__(codec_threads<kKind>()) k_codec(const uint8_t* __restrict__ src, uint8_t* __restrict__ img,
                                                 const CodecEntry* __restrict__ ent, int32_t n,
                                                 uint32_t* __restrict__ status) {
    constexpr bool kGzip = kKind == 1, kZstd = kKind == 2;
    constexpr bool kPipe = kKind == 0;  // SNAPPY / LZ4 on two waves (parser 0, executor 1)
    static_assert(!(kGzip && kSmall), "GZIP keeps the full layout (its Huffman tables)");
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    CodecLds& L = *reinterpret_cast<CodecLds*>(smem);
    constexpr size_t kRingOff = kSmall ? (kZstd ? offsetof(ZSCodecLds, ring) : offsetof(SCodecLds, ring))
                                       : (kZstd ? offsetof(ZCodecLds, ring) : offsetof(CodecLds, ring));
    constexpr size_t kInOff = kSmall ? (kZstd ? offsetof(ZSCodecLds, in) : offsetof(SCodecLds, in))
                                     : (kZstd ? offsetof(ZCodecLds, in) : offsetof(CodecLds, in));
    lds8* lring = (lds8*)(smem + kRingOff);
    lds8* lin = (lds8*)(smem + kInOff);
    using OutK = Out<kGzip, kSmall ? kSRing : (kZstd ? kZRing : kRing)>;
    using InK = typename std::conditional<kSmall, InS, In>::type;
    lds32* lcrc = (lds32*)(smem + offsetof(CodecLds, crc_tab));
    if constexpr (kGzip) {
        for (uint32_t b = lane(); b < 256; b += kWave) {  // CRC-32 byte table
            uint32_t c = b;
            for (int k = 0; k < 8; k++) c = (c >> 1) ^ ((0u - (c & 1u)) & kCrcPoly);
            lcrc[b] = c;
        }
        wsync();
    }
    using LL = typename std::conditional<kSmall, LzSLds, LzLds>::type;
    lds32* qrec = (lds32*)(smem + offsetof(LL, rec));
    lds32* qctl = (lds32*)(smem + offsetof(LL, ctl));
    const uint32_t wv = kPipe ? threadIdx.x / kWave : 1u;
    for (int32_t i = static_cast<int32_t>(blockIdx.x); i < n; i += static_cast<int32_t>(gridDim.x)) {
        const CodecEntry e = ent[i];
        if (!kGzip && (e.out_len < kSRing) != kSmall) continue;  // the other layout's page
        const bool lz = kPipe && (e.codec == 1 || e.codec == 5 || e.codec == 7);
        if constexpr (kPipe) {
            __syncthreads();  // both waves are done with the previous entry's queue
            if (threadIdx.x == kWave)
                for (uint32_t c = 0; c < Q_CTL; c++) vstore(qctl + c, 0u);
            __syncthreads();
            if (wv == 0) {  // the parser
                if (lz) {
                    using InP = InT<kSmall ? kSWin : kPWin>;  // (the size of LL::pin)
                    InP Ip{src + e.src, e.src_len, 0u, 0u, (lds8*)(smem + offsetof(LL, pin))};
                    Ip.refill(0);
                    QSink Q{qrec, qctl, OutK::kRingSize};
                    uint32_t p = 0, vb = 0;
                    if (e.flags & kCodecV2) {  // (the executor writes the level sections)
                        p = e.def_len + e.rep_len;
                        vb = ((e.flags & kCodecDefPrefix) ? 4 + e.def_len : 0u) + ((e.flags & kCodecRepPrefix) ? 4 + e.rep_len : 0u);
                        if (p > e.src_len) Q.st = ST_CORRUPT;
                    }
                    Q.op = vb;
                    Q.vbase = vb;
                    Q.cap = e.out_len;
                    if (Q.st == ST_OK) {
                        if (e.codec == 1) snappy(Ip, Q, p, e.src_len, e.out_len - vb);
                        else if (e.codec == 5) lz4_hadoop(Ip, Q, p, e.src_len);
                        else lz4_block(Ip, Q, p, e.src_len);
                    }
                    Q.finish();
                }
                continue;
            }
        }
        InK I{src + e.src, e.src_len, 0u, 0u, lin};
        I.refill(0);
        OutK O{lring, img + e.dst, 0u, 0u, e.out_len, 0u, ST_OK};
        O.crc_tab = lcrc;
        uint32_t p = 0;
        if (e.flags & kCodecV2) {  // level sections, as is, behind their V1 length prefixes
            const uint32_t lv = e.def_len + e.rep_len;
            if (lv > e.src_len) O.st = ST_CORRUPT;
            // V2 pages hold repetition then definition levels; the reference reads
            // [u32 def_len][def][u32 rep_len][rep] (column_reader.cpp:146-170)
            if (O.st == ST_OK && (e.flags & kCodecDefPrefix)) {
                O.put_u32(e.def_len);
                if (O.st == ST_OK && e.def_len) O.lit(I, e.rep_len, e.def_len);
            }
            if (O.st == ST_OK && (e.flags & kCodecRepPrefix)) {
                O.put_u32(e.rep_len);
                if (O.st == ST_OK && e.rep_len) O.lit(I, 0, e.rep_len);
            }
            p = lv;
        }
        O.vbase = O.op;
        const uint32_t end = e.src_len;
        const uint32_t expect = e.out_len - O.op;
        if (O.st == ST_OK) {
            if constexpr (kGzip) {
                if (e.codec == 2) gzip(L, I, O, p, end);
                else if (e.codec == 0) O.lit(I, p, end - p);
                else O.st = ST_UNSUPPORTED;
            } else {
                switch (e.codec) {
                    case 0: O.lit(I, p, end - p); break;
                    case 1: case 5: case 7:
                        if constexpr (kPipe) {
                            lz_execute(I, O, qrec, qctl);
                            break;
                        } else {
                            if (e.codec == 1) snappy(I, O, p, end, expect);
                            else if (e.codec == 5) lz4_hadoop(I, O, p, end);
                            else lz4_block(I, O, p, end);
                            break;
                        }
                    case 6:
                        if constexpr (kZstd) {
                            // the tables after the ring and the window (this instantiation's launch only)
                            using ZL = typename std::conditional<kSmall, ZSCodecLds, ZCodecLds>::type;
                            zs::ZTables& T = *reinterpret_cast<zs::ZTables*>(smem + offsetof(ZL, T));
                            const ZSrc<InK> zsrc{&I, p, end - p};
                            ZOut<OutK, InK> zo{&O, &I, p, (lds8*)(smem + offsetof(ZL, zstage))};
                            const uint32_t st = zs::decompress(zsrc, end - p, T, zo);
                            if (O.st == ST_OK && st != zs::ZS_OK)
                                O.st = st == zs::ZS_SIZE ? ST_SIZE : (st == zs::ZS_UNSUPPORTED ? ST_UNSUPPORTED : ST_CORRUPT);
                            break;
                        }
                        O.st = ST_UNSUPPORTED;
                        break;
                    default: O.st = ST_UNSUPPORTED;  // (GZIP: the other instantiation)
                }
            }
        }
        if constexpr (kPipe)  // (a parser still waiting for room stops: e.g. a bad V2 prologue)
            if (lz && lane() == 0) vstore(qctl + Q_STOP, 1u);
        if (O.st == ST_OK && O.op != e.out_len) O.st = ST_SIZE;
        if (O.st == ST_OK) O.flush(true);
        if (lane() == 0) status[i] = O.st;
        wsync();
    }
}

}  // namespace

size_t codec_lds_bytes() { return sizeof(CodecLds); }

template <int kKind, bool kSmall>
static void codec_launch(hipStream_t s, const uint8_t* src, uint8_t* img, const CodecEntry* ent, int32_t n,
                         uint32_t* status, int cus, uint32_t lds, int32_t pages) {
    const void* k = reinterpret_cast<const void*>(k_codec<kKind, kSmall>);
    ensure_dyn_lds(k, lds);
    const int per_cu = std::max(1, resident_blocks(k, codec_threads<kKind>(), lds));
    const int grid = std::min(std::max(pages, 1), std::max(1, cus) * per_cu);
    hipLaunchKernelGGL((k_codec<kKind, kSmall>), dim3(grid), dim3(codec_threads<kKind>()), lds, s, src, img, ent, n, status);
}

void launch_codec(hipStream_t s, const uint8_t* src, uint8_t* img, const CodecEntry* ent, int32_t n,
                  uint32_t* status, int cus, int kind, int32_t nsmall) {
    if (n <= 0) return;
    // kind 2 (ZSTD): its own layout (a smaller ring and the decode tables);
    // nsmall: entries whose payload is under kSRing (the small-page layout)
    const int32_t nbig = kind == 1 ? n : n - nsmall;
    if (kind == 1) codec_launch<1, false>(s, src, img, ent, n, status, cus, sizeof(CodecLds), n);
    if (kind == 2) {
        if (nsmall > 0) codec_launch<2, true>(s, src, img, ent, n, status, cus, sizeof(ZSCodecLds), nsmall);
        if (nbig > 0) codec_launch<2, false>(s, src, img, ent, n, status, cus, sizeof(ZCodecLds), nbig);
    }
    if (kind == 0) {
        if (nsmall > 0) codec_launch<0, true>(s, src, img, ent, n, status, cus, sizeof(LzSLds), nsmall);
        if (nbig > 0) codec_launch<0, false>(s, src, img, ent, n, status, cus, sizeof(LzLds), nbig);
    }
}

uint32_t codec_small_bytes() { return kSRing; }

}  // namespace pqk
