// gzip_check.cpp — host build of the codec pass's DEFLATE decoder
// (csrc/kernels/deflate.hpp: GZIP members / one zlib stream) for the CPU
// tests (tests/test_gzip_host.py) and the sanitizer fuzz driver
// (tools/fuzz_host.cpp `gzip`): the same decoder the GPU runs, on one lane,
// with an output that applies k_codec's Out checks (codec.hip: a byte must
// fit the page, a copy's distance must lie in [1, min(history, 65,535)]) and
// writes an exact-size buffer, so ASan sees any command the checks let
// through that reaches outside the input or the output.  The GZIP CRC-32 is
// kept over the output as the device keeps it over its ring.
// Test infrastructure only; the product decodes GZIP pages in k_codec.
#include <cstdint>
#include <cstring>
#include <memory>
#define DF_HD inline
#define DF_CONST constexpr
#include "kernels/deflate.hpp"

namespace {
struct HWave {
    static constexpr uint32_t kWave = 1;
    static uint32_t lane() { return 0; }
    static void sync() {}
    static uint32_t uni(uint32_t v) { return v; }
    static uint32_t bitrev(uint32_t v) {
        uint32_t r = 0;
        for (int i = 0; i < 32; i++) r |= ((v >> i) & 1u) << (31 - i);
        return r;
    }
};
struct HLds {  // k_codec's CodecLds tables
    uint16_t lt[1 << pqinf::kFast];
    uint16_t dt[1 << pqinf::kFast];
    uint16_t sym[320];
    uint16_t code[320];
    uint16_t cnt[2][16];
    uint8_t lens[320];
    uint16_t nxt[16], offs[16];
    uint32_t scratch[4];
};
struct HIn {
    const uint8_t* d;
    uint32_t n;
    void ensure(uint32_t, uint32_t) {}
    uint32_t byte(uint32_t p) const { return p < n ? d[p] : 0u; }  // (the device window reads zeros past the page)
    uint32_t u16le(uint32_t p) const { return byte(p) | (byte(p + 1) << 8); }
    uint32_t u32le(uint32_t p) const { return u16le(p) | (u16le(p + 2) << 16); }
};
constexpr uint32_t kRing = 65536;  // k_codec's GZIP history
struct HOut {
    uint8_t* dst;
    uint32_t cap;
    uint32_t st = pqinf::ST_OK, op = 0;
    static constexpr uint32_t kCrcSlack = 1024;
    bool crc_on = false;
    uint32_t crc = 0, crc_pos = 0;
    bool room(uint32_t n) {
        if (op + n > cap || op + n < op) { st = pqinf::ST_SIZE; return false; }
        return true;
    }
    void lit(HIn& I, uint32_t p, uint32_t n) {
        if (!room(n)) return;
        std::memcpy(dst + op, I.d + p, n);  // (inflate has checked p + n <= the input's end)
        op += n;
    }
    void put1(uint32_t b) {
        if (!room(1)) return;
        dst[op++] = static_cast<uint8_t>(b);
    }
    void copy(uint32_t d, uint32_t n) {
        if (d == 0 || d > op || d > kRing - 1) { st = pqinf::ST_CORRUPT; return; }
        if (!room(n)) return;
        for (uint32_t i = 0; i < n; i++) dst[op + i] = dst[op + i - d];
        op += n;
    }
    void crc_keep() {}
    void crc_upto(uint32_t to) {  // CRC-32 (reflected 0xEDB88320) of bytes [crc_pos, to), finalized form
        if (!crc_on || to <= crc_pos) return;
        uint32_t c = ~crc;
        for (uint32_t q = crc_pos; q < to; q++) {
            c ^= dst[q];
            for (int k = 0; k < 8; k++) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
        }
        crc = ~c;
        crc_pos = to;
    }
};
}  // namespace

// One GZIP / zlib page payload into dst (cap = the page's uncompressed
// size).  Returns the status (0 ok, 1 corrupt, 2 size); *out_len = bytes
// produced.
extern "C" int gz_decompress(const uint8_t* src, uint32_t len, uint8_t* dst, uint32_t cap, uint32_t* out_len) {
    auto L = std::make_unique<HLds>();
    HIn I{src, len};
    HOut O{dst, cap};
    pqinf::gzip<HWave>(*L, I, O, 0, len);
    if (O.st == pqinf::ST_OK && O.op != cap) O.st = pqinf::ST_SIZE;  // k_codec: the page must fill its slot
    *out_len = O.op;
    return static_cast<int>(O.st);
}
