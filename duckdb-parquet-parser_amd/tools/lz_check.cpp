// lz_check.cpp — host build of the codec pass's SNAPPY and LZ4 parsers
// (csrc/kernels/lz.hpp) for the CPU tests (tests/test_lz_host.py) and the
// sanitizer fuzz driver (tools/fuzz_host.cpp `lz`): the same parse the GPU
// runs, over plain memory, with an output that applies k_codec's QSink checks
// (codec.hip: a literal must fit the output, a copy's distance must lie in
// [1, min(history, ring - 1)] and its bytes fit) and then executes the
// command on an exact-size buffer, so ASan sees any command the checks let
// through that reads or writes outside the input or the output.
// Test infrastructure only; the product decodes these pages in k_codec.
#include <cstdint>
#include <cstring>
#define LZ_HD inline
#include "kernels/lz.hpp"

namespace {
struct HIn {
    const uint8_t* d;
    uint32_t n;
    void ensure(uint32_t, uint32_t) {}
    uint32_t byte(uint32_t p) const { return p < n ? d[p] : 0u; }  // (the device window reads zeros past the page)
    uint32_t u32be(uint32_t p) const { return (byte(p) << 24) | (byte(p + 1) << 16) | (byte(p + 2) << 8) | byte(p + 3); }
};
struct HWin {
    HIn* I;
    void need(uint32_t, uint32_t) {}
    uint32_t byte(uint32_t q) const { return I->byte(q); }
    uint32_t u16le(uint32_t q) const { return byte(q) | (byte(q + 1) << 8); }
    uint32_t u32le(uint32_t q) const { return byte(q) | (byte(q + 1) << 8) | (byte(q + 2) << 16) | (byte(q + 3) << 24); }
    static uint32_t uni(uint32_t v) { return v; }
};
struct HSink {
    uint8_t* dst;
    uint32_t cap, ring;
    uint32_t st = pqlz::ST_OK, op = 0, vbase = 0;
    void lit(HIn& I, uint32_t p, uint32_t n) {
        if (n > cap - op) { st = pqlz::ST_SIZE; return; }
        std::memcpy(dst + op, I.d + p, n);  // (the parser has checked p + n <= the input's end)
        op += n;
    }
    void copy(uint32_t d, uint32_t n) {
        const uint32_t hist = op - vbase < ring - 1 ? op - vbase : ring - 1;
        if (d - 1u >= hist) { st = pqlz::ST_CORRUPT; return; }
        if (n > cap - op) { st = pqlz::ST_SIZE; return; }
        for (uint32_t i = 0; i < n; i++) dst[op + i] = dst[op + i - d];
        op += n;
    }
};
}  // namespace

// codec 1 SNAPPY, 5 LZ4 (Hadoop framing), 7 LZ4_RAW; cap: the page's
// uncompressed size; ring: the executor's history bytes (65,536, or 8,192 for
// k_codec's small-page layout).  Returns the status (0 ok, 1 corrupt, 2 size;
// 4 for an unknown codec); *out_len = bytes produced.
extern "C" int lz_decompress(int codec, const uint8_t* src, uint32_t len, uint8_t* dst, uint32_t cap, uint32_t ring,
                             uint32_t* out_len) {
    HIn I{src, len};
    HSink O{dst, cap, ring};
    if (codec == 1) pqlz::snappy<HWin>(I, O, 0, len, cap);
    else if (codec == 5) pqlz::lz4_hadoop<HWin>(I, O, 0, len);
    else if (codec == 7) pqlz::lz4_block<HWin>(I, O, 0, len);
    else return 4;
    if (O.st == pqlz::ST_OK && O.op != cap) O.st = pqlz::ST_SIZE;  // k_codec: the page must fill its slot
    *out_len = O.op;
    return static_cast<int>(O.st);
}
