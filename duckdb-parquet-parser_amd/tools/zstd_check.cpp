// zstd_check.cpp — host build of the codec pass's zstd decoder
// (csrc/kernels/zstd.hpp) for the CPU tests (tests/test_zstd_host.py): the
// same source the GPU runs, over plain memory, pinned against pyarrow's zstd.
// Test infrastructure only; the product decodes ZSTD pages in k_codec.
#include <cstdint>
#include <cstring>
#include <vector>
#define ZS_HD inline
#include "kernels/zstd.hpp"

namespace {
struct HSrc {
    const uint8_t* d;
    uint32_t n;
    uint32_t byte(uint32_t p) const { return p < n ? d[p] : 0u; }
};
struct HOut {
    const HSrc* src;
    uint8_t* dst;
    uint32_t cap, op = 0;
    std::vector<uint8_t> lit;
    uint32_t lp = 0;
    bool lit_begin(uint32_t n) {
        lit.assign(n, 0);
        lp = 0;
        return true;
    }
    void lit_at(uint32_t k, uint32_t b) {
        if (k < lit.size()) lit[k] = static_cast<uint8_t>(b);
    }
    void lit_done() {}
    bool lits(uint32_t n) {
        if (lp + n > lit.size() || op + n > cap) return false;
        std::memcpy(dst + op, lit.data() + lp, n);
        lp += n;
        op += n;
        return true;
    }
    bool raw(uint32_t p, uint32_t n) {
        if (op + n > cap) return false;
        for (uint32_t i = 0; i < n; i++) dst[op + i] = static_cast<uint8_t>(src->byte(p + i));
        op += n;
        return true;
    }
    bool rle(uint32_t b, uint32_t n) {
        if (op + n > cap) return false;
        std::memset(dst + op, static_cast<int>(b), n);
        op += n;
        return true;
    }
    uint32_t copy(uint32_t off, uint32_t n) {
        if (off > op) return zs::ZS_CORRUPT;
        if (op + n > cap) return zs::ZS_SIZE;
        for (uint32_t i = 0; i < n; i++) dst[op + i] = dst[op + i - off];
        op += n;
        return zs::ZS_OK;
    }
};
}  // namespace

extern "C" int zs_decompress(const uint8_t* src, uint32_t len, uint8_t* dst, uint32_t cap, uint32_t* out_len) {
    static zs::ZTables T;
    HSrc s{src, len};
    HOut o{&s, dst, cap};
    const uint32_t st = zs::decompress(s, len, T, o);
    *out_len = o.op;
    return static_cast<int>(st);
}
