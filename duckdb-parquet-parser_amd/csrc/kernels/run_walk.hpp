// run_walk.hpp — the lock-step run-header walk shared by the run-table
// kernels (dict_pipe.hip k_pipe_runs, fixed_fast.hip k_fixed_levels2): one
// hybrid RLE/bit-packed stream per lane (rle_decoder.hpp:36-95), one run
// record per step.
#pragma once
#include <type_traits>
#include "kernels/device_common.hpp"
#include "kernels/lane_walk.hpp"

namespace pqk {
namespace dev {

// One hybrid stream per lane, walked with every lane in lock step: each
// step parses one run header (rle_decoder.hpp:36-95) and appends one record.
struct RunWalk {
    bool alive;
    uint32_t q, end, bw, n, sbase, cap;
    uint2* out;
    const uint8_t* gp;
};

// kPair: records go out two at a time as one 16-byte store (W.out 16-byte
// aligned, nrec even on entry): half the store instructions, whole 16-byte
// pieces of the record lines instead of 8-byte ones
template <bool kStaged, bool kPair = false>
__device__ __forceinline__ void walk_runs(RunWalk& W, const uint32_t* stage, uint32_t& flag, uint32_t& nrec,
                                          bool nostore = false) {  // nostore: timing ablation only
    const uint32_t nbv = (W.bw + 7) / 8;
    const uint32_t vmask = nbv >= 2 ? 0xFFFFu : (nbv ? 0xFFu : 0u);
    const uint32_t litpay = W.bw ? 0x80000000u : 0u;
    const uint32_t litsh = W.bw ? 0xFFFFFFFFu : 0u;  // literal payload: bit offset qh * 8 when bw > 0
    uint32_t cnt = 0, q = W.q, nr = nrec, fl = flag;
    bool alive = W.alive && W.n > 0;
    // eight bytes at stream position qq; the next header's bytes are loaded
    // as soon as its position is known, so the load's latency overlaps the
    // current step's record (a lane that stops keeps its position)
    auto load = [&](uint32_t qq, bool live, uint32_t& x0, uint32_t& x1) {
        if (kStaged) {
            const uint32_t a = W.sbase + qq, wi = a >> 2, sh = a & 3;
            const uint32_t w0 = stage[wi], w1 = stage[wi + 1], w2 = stage[wi + 2];
            x0 = __builtin_amdgcn_alignbyte(w1, w0, sh);
            x1 = __builtin_amdgcn_alignbyte(w2, w1, sh);
        } else {
            const uint64_t x = live ? gld8(W.gp, qq) : 0ull;
            x0 = static_cast<uint32_t>(x);
            x1 = static_cast<uint32_t>(x >> 32);
        }
    };
    uint32_t x0, x1;
    load(q, alive, x0, x1);
    uint2 held = make_uint2(0u, 0u);  // kPair: the record at an even index, waiting for its partner
    // branch-free step: every quantity is computed, one predicated store.
    // kOne: every live header is one byte (runs of < 64 values or groups:
    // what both writers emit for these pages), so the varint parse, the
    // header-length selects and the 2^16 group clamp fold away.
    auto step = [&](auto one) {
        constexpr bool kOne = decltype(one)::value;
        const uint32_t exh = q >= W.end ? 1u : 0u;  // rest of the batch is 0 (rle_decoder.hpp:20-23)
        // varint header (76-86): at most 5 bytes, inside the stream
        uint32_t hl, ind;
        if constexpr (kOne) {
            hl = 1;
            ind = x0 & 0x7Fu;
        } else {
            const uint32_t st0 = ~x0 & 0x80808080u;
            const uint32_t hl4 = (__builtin_ctz(st0 | 0x80000000u) >> 3) + 1;
            const uint32_t hl5 = (~x1 & 0x80u) ? 5u : 9u;
            hl = st0 ? hl4 : hl5;
            const uint32_t lm = (hl >= 4) ? 0xFFFFFFFFu : ((1u << (8 * (hl & 3))) - 1u);
            const uint32_t x0m = x0 & lm;
            const uint32_t top = (hl >= 5) ? (x1 << 28) : 0u;
            ind = (x0m & 0x7Fu) | ((x0m >> 1) & 0x3F80u) | ((x0m >> 2) & 0x1FC000u) | ((x0m >> 3) & 0xFE00000u) | top;
        }
        const uint32_t g = ind >> 1;
        const uint32_t lit = ind & 1u;
        const uint32_t left = W.n - cnt;
        const uint32_t qh = q + hl;
        const uint32_t cl = (g >= (left + 7) / 8) ? left : g * 8;
        const uint32_t cr = min(g, left);
        const uint32_t c = lit ? cl : cr;
        // zero-count runs (counter wrap / stale literal cursor), truncated headers or values
        const uint32_t badh = (!kOne && hl > 5 ? 1u : 0u) | (qh > W.end ? 1u : 0u) | (g == 0 ? 1u : 0u) |
                              ((lit ^ 1u) & (qh + nbv > W.end ? 1u : 0u));
        const uint32_t full = nr >= W.cap ? 1u : 0u;
        const uint32_t ok = (alive ? 1u : 0u) & (full ^ 1u) & (exh | (badh ^ 1u));
        // selects by mask (the compiler turns a ternary on `lit` into a branch)
        const uint32_t litm = 0u - lit;
        // g clamps at 2^16: a longer literal run overruns the stream (<= 64 KiB) either way
        // (24-bit multiplies: g <= 2^16, bw <= 32)
        const uint32_t nqlc = min(__umul24(kOne ? g : min(g, 0x10000u), W.bw) + qh, W.end);
        const uint32_t nq = (litm & nqlc) | (~litm & (qh + nbv));
        const uint32_t ncnt = exh ? W.n : cnt + c;
        const uint32_t qn = (ok & (exh ^ 1u)) ? nq : q;
        const bool an = ok && !exh && ncnt < W.n;
        uint32_t y0, y1;
        load(qn, an, y0, y1);
        const uint32_t rx = cnt | ((exh ? left : c) << 16);
        uint32_t vraw;
        if constexpr (kOne) {
            vraw = x0 >> 8;  // the RLE value's (<= 2) bytes after the header
        } else {
            const uint32_t va = __builtin_amdgcn_alignbyte(x1, x0, hl);
            const uint32_t vb = x1 >> (8 * ((hl - 4) & 3));
            vraw = (hl < 4) ? va : vb;
        }
        const uint32_t pl = (litm & (litpay | ((qh << 3) & litsh))) | (~litm & vraw & vmask);
        const uint32_t ry = exh ? 0u : pl;
        if constexpr (kPair) {
            if (ok && (nr & 1u) && !nostore) *reinterpret_cast<uint4*>(W.out + nr - 1) = make_uint4(held.x, held.y, rx, ry);
            if (ok && !(nr & 1u)) held = make_uint2(rx, ry);
        } else {
            if (ok) W.out[nr] = make_uint2(rx, ry);
        }
        fl |= (alive ? 1u : 0u) & (ok ^ 1u);
        nr += ok;
        cnt = ncnt;
        q = qn;
        alive = an;
        x0 = y0;
        x1 = y1;
    };
    while (__ballot(alive)) {
        if (__ballot(alive && q < W.end && (x0 & 0x80u)) == 0) step(std::true_type{});
        else step(std::false_type{});
    }
    if constexpr (kPair) {
        if (nr & 1u) W.out[nr - 1] = held;
    }
    nrec = nr;
    flag = fl;
}

}  // namespace dev
}  // namespace pqk
