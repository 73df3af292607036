// run_spec.hpp — one hybrid RLE/bit-packed stream's run records built by the
// whole workgroup (rle_decoder.hpp:36-95), the same records walk_runs
// (run_walk.hpp) writes one header at a time:
//   x = first value | count << 16, y = literal << 31 | payload
// (RLE value, or the page bit offset of the literal run's first value).
// A stream of a few hundred runs is a long serial chain for one lane; here
//   1. every byte of the stream is parsed as if a run header started there:
//      the next header's position or kSpStop (bad header, stream end);
//   2. kSpJumpLog pointer-doubling rounds give kSpJump-run jumps;
//   3. one lane follows the jumps from the stream start, listing every
//      kSpJump-th header (a few dozen dependent LDS reads);
//   4. one thread per listed header re-parses its kSpJump runs exactly, with
//      untruncated counts;
//   5. a scan of the counts gives every record its first value; records past
//      the value count drop, the crossing one is truncated, an exhausted
//      stream gets its zero run (rle_decoder.hpp:20-23).
// Zero-count runs, headers cut by the stream end and table overflow before
// the value count return ~0u (the caller takes its exact serial path).
#pragma once
#include "kernels/device_common.hpp"

namespace pqk {
namespace dev {

constexpr uint32_t kSpStop = 0xFFFFu;
constexpr int kSpJumpLog = 4;
constexpr uint32_t kSpJump = 1u << kSpJumpLog;
constexpr uint32_t kSpCountCap = 1u << 20;

struct SpecHdr {
    uint32_t hl, g, lit, qh, vraw;
};
// A run header at LDS byte q of the staged words (the walk_runs parse).
__device__ __forceinline__ SpecHdr spec_hdr(const uint32_t* stw, uint32_t q) {
    const uint64_t x = lds_u64(stw, q);
    const uint32_t x0 = static_cast<uint32_t>(x), x1 = static_cast<uint32_t>(x >> 32);
    const uint32_t st0 = ~x0 & 0x80808080u;
    SpecHdr h;
    h.hl = st0 ? (__builtin_ctz(st0) >> 3) + 1 : ((~x1 & 0x80u) ? 5u : 9u);
    const uint32_t lm = (h.hl >= 4) ? 0xFFFFFFFFu : ((1u << (8 * (h.hl & 3))) - 1u);
    const uint32_t x0m = x0 & lm;
    const uint32_t top = (h.hl >= 5) ? (x1 << 28) : 0u;
    const uint32_t ind = (x0m & 0x7Fu) | ((x0m >> 1) & 0x3F80u) | ((x0m >> 2) & 0x1FC000u) |
                         ((x0m >> 3) & 0xFE00000u) | top;
    h.g = ind >> 1;
    h.lit = ind & 1u;
    h.qh = q + h.hl;
    const uint32_t va = __builtin_amdgcn_alignbyte(x1, x0, h.hl);
    const uint32_t vb = x1 >> (8 * ((h.hl - 4) & 3));
    h.vraw = (h.hl < 4) ? va : vb;
    return h;
}
// zero-count runs, headers past the stream end, RLE values cut by it
__device__ __forceinline__ bool spec_bad(const SpecHdr& h, uint32_t e, uint32_t nbv) {
    return h.hl > 5 || h.qh > e || h.g == 0 || (!h.lit && h.qh + nbv > e);
}

// The stream is at staged bytes [base, base + len) of `stw` (the page from
// byte 0, so staged positions are page positions), len <= kThreads *
// kPerThread.  Scratch: tab (len u16), list and esum (lcap u32 each), sh (4
// u32).  Records go to rec[0 .. rcap).  Every thread of the workgroup calls
// this (it holds barriers); returns the record count or ~0u.
template <int kThreads, int kPerThread, bool kBlocked = false, int kJumpLog = kSpJumpLog>
__device__ uint32_t spec_runs(const uint32_t* stw, uint32_t base, uint32_t len, uint32_t bw, uint32_t n,
                              uint16_t* tab, uint32_t* list, uint32_t* esum, uint32_t lcap, uint2* rec, uint32_t rcap,
                              uint32_t* sh) {
    constexpr uint32_t kJump = 1u << kJumpLog;
    const uint32_t tid = threadIdx.x, e = base + len, nbv = (bw + 7) / 8;
    // 1. speculative headers
    for (uint32_t j = tid; j < len; j += kThreads) {
        const SpecHdr h = spec_hdr(stw, base + j);
        const uint64_t nx = h.lit ? static_cast<uint64_t>(h.qh) + static_cast<uint64_t>(h.g) * bw : h.qh + nbv;
        tab[j] = static_cast<uint16_t>((spec_bad(h, e, nbv) || nx >= e) ? kSpStop : static_cast<uint32_t>(nx - base));
    }
    if (tid < 4) sh[tid] = 0;
    __syncthreads();
    // 2. kJump-run jumps.  kBlocked: thread t owns positions
    //    [t * kPerThread, (t + 1) * kPerThread) as 16-byte LDS vectors (tab
    //    16-byte aligned, kPerThread % 8 == 0), so a round holds kPerThread
    //    u16 jumps in kPerThread / 2 registers; else positions t + i * kThreads.
    if constexpr (kBlocked) {
        static_assert(kPerThread % 8 == 0, "blocked rounds load 8 jumps at once");
        constexpr int kV = kPerThread / 8;
        uint4* t4 = reinterpret_cast<uint4*>(tab);
        for (int r = 0; r < kJumpLog; r++) {
            uint4 nv[kV];
#pragma unroll
            for (int v = 0; v < kV; v++) {
                const uint32_t j = tid * kPerThread + static_cast<uint32_t>(v) * 8;
                uint4 c = j < len ? t4[j / 8] : make_uint4(~0u, ~0u, ~0u, ~0u);
                uint32_t w[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
                for (int h = 0; h < 4; h++) {
                    uint32_t lo = w[h] & 0xFFFFu, hi = w[h] >> 16;
                    if (lo != kSpStop) lo = tab[lo];
                    if (hi != kSpStop) hi = tab[hi];
                    w[h] = lo | (hi << 16);
                }
                nv[v] = make_uint4(w[0], w[1], w[2], w[3]);
            }
            __syncthreads();
#pragma unroll
            for (int v = 0; v < kV; v++) {
                const uint32_t j = tid * kPerThread + static_cast<uint32_t>(v) * 8;
                if (j < len) t4[j / 8] = nv[v];
            }
            __syncthreads();
        }
    } else {
        for (int r = 0; r < kJumpLog; r++) {
            uint32_t nv[(kPerThread + 1) / 2];  // two u16 jumps per register
#pragma unroll
            for (int i = 0; i < kPerThread; i++) {
                const uint32_t j = tid + static_cast<uint32_t>(i) * kThreads;
                uint32_t t = kSpStop;
                if (j < len) {
                    t = tab[j];
                    if (t != kSpStop) t = tab[t];
                }
                if (i & 1) nv[i >> 1] |= t << 16;
                else nv[i >> 1] = t;
            }
            __syncthreads();
#pragma unroll
            for (int i = 0; i < kPerThread; i++) {
                const uint32_t j = tid + static_cast<uint32_t>(i) * kThreads;
                if (j < len) tab[j] = static_cast<uint16_t>(nv[i >> 1] >> (16 * (i & 1)));
            }
            __syncthreads();
        }
    }
    // 3. every kJump-th header of the real chain
    const uint32_t lmax = rcap > kJump + 1 ? min(lcap, (rcap - kJump - 1) / kJump + 1) : 0u;
    if (tid == 0) {
        uint32_t k = 0, q = 0;
        for (;;) {
            if (k >= lmax) { k = ~0u; break; }
            list[k++] = q;
            if (q >= len) break;
            const uint32_t t = tab[q];
            if (t == kSpStop) break;
            q = t;
        }
        sh[0] = k;
    }
    __syncthreads();
    const uint32_t nl = sh[0];
    if (nl == ~0u) return ~0u;
    // 4. exact runs of each listed header: untruncated counts, first bad step
    const uint32_t vmask = nbv >= 3 ? 0xFFFFFFu : nbv == 2 ? 0xFFFFu : (nbv ? 0xFFu : 0u);  // RLE values of bw <= 24 exact
    const uint32_t litpay = bw ? 0x80000000u : 0u, litmul = bw ? 8u : 0u;
    for (uint32_t i = tid; i < nl; i += kThreads) {
        uint32_t q = base + list[i];
        uint2* out = rec + i * kJump;
        uint32_t s = 0, sum = 0, bad = kJump, ended = 0;
        for (; s < kJump; s++) {
            if (q >= e) { ended = 1; break; }
            const SpecHdr h = spec_hdr(stw, q);
            if (spec_bad(h, e, nbv)) { bad = s; break; }
            const uint32_t c = h.lit ? min(h.g, kSpCountCap / 8) * 8 : min(h.g, kSpCountCap);
            out[s] = make_uint2(c, h.lit ? (litpay | (h.qh * litmul)) : (h.vraw & vmask));
            sum = min(sum + c, kSpCountCap);
            const uint64_t nql = static_cast<uint64_t>(h.qh) + static_cast<uint64_t>(h.g) * bw;
            q = h.lit ? (nql > e ? e : static_cast<uint32_t>(nql)) : h.qh + nbv;
        }
        if (s == kJump && q >= e) ended = 1;
        esum[i] = sum;
        list[i] = s | (bad << 8) | (ended << 16);
    }
    __syncthreads();
    // 5. exclusive scan of the counts (wave 0), truncation, exhaustion
    if (tid < kWave) {
        const uint32_t per = (nl + kWave - 1) / kWave;
        const uint32_t a0 = min(nl, tid * per), a1 = min(nl, a0 + per);
        uint32_t sum = 0;
        for (uint32_t i = a0; i < a1; i++) sum += esum[i];
        uint32_t run = wave_incl_scan(sum) - sum;
        for (uint32_t i = a0; i < a1; i++) {
            const uint32_t x = esum[i];
            esum[i] = run;
            run += x;
        }
    }
    __syncthreads();
    for (uint32_t i = tid; i < nl; i += kThreads) {
        const uint32_t meta = list[i];
        const uint32_t nr = meta & 0xFFu, bad = (meta >> 8) & 0xFFu, ended = meta >> 16;
        const uint32_t b0 = esum[i];
        if (b0 >= n) continue;
        uint2* out = rec + i * kJump;
        uint32_t c0 = b0, kept = 0;
        for (uint32_t s = 0; s < nr && c0 < n; s++) {
            const uint32_t c = out[s].x;
            out[s].x = c0 | (min(c, n - c0) << 16);
            c0 += c;
            kept = s + 1;
        }
        if (c0 >= n) {
            sh[1] = i * kJump + kept;
        } else if (bad < kJump || (i + 1 == nl && (!ended || i * kJump + nr >= rcap))) {
            atomicOr(&sh[2], 1u);  // a bad header before the value count
        } else if (i + 1 == nl) {  // exhausted: the rest of the values are 0
            out[nr] = make_uint2(c0 | ((n - c0) << 16), 0u);
            sh[1] = i * kJump + nr + 1;
        }
    }
    __syncthreads();
    return (sh[2] || sh[1] == 0) ? ~0u : sh[1];
}


// Two streams of one page at once (k_wide_rows: the def levels and the
// dictionary indices): one table over both streams' positions (stream 0 at
// [0, len0), stream 1 at [len0, len0 + len1); a chain never leaves its stream
// because each stops at its own end), one set of doubling rounds and
// barriers, the two list walks on different waves at the same time, the
// exact re-parse and the scans of both in the same passes.  Records of stream
// s go to rec_s[0 .. rcap_s); list/esum hold lcap0 + lcap1 entries.  Returns
// both record counts in out[0], out[1] (~0u: that stream needs the serial
// path).  Blocked rounds as spec_runs<.., true, ..>; len0 + len1 <= kThreads
// * kPerThread < 65535.
template <int kThreads, int kPerThread, int kJumpLog = kSpJumpLog>
__device__ void spec_runs2(const uint32_t* stw, const uint32_t base_[2], const uint32_t len_[2], const uint32_t bw_[2],
                           const uint32_t n_[2], uint16_t* tab, uint32_t* list, uint32_t* esum, const uint32_t lcap_[2],
                           uint2* const rec_[2], const uint32_t rcap_[2], uint32_t* sh, uint32_t out[2]) {
    constexpr uint32_t kJump = 1u << kJumpLog;
    const uint32_t tid = threadIdx.x;
    const uint32_t L0 = len_[0], L = len_[0] + len_[1];
    // 1. speculative headers of both streams
    for (uint32_t j = tid; j < L; j += kThreads) {
        const uint32_t s = j < L0 ? 0u : 1u;
        const uint32_t off = s ? L0 : 0u, base = base_[s], bw = bw_[s], e = base + len_[s], nbv = (bw + 7) / 8;
        const SpecHdr h = spec_hdr(stw, base + (j - off));
        const uint64_t nx = h.lit ? static_cast<uint64_t>(h.qh) + static_cast<uint64_t>(h.g) * bw : h.qh + nbv;
        tab[j] = static_cast<uint16_t>((spec_bad(h, e, nbv) || nx >= e) ? kSpStop
                                                                        : off + static_cast<uint32_t>(nx - base));
    }
    if (tid < 8) sh[tid] = 0;
    __syncthreads();
    // 2. kJump-run jumps (blocked, as spec_runs)
    {
        static_assert(kPerThread % 8 == 0, "blocked rounds load 8 jumps at once");
        constexpr int kV = kPerThread / 8;
        uint4* t4 = reinterpret_cast<uint4*>(tab);
        for (int r = 0; r < kJumpLog; r++) {
            uint4 nv[kV];
#pragma unroll
            for (int v = 0; v < kV; v++) {
                const uint32_t j = tid * kPerThread + static_cast<uint32_t>(v) * 8;
                uint4 c = j < L ? t4[j / 8] : make_uint4(~0u, ~0u, ~0u, ~0u);
                uint32_t w[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
                for (int h = 0; h < 4; h++) {
                    uint32_t lo = w[h] & 0xFFFFu, hi = w[h] >> 16;
                    if (lo != kSpStop) lo = tab[lo];
                    if (hi != kSpStop) hi = tab[hi];
                    w[h] = lo | (hi << 16);
                }
                nv[v] = make_uint4(w[0], w[1], w[2], w[3]);
            }
            __syncthreads();
#pragma unroll
            for (int v = 0; v < kV; v++) {
                const uint32_t j = tid * kPerThread + static_cast<uint32_t>(v) * 8;
                if (j < L) t4[j / 8] = nv[v];
            }
            __syncthreads();
        }
    }
    // 3. every kJump-th header of each chain: stream 0 by thread 0, stream 1
    //    by thread kWave (another wave), concurrently; positions stream-local
    if (tid == 0 || tid == kWave) {
        const uint32_t s = tid == 0 ? 0u : 1u;
        const uint32_t off = s ? L0 : 0u, len = len_[s], rcap = rcap_[s];
        uint32_t* lst = list + (s ? lcap_[0] : 0u);
        const uint32_t lmax = rcap > kJump + 1 ? min(lcap_[s], (rcap - kJump - 1) / kJump + 1) : 0u;
        uint32_t k = 0, q = 0;
        for (;;) {
            if (k >= lmax) { k = ~0u; break; }
            lst[k++] = q;
            if (q >= len) break;
            const uint32_t t = tab[off + q];
            if (t == kSpStop) break;
            q = t - off;
        }
        sh[4 * s] = k;
    }
    __syncthreads();
    const uint32_t nl_[2] = {sh[0], sh[4]};
    const uint32_t nla = nl_[0] == ~0u ? 0u : nl_[0], nlb = nl_[1] == ~0u ? 0u : nl_[1];
    // 4. exact runs of each listed header (both streams)
    for (uint32_t g = tid; g < nla + nlb; g += kThreads) {
        const uint32_t s = g < nla ? 0u : 1u, i = s ? g - nla : g;
        const uint32_t base = base_[s], bw = bw_[s], e = base + len_[s], nbv = (bw + 7) / 8;
        const uint32_t vmask = nbv >= 3 ? 0xFFFFFFu : nbv == 2 ? 0xFFFFu : (nbv ? 0xFFu : 0u);
        const uint32_t litpay = bw ? 0x80000000u : 0u, litmul = bw ? 8u : 0u;
        uint32_t* lst = list + (s ? lcap_[0] : 0u);
        uint32_t* es = esum + (s ? lcap_[0] : 0u);
        uint32_t q = base + lst[i];
        uint2* o = rec_[s] + i * kJump;
        uint32_t st = 0, sum = 0, bad = kJump, ended = 0;
        for (; st < kJump; st++) {
            if (q >= e) { ended = 1; break; }
            const SpecHdr h = spec_hdr(stw, q);
            if (spec_bad(h, e, nbv)) { bad = st; break; }
            const uint32_t c = h.lit ? min(h.g, kSpCountCap / 8) * 8 : min(h.g, kSpCountCap);
            o[st] = make_uint2(c, h.lit ? (litpay | (h.qh * litmul)) : (h.vraw & vmask));
            sum = min(sum + c, kSpCountCap);
            const uint64_t nql = static_cast<uint64_t>(h.qh) + static_cast<uint64_t>(h.g) * bw;
            q = h.lit ? (nql > e ? e : static_cast<uint32_t>(nql)) : h.qh + nbv;
        }
        if (st == kJump && q >= e) ended = 1;
        es[i] = sum;
        lst[i] = st | (bad << 8) | (ended << 16);
    }
    __syncthreads();
    // 5. exclusive scans of the counts: stream 0 by wave 0, stream 1 by wave 1
    const uint32_t wv = tid / kWave;
    if (wv < 2) {
        const uint32_t s = wv, nl = s ? nlb : nla, ln = tid % kWave;
        uint32_t* es = esum + (s ? lcap_[0] : 0u);
        const uint32_t per = (nl + kWave - 1) / kWave;
        const uint32_t a0 = min(nl, ln * per), a1 = min(nl, a0 + per);
        uint32_t sum = 0;
        for (uint32_t i = a0; i < a1; i++) sum += es[i];
        uint32_t run = wave_incl_scan(sum) - sum;
        for (uint32_t i = a0; i < a1; i++) {
            const uint32_t x = es[i];
            es[i] = run;
            run += x;
        }
    }
    __syncthreads();
    for (uint32_t g = tid; g < nla + nlb; g += kThreads) {
        const uint32_t s = g < nla ? 0u : 1u, i = s ? g - nla : g, nl = s ? nlb : nla, n = n_[s];
        const uint32_t* lst = list + (s ? lcap_[0] : 0u);
        const uint32_t* es = esum + (s ? lcap_[0] : 0u);
        const uint32_t meta = lst[i];
        const uint32_t nr = meta & 0xFFu, bad = (meta >> 8) & 0xFFu, ended = meta >> 16;
        const uint32_t b0 = es[i];
        if (b0 >= n) continue;
        uint2* o = rec_[s] + i * kJump;
        uint32_t c0 = b0, kept = 0;
        for (uint32_t t = 0; t < nr && c0 < n; t++) {
            const uint32_t c = o[t].x;
            o[t].x = c0 | (min(c, n - c0) << 16);
            c0 += c;
            kept = t + 1;
        }
        if (c0 >= n) {
            sh[4 * s + 1] = i * kJump + kept;
        } else if (bad < kJump || (i + 1 == nl && (!ended || i * kJump + nr >= rcap_[s]))) {
            atomicOr(&sh[4 * s + 2], 1u);  // a bad header before the value count
        } else if (i + 1 == nl) {  // exhausted: the rest of the values are 0
            o[nr] = make_uint2(c0 | ((n - c0) << 16), 0u);
            sh[4 * s + 1] = i * kJump + nr + 1;
        }
    }
    __syncthreads();
    for (uint32_t s = 0; s < 2; s++)
        out[s] = (nl_[s] == ~0u || sh[4 * s + 2] || sh[4 * s + 1] == 0) ? ~0u : sh[4 * s + 1];
    __syncthreads();
}

}  // namespace dev
}  // namespace pqk
