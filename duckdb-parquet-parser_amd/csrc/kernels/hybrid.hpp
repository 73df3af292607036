// hybrid.hpp — lane-parallel decode of one hybrid RLE/bit-packed stream
// (rle_decoder.hpp:6-108) held in LDS, for one wavefront.
//
// The run headers form a chain: header -> payload -> next header.  Walking it
// on the scalar unit costs ~100 SALU per run and the scalar unit is shared by
// every wave of a CU, so for run-dense streams (short RLE runs, 8-value
// bit-packed groups) the decode is bound by SALU issue.  Here every byte
// position of the stream is parsed as if a header started there (one lane per
// position), giving a successor function next(p).  The positions on the true
// chain — the set reachable from position 0 — come from pointer doubling:
//   S_0 = {0},  S_{k+1} = S_k ∪ J_k(S_k),  J_{k+1} = J_k ∘ J_k
// which needs ceil(log2(runs)) rounds of LDS gathers.  A prefix sum of the run
// lengths over chain positions (chain order = byte order) gives each run's
// first output slot; a max-scan of run ids scattered at those slots gives the
// run of every output, which is then expanded from the run's value (RLE) or
// from its bit-packed payload in the staged page.
//
// Streams with anything unusual on the chain before the last needed value —
// a zero-length run (the reference's literal_count_ wrap), a varint that
// runs past the stream or over five bytes, bw > 32, a header too wide for
// the 8-byte window — report "serial" and the caller runs the scalar walk
// (stream.hpp), which restates the reference state machine exactly.
#pragma once
#include "kernels/device_common.hpp"

namespace pqk {
namespace dev {

constexpr uint32_t kHybMaxPos = 1024;  // stream bytes decoded in parallel (else: serial walk)

// Per-wave LDS scratch for hyb_decode, sized for `maxpos` stream bytes and
// `maxruns` runs (see hyb_scratch_bytes).
struct HybScratch {
    uint16_t* nx0;    // maxpos + 1: successor (ping)
    uint16_t* nx1;    // maxpos + 1: successor (pong)
    uint16_t* cnt;    // maxpos: run length (saturated at 65535)
    uint32_t* aux;    // maxpos: RLE value, or payload byte offset in the page
    uint8_t* on;      // maxpos + 1: position is on the chain
    uint8_t* meta;    // maxpos: bit0 literal, bit1 serial-only
    uint16_t* rpos;   // maxruns: position of run r
    uint16_t* rstart; // maxruns: first output slot of run r
};

__host__ __device__ constexpr uint32_t hyb_align4(uint32_t x) { return (x + 3u) & ~3u; }

__host__ __device__ inline uint32_t hyb_scratch_bytes(uint32_t maxpos, uint32_t maxruns) {
    return 2 * hyb_align4(2 * (maxpos + 1)) + hyb_align4(2 * maxpos) + 4 * maxpos +
           hyb_align4(maxpos + 1) + hyb_align4(maxpos) + 2 * hyb_align4(2 * maxruns);
}

__device__ inline HybScratch hyb_carve(uint8_t* p, uint32_t maxpos, uint32_t maxruns) {
    HybScratch s;
    s.aux = reinterpret_cast<uint32_t*>(p); p += 4 * maxpos;
    s.nx0 = reinterpret_cast<uint16_t*>(p); p += hyb_align4(2 * (maxpos + 1));
    s.nx1 = reinterpret_cast<uint16_t*>(p); p += hyb_align4(2 * (maxpos + 1));
    s.cnt = reinterpret_cast<uint16_t*>(p); p += hyb_align4(2 * maxpos);
    s.rpos = reinterpret_cast<uint16_t*>(p); p += hyb_align4(2 * maxruns);
    s.rstart = reinterpret_cast<uint16_t*>(p); p += hyb_align4(2 * maxruns);
    s.on = p; p += hyb_align4(maxpos + 1);
    s.meta = p;
    return s;
}

// Decode the first n values of the stream at page bytes [base, base + S)
// (page words `pw`, page size `psize`) with bit width bw.  out(j, v) for
// j < n.  R: n u16 slots of LDS scratch (may alias the output array when
// out writes slot j only after reading R[j] in the same lane).  Returns 0,
// or 1 if the stream needs the serial walk (nothing was written then).
struct NoMark {
    __device__ void operator()(int) const {}
};

// mark(phase) is called after each of the phases A..D (0..3), for profiling.
template <class Out, class Mark = NoMark>
__device__ int hyb_decode(const uint32_t* pw, uint32_t psize, uint32_t base, uint32_t S, uint32_t bw,
                          uint32_t n, const HybScratch& sc, uint32_t maxruns, uint16_t* R, Out&& out,
                          Mark&& mark = Mark()) {
    constexpr uint32_t U = 4;  // positions / outputs per lane per batch (loads issued together)
    if (n == 0) return 0;
    if (S > kHybMaxPos || bw > 32) return 1;
    const uint32_t nb = (bw + 7) / 8;
    // A. parse a header at every position
    for (uint32_t p0 = 0; p0 < S; p0 += U * kWave) {
        uint64_t xs[U];
#pragma unroll
        for (uint32_t u = 0; u < U; u++) {
            const uint32_t p = p0 + u * kWave + lane();
            xs[u] = p < S ? lds_u64(pw, base + p) : 0ull;
        }
#pragma unroll
        for (uint32_t u = 0; u < U; u++) {
            const uint32_t p = p0 + u * kWave + lane();
            if (p >= S) continue;
            const uint32_t rem = S - p;
            uint64_t x = xs[u];
            if (rem < 8) x &= (1ull << (8 * rem)) - 1ull;
            const uint32_t vb = min(rem, 5u);  // varint bytes available
            const uint64_t stops = ~x & 0x8080808080ull & ((1ull << (8 * vb)) - 1ull);
            uint32_t meta = 0, next = S, count = 0, aux = 0;
            if (stops == 0) {
                meta = 2;
            } else {
                const uint32_t hl = (static_cast<uint32_t>(__builtin_ctzll(stops)) >> 3) + 1;
                uint64_t v = (x & 0x7full) | ((x >> 1) & 0x3f80ull) | ((x >> 2) & 0x1fc000ull) |
                             ((x >> 3) & 0xfe00000ull) | ((x >> 4) & 0x7f0000000ull);
                v &= (1ull << (7 * hl)) - 1ull;
                const uint32_t ind = static_cast<uint32_t>(v);
                if (ind & 1u) {
                    count = (ind >> 1) * 8u;
                    const uint64_t end = static_cast<uint64_t>(p) + hl + (static_cast<uint64_t>(count) * bw + 7) / 8;
                    next = end >= S ? S : static_cast<uint32_t>(end);
                    aux = base + p + hl;
                    meta = 1;
                } else {
                    count = ind >> 1;
                    const uint32_t take = min(nb, rem - hl);
                    if (hl + take > 8) meta = 2;
                    aux = take ? static_cast<uint32_t>((x >> (8 * hl)) &
                                                       ((take >= 4) ? 0xFFFFFFFFull : ((1ull << (8 * take)) - 1ull)))
                               : 0u;
                    next = min(S, p + hl + take);
                }
                if (count == 0) meta = 2;
            }
            sc.nx0[p] = static_cast<uint16_t>(next);
            sc.cnt[p] = static_cast<uint16_t>(min(count, 65535u));
            sc.aux[p] = aux;
            sc.meta[p] = static_cast<uint8_t>(meta);
            sc.on[p] = p == 0;
        }
    }
    if (lane() == 0) { sc.nx0[S] = static_cast<uint16_t>(S); sc.nx1[S] = static_cast<uint16_t>(S); sc.on[S] = 0; }
    __builtin_amdgcn_wave_barrier();
    mark(0);
    // B. chain membership by pointer doubling: on |= J(on), J = J o J
    uint16_t* J = sc.nx0;
    uint16_t* K = sc.nx1;
    // J[0] of the round is read by lane 0 in the round's first batch, so the
    // termination test costs no extra LDS round trip
    for (;;) {
        uint32_t j0 = S;
        for (uint32_t p0 = 0; p0 < S; p0 += U * kWave) {
            uint32_t jp[U], o[U], jj[U];
#pragma unroll
            for (uint32_t u = 0; u < U; u++) {
                const uint32_t p = p0 + u * kWave + lane();
                jp[u] = p < S ? J[p] : S;
                o[u] = p < S ? sc.on[p] : 0u;
            }
            if (p0 == 0) {
                j0 = __builtin_amdgcn_readfirstlane(jp[0]);
                if (j0 >= S) break;  // chain fully marked: nothing written this round
            }
#pragma unroll
            for (uint32_t u = 0; u < U; u++) jj[u] = J[jp[u]];
#pragma unroll
            for (uint32_t u = 0; u < U; u++) {
                const uint32_t p = p0 + u * kWave + lane();
                if (p < S) K[p] = static_cast<uint16_t>(jj[u]);
                if (o[u]) sc.on[jp[u]] = 1;
            }
        }
        if (j0 >= S) break;
        __builtin_amdgcn_wave_barrier();
        uint16_t* t = J; J = K; K = t;
    }
    __builtin_amdgcn_wave_barrier();
    mark(1);
    // C. run starts (prefix of lengths in byte order), run list, serial check
    for (uint32_t j = lane(); j < n; j += kWave) R[j] = 0;
    __builtin_amdgcn_wave_barrier();
    bool serial = false;
    uint32_t csum = 0, rsum = 0;
    for (uint32_t p0 = 0; p0 < S && csum < n; p0 += U * kWave) {
        uint32_t o[U], c[U], m[U];
#pragma unroll
        for (uint32_t u = 0; u < U; u++) {
            const uint32_t p = p0 + u * kWave + lane();
            o[u] = p < S ? sc.on[p] : 0u;
            c[u] = p < S ? sc.cnt[p] : 0u;
            m[u] = p < S ? sc.meta[p] : 0u;
        }
#pragma unroll
        for (uint32_t u = 0; u < U; u++) {
            const uint32_t p = p0 + u * kWave + lane();
            const bool on = o[u] != 0;
            const uint32_t cc = on ? c[u] : 0u;
            const uint32_t ci = wave_incl_scan(cc);
            const uint64_t om = __ballot(on);
            const uint32_t st = csum + ci - cc;
            const uint32_t ri = rsum + popc_below(om);
            if (on && st < n) {
                serial |= (m[u] & 2u) != 0;
                if (ri < maxruns) {
                    sc.rpos[ri] = static_cast<uint16_t>(p);
                    sc.rstart[ri] = static_cast<uint16_t>(st);
                    R[st] = static_cast<uint16_t>(ri);
                } else {
                    serial = true;
                }
            }
            csum += bcast_last(ci);
            rsum += __popcll(om);
        }
    }
    if (__ballot(serial)) return 1;
    __builtin_amdgcn_wave_barrier();
    mark(2);
    // D. run of every output (max-scan) and expansion
    const uint32_t total = csum;
    uint32_t carry = 0;
    for (uint32_t j0 = 0; j0 < n; j0 += U * kWave) {
        uint32_t r[U], rp[U], rs[U], av[U], me[U];
#pragma unroll
        for (uint32_t u = 0; u < U; u++) {
            const uint32_t j = j0 + u * kWave + lane();
            r[u] = j < n ? R[j] : 0u;
        }
#pragma unroll
        for (uint32_t u = 0; u < U; u++) {
            r[u] = max(wave_incl_max(r[u]), carry);
            carry = bcast_last(r[u]);
        }
#pragma unroll
        for (uint32_t u = 0; u < U; u++) {
            rp[u] = sc.rpos[r[u]];
            rs[u] = sc.rstart[r[u]];
        }
#pragma unroll
        for (uint32_t u = 0; u < U; u++) {
            av[u] = sc.aux[rp[u]];
            me[u] = sc.meta[rp[u]];
        }
#pragma unroll
        for (uint32_t u = 0; u < U; u++) {
            const uint32_t j = j0 + u * kWave + lane();
            // literal: bits of value (j - start); RLE: the run value
            const uint64_t bit = static_cast<uint64_t>(av[u]) * 8u + static_cast<uint64_t>(j - rs[u]) * bw;
            const uint32_t lit = (me[u] & 1u) && bw && j < total ? lds_bits(pw, psize, bit, bw) : 0u;
            if (j < n) out(j, j >= total ? 0u : ((me[u] & 1u) ? lit : av[u]));
        }
    }
    __builtin_amdgcn_wave_barrier();
    mark(3);
    return 0;
}

}  // namespace dev
}  // namespace pqk
