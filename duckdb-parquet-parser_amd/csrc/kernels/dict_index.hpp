// dict_index.hpp — dictionary page -> entry table (SURVEY §8a R-DICT-PAGE,
// column_reader.cpp:98-118): one workgroup of W waves per dictionary page,
// the page staged in LDS.  Shared by k_dict_index (dict_fused.hip) and the
// dictionary workgroups of k_pipe_runs (dict_pipe.hip).
#pragma once
#include "kernels/device_common.hpp"
#include "kernels/kernels.hpp"
#include "kernels/stream.hpp"

namespace pqk {
namespace dev {

// ── dictionary entry table ─────────────────────────────────────────────────
constexpr uint32_t kBad = 0xFFFFFFFFu;

// Unaligned dword at LDS byte address a.
__device__ __forceinline__ uint32_t lds_u32(const uint32_t* words, uint32_t a) {
    uint32_t w0 = words[a >> 2], w1 = words[(a >> 2) + 1];
    return __builtin_amdgcn_alignbyte(w1, w0, a & 3);
}
__device__ __forceinline__ uint32_t lds_u8(const uint32_t* words, uint32_t a) {
    return (words[a >> 2] >> (8 * (a & 3))) & 0xFFu;
}

__device__ __forceinline__ uint64_t entry_code(uint32_t len, uint32_t pos) {
    return (static_cast<uint64_t>(len) << 32) | pos;
}

// Fine slices (the common case: entries of <= 60 bytes).  The page in LDS is
// cut into kDSlice-byte slices; each wave takes 16 slices at a time, lane l
// testing whether offset l of each can start an entry (its u32 and bytes fit
// in the page; slice 0: offset 0 only) and the first kPCandD candidates per
// slice walking the chain to the slice end (chains of ~16 entries instead of
// the 1/16 page slices below).  The link is speculative and parallel, one
// thread per slice: slice s is entered where slice s - 1's first continuing
// candidate (no bounds error, exit in slice s's first 64 bytes) left, and
// every slice must hold a candidate at that entry whose exit is the one it
// advertised.  Any slice failing that, a chosen chain with a bounds error, or
// a chain ending before the declared count falls back to the coarse slices
// (which produce the reference's exact error).  Returns true when done.
constexpr uint32_t kDSlice = 256;
constexpr uint32_t kDSliceMax = 128 * 1024 / kDSlice;  // pages up to the LDS cap
constexpr uint32_t kPCandD = kPCandDHost;
constexpr uint32_t kDNone = 0xFFFFFFFFu;
// candidate record: exit (18 bits) | count << 18 (7 bits) | entry << 25 (6 bits) | error << 31
__device__ __forceinline__ uint32_t dc_exit(uint32_t r) { return r & 0x3FFFFu; }
__device__ __forceinline__ uint32_t dc_cnt(uint32_t r) { return (r >> 18) & 0x7Fu; }
__device__ __forceinline__ uint32_t dc_ent(uint32_t r) { return (r >> 25) & 0x3Fu; }

template <int W>
__device__ bool dict_index_fine(const uint32_t* words, uint32_t size, uint32_t n, uint64_t* out, DevErr* err,
                                int32_t* err_any, int32_t* count) {
    __shared__ uint32_t cand[kDSliceMax * kPCandD];
    __shared__ uint32_t cx[kDSliceMax];
    __shared__ uint32_t wsum[W];
    __shared__ int all_ok;
    const uint32_t nsl = (size + kDSlice - 1) / kDSlice;
    // one linking thread per slice
    if (n == 0 || size == 0 || nsl > kDSliceMax || nsl > W * kWave || size >= (1u << 18)) return false;
    const uint32_t w = threadIdx.x / kWave, l = lane();
    // candidates and their chains
    const uint32_t jm = l / kPCandD, sl = l % kPCandD;
    for (uint32_t g = w * 16; g < nsl; g += W * 16) {
        uint64_t mk = 0;
#pragma unroll
        for (uint32_t j = 0; j < 16; j++) {
            const uint32_t sc = g + j, cs = sc * kDSlice;
            const uint32_t q = cs + l, ce = min(cs + kDSlice, size);
            bool plaus = sc < nsl && q < ce && q + 4 <= size &&
                         static_cast<uint64_t>(q) + 4 + lds_u32(words, min(q, size)) <= size;
            if (sc == 0) plaus = l == 0;
            const uint64_t m = __ballot(plaus);
            if (j == jm) mk = m;
        }
        const uint32_t sc = g + jm;
        for (uint32_t i = 0; i < sl; i++) mk &= mk - 1;
        uint32_t rec = kDNone;
        if (sc < nsl && mk) {
            const uint32_t cs = sc * kDSlice, ce = min(cs + kDSlice, size);
            const uint32_t e = static_cast<uint32_t>(__builtin_ctzll(mk));
            uint32_t q = cs + e, cnt = 0, bad = 0;
            while (q < ce) {
                if (q + 4 > size) { bad = 1; break; }
                const uint32_t len = lds_u32(words, q);
                if (static_cast<uint64_t>(q) + 4 + len > size) { bad = 1; break; }
                q += 4 + len;
                cnt++;
            }
            rec = q | (cnt << 18) | (e << 25) | (bad << 31);
        }
        if (sc < nsl) cand[sc * kPCandD + sl] = rec;
    }
    if (threadIdx.x == 0) all_ok = 1;
    __syncthreads();
    // speculative link, one thread per slice
    const uint32_t t = threadIdx.x;
    uint32_t r[kPCandD];
    uint32_t cexit = kDNone;
    if (t < nsl) {
#pragma unroll
        for (uint32_t k = 0; k < kPCandD; k++) r[k] = cand[t * kPCandD + k];
        const uint32_t se = (t + 1) * kDSlice;
#pragma unroll
        for (int k = static_cast<int>(kPCandD) - 1; k >= 0; k--)
            if (r[k] != kDNone && !(r[k] >> 31) && dc_exit(r[k]) >= se && dc_exit(r[k]) < se + 64) cexit = dc_exit(r[k]);
        cx[t] = cexit;
    }
    __syncthreads();
    uint32_t pr = kDNone, cnt = 0, ent = 0;
    if (t < nsl) {
        const uint32_t e = t == 0 ? 0u : cx[t - 1];
#pragma unroll
        for (uint32_t k = 0; k < kPCandD; k++)
            if (r[k] != kDNone && t * kDSlice + dc_ent(r[k]) == e) pr = r[k];
        const bool lastc = t + 1 == nsl;
        const bool ok = pr != kDNone && (lastc || (!(pr >> 31) && dc_exit(pr) == cexit));
        if (!ok) all_ok = 0;
        cnt = ok ? dc_cnt(pr) : 0u;
        ent = e;
    }
    // entries before each slice: block scan of the chosen counts
    const uint32_t inc = wave_incl_scan(cnt);
    if (l == kWave - 1) wsum[w] = inc;
    __syncthreads();
    if (!all_ok) return false;
    uint32_t before = inc - cnt;
    uint32_t total = 0;
    for (uint32_t v = 0; v < W; v++) {
        if (v < w) before += wsum[v];
        total += wsum[v];
    }
    // the last chain: a bounds error before the count needs the exact error
    // (coarse path); reaching the page end short of the count is the
    // reference's read at the page end
    __shared__ uint32_t last_rec;
    if (t + 1 == nsl) last_rec = pr;
    __syncthreads();
    if (total < n && (last_rec >> 31)) return false;
    if (t < nsl && before < n) {
        const uint32_t m = min(cnt, n - before);
        uint32_t q = ent;
        for (uint32_t k = 0; k < m; k++) {
            const uint32_t len = lds_u32(words, q);
            out[before + k] = entry_code(len, q + 4);
            q += 4 + len;
        }
    }
    if (threadIdx.x == 0) {
        if (total < n) set_err(err, err_any, PQ_ERR_BUFFER, size, 4, size);
        *count = static_cast<int32_t>(min(total, n));
    }
    return true;
}

// One dictionary page per workgroup of W waves (di: its index), the page in
// `words` (LDS, lds_cap bytes).  k_dict_index (W = 16) and k_pipe_runs'
// leading workgroups (W = 4) run it.
template <int W>
__device__ void dict_index_block(const uint8_t* __restrict__ bytes, const DevDict* __restrict__ dicts, int di,
                                 uint64_t* __restrict__ entries, int32_t* __restrict__ dict_count,
                                 DevErr* __restrict__ dict_err, int32_t* __restrict__ err_any, uint32_t lds_cap,
                                 uint32_t* words) {
    __shared__ uint32_t ex[W * kWave];  // chain exit per candidate (kBad: overran the page)
    __shared__ uint32_t ec[W * kWave];  // entries walked per candidate
    __shared__ int32_t seg_lane[W];
    __shared__ uint32_t seg_base[W], seg_n[W];

    const DevDict d = dicts[di];
    const uint32_t size = static_cast<uint32_t>(max(d.size, 0));
    const uint32_t n = static_cast<uint32_t>(max(d.nvals, 0));
    DevErr* err = dict_err + di;
    uint64_t* out = entries + d.entry_base;
    const uint8_t* page = bytes + d.off;

    if (size + 32 > lds_cap) {
        // too large for LDS: k_dict_index leaves it to launch_dict_big; other
        // callers (never given such pages) walk it serially with wave 0
        if (lds_cap == kDictLdsCap || threadIdx.x >= kWave) return;
        uint32_t pos = 0, k = 0;
        for (; k < n; k++) {
            if (static_cast<uint64_t>(pos) + 4 > size) { set_err(err, err_any, PQ_ERR_BUFFER, pos, 4, size); break; }
            uint32_t len = suni(sload_u32(page, pos));
            pos += 4;
            if (static_cast<uint64_t>(pos) + len > size) { set_err(err, err_any, PQ_ERR_BUFFER, pos, len, size); break; }
            if (lane() == 0) out[k] = entry_code(len, pos);
            pos += len;
        }
        if (lane() == 0) dict_count[di] = static_cast<int32_t>(k);
        return;
    }
    {  // payload (+ one block of the image's zero padding) -> LDS
        const uint4* src = reinterpret_cast<const uint4*>(page);
        uint4* dst = reinterpret_cast<uint4*>(words);
        const uint32_t n16 = (size + 15) / 16 + 1;
        copy_blocks(dst, src, n16, threadIdx.x, blockDim.x);
    }
    __syncthreads();
    if (dict_index_fine<W>(words, size, n, out, err, err_any, dict_count + di)) return;
    const uint32_t w = threadIdx.x / kWave, l = lane();
    const uint32_t S = (size + W - 1) / W;
    const uint32_t s0 = min(size, w * S), s1 = min(size, s0 + S);
    {
        uint32_t p = s0 + l, cnt = 0;
        bool bad = p >= s1;
        while (!bad && p < s1) {
            if (p + 4 > size) { bad = true; break; }
            uint32_t len = lds_u32(words, p);
            if (static_cast<uint64_t>(p) + 4 + len > size) { bad = true; break; }
            p += 4 + len;
            cnt++;
        }
        ex[threadIdx.x] = bad ? kBad : p;
        ec[threadIdx.x] = cnt;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0, run = 0;
        bool stop = n == 0;
        for (uint32_t v = 0; v < W; v++) {
            seg_lane[v] = -1;
            seg_base[v] = run;
            seg_n[v] = 0;
            const uint32_t a0 = min(size, v * S), a1 = min(size, a0 + S);
            if (stop || t >= a1) continue;
            const uint32_t c = t - a0;
            if (c < kWave && ex[v * kWave + c] != kBad) {
                uint32_t m = min(ec[v * kWave + c], n - run);
                seg_lane[v] = static_cast<int32_t>(c);
                seg_n[v] = m;
                run += m;
                t = ex[v * kWave + c];
                if (run == n) stop = true;
                continue;
            }
            while (t < a1 && run < n) {  // uncovered entry point: serial walk
                if (t + 4 > size) { set_err(err, err_any, PQ_ERR_BUFFER, t, 4, size); stop = true; break; }
                uint32_t len = lds_u32(words, t);
                if (static_cast<uint64_t>(t) + 4 + len > size) {
                    set_err(err, err_any, PQ_ERR_BUFFER, t + 4, len, size);
                    stop = true;
                    break;
                }
                out[run++] = entry_code(len, t + 4);
                t += 4 + len;
            }
            if (run == n) stop = true;
        }
        // chain reached the page end with entries still declared (t == size)
        if (!stop && run < n) set_err(err, err_any, PQ_ERR_BUFFER, t, 4, size);
        dict_count[di] = static_cast<int32_t>(run);
    }
    __syncthreads();
    if (seg_lane[w] == static_cast<int32_t>(l)) {
        uint32_t p = s0 + l;
        uint64_t* o = out + seg_base[w];
        for (uint32_t k = 0; k < seg_n[w]; k++) {
            uint32_t len = lds_u32(words, p);
            o[k] = entry_code(len, p + 4);
            p += 4 + len;
        }
    }
}

}  // namespace dev
}  // namespace pqk
