// regex.hip — bit-parallel Glushkov NFA page filter on gfx950.
//
// k_regex_dict   one workgroup per dictionary page: every entry is matched
//                once (dictionary-first, SURVEY §8a R-REGEX), result bytes
//                in dict_match[].
// k_regex_pages  one wavefront per data page: decode levels (and indices) with
//                the same state machine as the decode kernels, then
//                dictionary pages test match bits of their indices, PLAIN
//                pages run the NFA, one string per lane, bytes from LDS.
// A page is REPORTED (flag 1) iff no non-null value satisfies the predicate
// (match, or non-match under --neg-regex); NULLs satisfy neither.
#include <cstring>

#include "kernels/device_common.hpp"
#include "kernels/kernels.hpp"
#include "pq_gpu.h"
#include "regex/regex.hpp"

namespace pqre {
namespace {

using pqk::ColumnParams;
using pqk::DevDict;
using pqk::DevErr;
using pqk::DevPage;
using pqk::kTileRows;
using pqk::kWave;
using namespace pqk::dev;

constexpr int kWavesPerBlock = 4;
constexpr uint32_t kStageWords = 1024;

// Stage the program into LDS (whole workgroup).
__device__ void load_prog(DevProg* dst, const DevProg* src) {
    const uint4* s = reinterpret_cast<const uint4*>(src);
    uint4* d = reinterpret_cast<uint4*>(dst);
    for (uint32_t i = threadIdx.x; i < sizeof(DevProg) / 16; i += blockDim.x) d[i] = s[i];
    __syncthreads();
}

// NFA over one string; byte(i) yields the i-th byte.
template <class B>
__device__ __forceinline__ bool nfa_match(const DevProg& P, uint32_t n, B&& byte) {
    if (n == 0) return P.empty_string != 0;
    if (P.nonempty_trivial) return true;
    uint64_t D = 0;
    for (uint32_t i = 0; i < n; i++) {
        uint64_t f = i == 0 ? P.first_at0 : P.first_mid;
        for (uint32_t k = 0; k < P.nchunks; k++) f |= P.ftab[k][(D >> (8 * k)) & 0xFF];
        D = f & P.cls[byte(i)];
        if (D & P.last) return true;
        if (D == 0 && P.first_mid == 0) return false;
    }
    return (D & P.accept_end) != 0;
}

__global__ void __launch_bounds__(256) k_regex_dict(const DevProg* __restrict__ prog,
                                                    const uint8_t* __restrict__ bytes,
                                                    const DevDict* __restrict__ dicts,
                                                    const uint64_t* __restrict__ entries,
                                                    const int32_t* __restrict__ dict_count,
                                                    uint8_t* __restrict__ dict_match) {
    __shared__ DevProg P;
    load_prog(&P, prog);
    const DevDict d = dicts[blockIdx.x];
    const int32_t n = dict_count[blockIdx.x];
    const uint8_t* base = bytes + d.off;
    for (int32_t k = threadIdx.x; k < n; k += blockDim.x) {
        uint64_t e = entries[d.entry_base + k];
        const uint8_t* s = base + static_cast<uint32_t>(e);
        uint32_t len = static_cast<uint32_t>(e >> 32);
        dict_match[d.entry_base + k] = nfa_match(P, len, [&](uint32_t i) { return static_cast<uint32_t>(s[i]); });
    }
}

struct PageLds {
    uint32_t stage[kStageWords];
    uint32_t lv[kTileRows];
    uint32_t a[kTileRows];
    uint32_t b[kTileRows];
};


__global__ void __launch_bounds__(256) k_regex_pages(const DevProg* __restrict__ prog,
                                                     const uint8_t* __restrict__ bytes,
                                                     const DevPage* __restrict__ pages, int npages,
                                                     const DevDict* __restrict__ dicts,
                                                     const uint64_t* __restrict__ entries,
                                                     const int32_t* __restrict__ dict_count,
                                                     const uint8_t* __restrict__ dict_match,
                                                     ColumnParams cp, int neg,
                                                     uint8_t* __restrict__ page_flags,
                                                     DevErr* __restrict__ page_err,
                                                     int32_t* __restrict__ err_any) {
    __shared__ DevProg P;
    __shared__ PageLds lds_all[kWavesPerBlock];
    load_prog(&P, prog);
    const int wv = threadIdx.x / kWave;
    const int p = blockIdx.x * kWavesPerBlock + wv;
    if (p >= npages) return;
    PageLds& L = lds_all[wv];
    const DevPage pg = pages[p];
    DevErr* err = page_err + p;
    const uint8_t* g = bytes + pg.off;
    const uint32_t size = static_cast<uint32_t>(pg.size);
    Src s{nullptr, g, size};
    if (size <= kStageWords * 4) {
        stage_page(L.stage, g, size);
        s.lds = L.stage;
    }
    const int32_t nv = pg.nvals;
    uint32_t pos = 0;
    Rle def;
    const bool has_def = cp.max_def > 0;
    if (has_def) {
        if (pos + 4 > size) { set_err(err, err_any, PQ_ERR_BUFFER, pos, 4, size); return; }
        uint32_t def_len = src_u32(s, pos);
        pos += 4;
        if (static_cast<uint64_t>(pos) + def_len > size) { set_err(err, err_any, PQ_ERR_BUFFER, pos, def_len, size); return; }
        rle_init(def, pos, def_len, level_bw(cp.max_def));
        pos += def_len;
    }
    if (cp.max_rep > 0) {
        if (pos + 4 > size) { set_err(err, err_any, PQ_ERR_BUFFER, pos, 4, size); return; }
        uint32_t rep_len = src_u32(s, pos);
        pos += 4;
        if (static_cast<uint64_t>(pos) + rep_len > size) { set_err(err, err_any, PQ_ERR_BUFFER, pos, rep_len, size); return; }
        pos += rep_len;
    }
    const bool dict = pg.mode == pqk::MODE_DICT;
    Rle ix;
    uint32_t dict_n = 0, entry_base = 0;
    if (dict) {
        if (pos + 1 > size) { set_err(err, err_any, PQ_ERR_BUFFER, pos, 1, size); return; }
        uint32_t bw = src_byte(s, pos);
        pos += 1;
        rle_init(ix, pos, size - pos, bw);
        dict_n = static_cast<uint32_t>(dict_count[pg.dict]);
        entry_base = static_cast<uint32_t>(dicts[pg.dict].entry_base);
    }
    bool any = false;
    for (int32_t r0 = 0; r0 < nv; r0 += kTileRows) {
        const uint32_t m = min(static_cast<uint32_t>(nv - r0), static_cast<uint32_t>(kTileRows));
        int rc = 0;
        if (has_def) rc = rle_decode(def, s, m, [&](uint32_t j, uint32_t v) { L.lv[j] = v & 0xFFFFu; });
        else for (uint32_t j = lane(); j < m; j += kWave) L.lv[j] = static_cast<uint32_t>(cp.max_def);
        __builtin_amdgcn_wave_barrier();
        uint32_t nn = 0, above = 0;
        for (uint32_t j0 = 0; j0 < m; j0 += kWave) {
            uint32_t j = j0 + lane();
            int32_t d = j < m ? static_cast<int16_t>(L.lv[j]) : -32768;
            bool isnn = dict ? d == cp.max_def : d >= cp.max_def;
            nn += __popcll(__ballot(isnn));
            above |= __ballot(d > cp.max_def) != 0;
        }
        if (rc == 0 && dict && above) rc = PQ_ERR_UNSUPPORTED;
        if (rc) { set_err(err, err_any, rc, 0, 0, size); return; }
        if (dict) {
            rc = rle_decode(ix, s, nn, [&](uint32_t j, uint32_t v) { L.a[j] = v; });
            if (rc) { set_err(err, err_any, rc, 0, 0, size); return; }
            __builtin_amdgcn_wave_barrier();
            for (uint32_t k0 = 0; k0 < nn; k0 += kWave) {
                uint32_t k = k0 + lane();
                bool sat = false;
                if (k < nn) {
                    uint32_t idx = L.a[k];
                    bool ok = static_cast<int32_t>(idx) >= 0 && idx < dict_n;
                    sat = ok && ((dict_match[entry_base + idx] != 0) != (neg != 0));
                }
                any |= __ballot(sat) != 0;
            }
        } else {
            int failed = 0;
            if (lane() == 0) {  // PLAIN BYTE_ARRAY chain (column_reader.cpp:249-253)
                for (uint32_t k = 0; k < nn; k++) {
                    if (static_cast<uint64_t>(pos) + 4 > size) { set_err(err, err_any, PQ_ERR_BUFFER, pos, 4, size); failed = 1; break; }
                    uint32_t len = src_u32(s, pos);
                    pos += 4;
                    if (static_cast<uint64_t>(pos) + len > size) { set_err(err, err_any, PQ_ERR_BUFFER, pos, len, size); failed = 1; break; }
                    L.a[k] = pos;
                    L.b[k] = len;
                    pos += len;
                }
            }
            failed = __shfl(failed, 0, kWave);
            pos = __shfl(pos, 0, kWave);
            if (failed) return;
            __builtin_amdgcn_wave_barrier();
            if (!any) {
                for (uint32_t k0 = 0; k0 < nn && !any; k0 += kWave) {
                    uint32_t k = k0 + lane();
                    bool sat = false;
                    if (k < nn) {
                        uint32_t st = L.a[k], len = L.b[k];
                        bool mt = nfa_match(P, len, [&](uint32_t i) { return src_byte(s, st + i); });
                        sat = mt != (neg != 0);
                    }
                    any |= __ballot(sat) != 0;
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
    if (lane() == 0) page_flags[p] = any ? 0 : 1;
}

}  // namespace

DeviceProgram* upload_program(const Program& p, hipStream_t s) {
    DevProg h;
    build_dev(p, &h);
    auto* dp = new DeviceProgram{nullptr};
    if (hipMalloc(reinterpret_cast<void**>(&dp->d), sizeof(DevProg)) != hipSuccess) {
        delete dp;
        return nullptr;
    }
    if (hipMemcpyAsync(dp->d, &h, sizeof h, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess) {
        (void)hipFree(dp->d);
        delete dp;
        return nullptr;
    }
    return dp;
}

void free_device_program(DeviceProgram* p) {
    if (!p) return;
    if (p->d) (void)hipFree(p->d);
    delete p;
}

void launch_regex_dict(hipStream_t s, const DeviceProgram* prog, const uint8_t* bytes,
                       const DevDict* dicts, int ndicts, const uint64_t* entries,
                       const int32_t* dict_count, uint8_t* dict_match) {
    if (ndicts <= 0) return;
    hipLaunchKernelGGL(k_regex_dict, dim3(ndicts), dim3(256), 0, s, prog->d, bytes, dicts, entries,
                       dict_count, dict_match);
}

void launch_regex_pages(hipStream_t s, const DeviceProgram* prog, const uint8_t* bytes,
                        const DevPage* pages, int npages, const DevDict* dicts,
                        const uint64_t* entries, const int32_t* dict_count,
                        const uint8_t* dict_match, ColumnParams cp, int neg, uint8_t* page_flags,
                        DevErr* page_err, int32_t* err_any) {
    if (npages <= 0) return;
    int blocks = (npages + kWavesPerBlock - 1) / kWavesPerBlock;
    hipLaunchKernelGGL(k_regex_pages, dim3(blocks), dim3(256), 0, s, prog->d, bytes, pages, npages,
                       dicts, entries, dict_count, dict_match, cp, neg, page_flags, page_err,
                       err_any);
}

}  // namespace pqre
