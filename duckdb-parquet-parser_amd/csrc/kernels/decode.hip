// decode.hip — gfx950 kernels for ColumnReader::read_all's value decode.
//
// Reference behaviour restated here (file:line in the reference):
//   hybrid RLE/bit-packed decode   include/reader/rle_decoder.hpp:17-95
//   def/rep level sections         src/reader/column_reader.cpp:146-170
//   dictionary expansion           src/reader/column_reader.cpp:174-196
//   BOOLEAN bit unpack             src/reader/column_reader.cpp:197-212
//   PLAIN values                   src/reader/column_reader.cpp:213-268
//   dictionary page                src/reader/column_reader.cpp:128-138
//
// Work decomposition: one wavefront per page (or per dictionary
// page) for the serial stream parts, page bytes staged in LDS; the hybrid
// stream's run headers are walked wave-uniformly and each run is expanded
// 64 values per step across the lanes.  BYTE_ARRAY output is produced in two
// kernels: k_ba_rows resolves every row to (source offset, length) and sums
// per-tile bytes, a scan turns tile sums into output offsets, and
// k_ba_gather writes offsets, validity and characters with 16-byte aligned,
// coalesced stores.
#include "kernels.hpp"

#include "kernels/device_common.hpp"
#include "kernels/lane_walk.hpp"
#include "kernels/row_copy.hpp"
#include "kernels/run_spec.hpp"
#include "pq_gpu.h"

#include <algorithm>

namespace pqk {
namespace {

using namespace dev;

constexpr int kWavesPerBlock = 4;
constexpr uint32_t kStageWords = 1024;  // 4 KiB of page bytes staged per wave

// Page prologue shared by every data-page kernel: def-level stream, rep skip.
struct PagePrologue {
    uint32_t pos;       // ByteBuffer position after the level sections
    Rle def;
    int has_def;
};

__device__ int page_prologue(const Src& s, const ColumnParams& cp, PagePrologue& pp, DevErr* err,
                             int32_t* any) {
    uint32_t pos = 0;
    pp.has_def = cp.max_def > 0;
    if (pp.has_def) {  // 146-154
        if (pos + 4 > s.size) { set_err(err, any, PQ_ERR_BUFFER, pos, 4, s.size); return 1; }
        uint32_t def_len = src_u32(s, pos);
        pos += 4;
        if (static_cast<uint64_t>(pos) + def_len > s.size) {
            set_err(err, any, PQ_ERR_BUFFER, pos, def_len, s.size);
            return 1;
        }
        rle_init(pp.def, pos, def_len, level_bw(cp.max_def));
        pos += def_len;
    }
    if (cp.max_rep > 0) {  // 156-164: decoded then unused by flat output
        if (pos + 4 > s.size) { set_err(err, any, PQ_ERR_BUFFER, pos, 4, s.size); return 1; }
        uint32_t rep_len = src_u32(s, pos);
        pos += 4;
        if (static_cast<uint64_t>(pos) + rep_len > s.size) {
            set_err(err, any, PQ_ERR_BUFFER, pos, rep_len, s.size);
            return 1;
        }
        pos += rep_len;
    }
    pp.pos = pos;
    return 0;
}

// ── dictionary pages (column_reader.cpp:128-138) ───────────────────────────
// BYTE_ARRAY entries are a serial u32-length chain: one wave per dictionary
// page walks it in LDS; entries[] = (len << 32) | chars offset in the page.
__global__ void __launch_bounds__(64) k_dict_entries(const uint8_t* __restrict__ bytes,
                                                     const DevDict* __restrict__ dicts,
                                                     uint64_t* __restrict__ entries,
                                                     int32_t* __restrict__ dict_count,
                                                     DevErr* __restrict__ dict_err,
                                                     int32_t* __restrict__ err_any, int32_t type,
                                                     int32_t plain_width) {
    __shared__ uint32_t stage[8192];  // 32 KiB
    const DevDict d = dicts[blockIdx.x];
    const uint8_t* g = bytes + d.off;
    uint32_t size = static_cast<uint32_t>(d.size);
    DevErr* err = dict_err + blockIdx.x;
    if (type != PQ_BYTE_ARRAY) {
        // fixed width: entry k at k * plain_width; no walk needed
        int32_t n = d.nvals;
        if (n > 0 && type == PQ_FIXED_LEN_BYTE_ARRAY) {
            set_err(err, err_any, PQ_ERR_FLBA, 0, 0, size);
            if (lane() == 0) dict_count[blockIdx.x] = 0;
            return;
        }
        if (n > 0 && plain_width <= 0) {
            set_err(err, err_any, PQ_ERR_TYPE, 0, 0, size);
            if (lane() == 0) dict_count[blockIdx.x] = 0;
            return;
        }
        int32_t fit = plain_width > 0 ? static_cast<int32_t>(size / plain_width) : 0;
        if (n > fit) {
            set_err(err, err_any, PQ_ERR_BUFFER, fit * plain_width, plain_width, size);
            n = fit;
        }
        if (lane() == 0) dict_count[blockIdx.x] = n < 0 ? 0 : n;
        return;
    }
    Src s{nullptr, g, size};
    if (size <= sizeof(stage)) {
        stage_page(stage, g, size);
        s.lds = stage;
    }
    if (lane() == 0) {
        uint32_t pos = 0;
        int32_t k = 0;
        for (; k < d.nvals; k++) {
            if (pos + 4 > size) { set_err(err, err_any, PQ_ERR_BUFFER, pos, 4, size); break; }
            uint32_t len = src_u32(s, pos);
            pos += 4;
            if (static_cast<uint64_t>(pos) + len > size) {
                set_err(err, err_any, PQ_ERR_BUFFER, pos, len, size);
                break;
            }
            entries[d.entry_base + k] = (static_cast<uint64_t>(len) << 32) | pos;
            pos += len;
        }
        dict_count[blockIdx.x] = k;
    }
}

// ── BYTE_ARRAY rows: every row -> (len << 32 | source offset) or NULL ──────
template <uint32_t kSW>
struct RowsLds {
    uint32_t stage[kSW];
    uint32_t lv[kTileRows];   // def levels of the current tile
    uint32_t a[kTileRows];    // dict index / plain chars offset per non-null rank
    uint32_t b[kTileRows];    // plain length per non-null rank
};

// REQUIRED PLAIN pages above big_plain_min: k_plain_big_rows (plain_ba.hip)
__device__ __forceinline__ bool big_plain_page(const DevPage& pg, const ColumnParams& cp, uint32_t big_plain_min) {
    return big_plain_min && cp.max_def == 0 && cp.max_rep == 0 && pg.mode == MODE_PLAIN &&
           static_cast<uint32_t>(pg.size) > big_plain_min && pg.nvals <= 256 * kTileRows;
}

// One page by one wavefront, the reference state machine in order (def
// levels, then indices or the PLAIN length chain, tile by tile).  `staged`:
// the page's payload words already in LDS, or nullptr (read from HBM);
// lv / a / b: kTileRows words each of this wave's LDS scratch.
__device__ void ba_rows_page(const uint8_t* __restrict__ bytes, const DevPage& pg, int p, const uint32_t* staged,
                             uint32_t* lv_s, uint32_t* a_s, uint32_t* b_s, const DevDict* __restrict__ dicts,
                             const uint64_t* __restrict__ entries, const int32_t* __restrict__ dict_count,
                             ColumnParams cp, uint64_t* __restrict__ row_codes, int64_t* __restrict__ tile_chars,
                             const int32_t* __restrict__ page_tile0, DevErr* __restrict__ page_err,
                             int32_t* __restrict__ err_any) {
    struct {
        uint32_t* lv;
        uint32_t* a;
        uint32_t* b;
    } L{lv_s, a_s, b_s};
    DevErr* err = page_err + p;
    const uint32_t size = static_cast<uint32_t>(pg.size);
    Src s{staged, bytes + pg.off, size};
    const int32_t tile0 = page_tile0[p];
    const int32_t nv = pg.nvals;

    PagePrologue pp;
    if (page_prologue(s, cp, pp, err, err_any)) {
        for (int32_t t = 0; t * kTileRows < nv; t++)
            if (lane() == 0) tile_chars[tile0 + t] = 0;
        return;
    }
    uint32_t pos = pp.pos;
    const bool dict = pg.mode == MODE_DICT;
    Rle ix;
    uint32_t dict_n = 0;
    uint32_t entry_base = 0;
    if (dict) {  // 179-182: one bit-width byte, then the rest of the page
        if (pos + 1 > size) {
            set_err(err, err_any, PQ_ERR_BUFFER, pos, 1, size);
            for (int32_t t = 0; t * kTileRows < nv; t++)
                if (lane() == 0) tile_chars[tile0 + t] = 0;
            return;
        }
        uint32_t bw = src_byte(s, pos);
        pos += 1;
        rle_init(ix, pos, size - pos, bw);
        dict_n = static_cast<uint32_t>(dict_count[pg.dict]);
        entry_base = static_cast<uint32_t>(dicts[pg.dict].entry_base);
    }
    int failed = 0;
    for (int32_t r0 = 0, t = 0; r0 < nv; r0 += kTileRows, t++) {
        const uint32_t m = min(static_cast<uint32_t>(nv - r0), static_cast<uint32_t>(kTileRows));
        uint32_t* lv = L.lv;
        int rc = 0;
        if (pp.has_def) {
            rc = rle_decode(pp.def, s, m, [&](uint32_t j, uint32_t v) { lv[j] = v & 0xFFFFu; });
        } else {
            for (uint32_t j = lane(); j < m; j += kWave) lv[j] = static_cast<uint32_t>(cp.max_def);
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        // non-null count of this tile (def as int16, column_reader.cpp:166-170)
        uint32_t nn = 0, above = 0;
        for (uint32_t j0 = 0; j0 < m; j0 += kWave) {
            uint32_t j = j0 + lane();
            int32_t d = j < m ? static_cast<int16_t>(lv[j]) : -32768;
            bool isnn = dict ? d == cp.max_def : d >= cp.max_def;
            nn += __popcll(__ballot(isnn));
            above |= __ballot(d > cp.max_def) != 0;
        }
        if (rc == 0 && dict && above) rc = PQ_ERR_UNSUPPORTED;
        if (rc) { set_err(err, err_any, rc, 0, 0, size); failed = 1; }
        if (!failed && dict) {
            rc = rle_decode(ix, s, nn, [&](uint32_t j, uint32_t v) { L.a[j] = v; });
            if (rc) { set_err(err, err_any, rc, 0, 0, size); failed = 1; }
        } else if (!failed) {
            // PLAIN BYTE_ARRAY chain (249-253): serial by lane 0
            if (lane() == 0) {
                for (uint32_t k = 0; k < nn; k++) {
                    if (static_cast<uint64_t>(pos) + 4 > size) {
                        set_err(err, err_any, PQ_ERR_BUFFER, pos, 4, size);
                        failed = 1;
                        break;
                    }
                    uint32_t len = src_u32(s, pos);
                    pos += 4;
                    if (static_cast<uint64_t>(pos) + len > size) {
                        set_err(err, err_any, PQ_ERR_BUFFER, pos, len, size);
                        failed = 1;
                        break;
                    }
                    L.a[k] = pos;
                    L.b[k] = len;
                    pos += len;
                }
            }
            failed = __shfl(failed, 0, kWave);
            pos = __shfl(pos, 0, kWave);
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        uint64_t tile_sum = 0;
        uint32_t rank = 0;
        for (uint32_t j0 = 0; j0 < m; j0 += kWave) {
            uint32_t j = j0 + lane();
            bool in = j < m;
            int32_t d = in ? static_cast<int16_t>(lv[j]) : -32768;
            bool isnn = in && (dict ? d == cp.max_def : d >= cp.max_def);
            uint64_t mask = __ballot(isnn);
            uint32_t k = rank + popc_below(mask);
            rank += __popcll(mask);
            uint64_t code = 0xFFFFFFFFFFFFFFFFull;
            if (isnn && !failed) {
                if (dict) {
                    uint32_t idx = L.a[k];
                    if (static_cast<int32_t>(idx) >= 0 && idx < dict_n) code = entries[entry_base + idx];
                } else {
                    code = (static_cast<uint64_t>(L.b[k]) << 32) | L.a[k];
                }
            }
            if (in) row_codes[pg.first_row + r0 + j] = code;
            uint32_t len = code == 0xFFFFFFFFFFFFFFFFull ? 0u : static_cast<uint32_t>(code >> 32);
            // 64-bit wave sum
            uint64_t v = len;
#pragma unroll
            for (int dd = 32; dd >= 1; dd >>= 1) v += __shfl_xor(v, dd, kWave);
            tile_sum += v;
        }
        if (lane() == 0) tile_chars[tile0 + t] = failed ? 0 : static_cast<int64_t>(tile_sum);
        __builtin_amdgcn_wave_barrier();
    }
}

// kSW: LDS stage words per wave (pages up to 4 KiB, or up to 32 KiB with one
// wave per workgroup); kWPB: waves per workgroup.
template <uint32_t kSW, int kWPB>
__global__ void __launch_bounds__(kWPB * 64) k_ba_rows(const uint8_t* __restrict__ bytes,
                                                 const DevPage* __restrict__ pages, int npages,
                                                 const DevDict* __restrict__ dicts,
                                                 const uint64_t* __restrict__ entries,
                                                 const int32_t* __restrict__ dict_count,
                                                 ColumnParams cp, uint64_t* __restrict__ row_codes,
                                                 int64_t* __restrict__ tile_chars,
                                                 const int32_t* __restrict__ page_tile0,
                                                 DevErr* __restrict__ page_err,
                                                 int32_t* __restrict__ err_any, uint32_t big_plain_min) {
    __shared__ RowsLds<kSW> lds_all[kWPB];
    const int wv = threadIdx.x / kWave;
    const int p = blockIdx.x * kWPB + wv;
    if (p >= npages) return;
    RowsLds<kSW>& L = lds_all[wv];
    const DevPage pg = pages[p];
    if (big_plain_page(pg, cp, big_plain_min)) return;
    const uint32_t size = static_cast<uint32_t>(pg.size);
    const uint32_t* st = nullptr;
    if (size <= kSW * 4) {
        stage_page(L.stage, bytes + pg.off, size);
        st = L.stage;
    }
    ba_rows_page(bytes, pg, p, st, L.lv, L.a, L.b, dicts, entries, dict_count, cp, row_codes, tile_chars, page_tile0,
                 page_err, err_any);
}

// ── dictionary pages by a workgroup: k_wide_rows ───────────────────────────
// k_ba_rows walks a page's two hybrid streams one header at a time; a
// 20,000-row page with 17-bit indices (a 100k-entry dictionary, beyond the
// pipe's LDS dictionary) holds ~2,000 runs per stream, a serial chain of
// dependent reads.  Here one 16-wave workgroup owns a page (column_reader.cpp
// :174-196, max_def <= 1, no rep levels):
//   1. the payload -> LDS;
//   2. the def stream's run records by the whole workgroup (run_spec.hpp),
//      expanded per 512-row tile into a page validity bitmap in LDS and per-tile
//      non-null counts (def == max_def), scanned to tile ranks;
//   3. the index stream's records (num_non_null values, same scheme; the table
//      and the records reuse one region);
//   4. per tile: the tile's rank range expanded to indices (max-scan over the
//      record starts, 8 ranks per lane), then rows in order: NULL, index out
//      of range -> ~0, else the dictionary entry word (HBM/L2) -> row code and
//      the tile's character sum, exactly what k_ba_rows writes.
// Anything the record scheme does not take (non-dictionary pages, a level or
// prologue error, zero-count runs, table overflow, bw > 24) runs ba_rows_page
// on wave 0 over the staged payload, which also reports the reference's error.
constexpr int kWdWaves = 16;
constexpr uint32_t kWdThreads = kWdWaves * kWave;
constexpr uint32_t kWdPer = 48;  // spec positions per thread: streams up to 49,152 bytes (64 spill)
constexpr int kWdJumpLog = 4;  // 16-run jumps (64 measured slower: 0.206 -> 0.275 ms on the W column)
constexpr uint32_t kWdMaxRows = 65535;
constexpr uint32_t kWdTiles = (kWdMaxRows + kTileRows) / kTileRows;
constexpr uint32_t kWdWaveScratch = kTileRows * 2 + kTileRows * 4;  // mark u16 + ranks' indices u32
static_assert(kWdWaveScratch * kWdWaves >= 3 * kTileRows * 4, "exact path scratch fits the wave scratch");

struct WideLayout {
    uint32_t stage, stage_bytes;   // payload
    uint32_t tab, tab_bytes;       // speculative table, then the records (rcap), then wave scratch
    uint32_t rcap, scratch;        // records; wave scratch offset (inside the tab region)
    uint32_t list, esum, lcap;     // spec lists
    uint32_t pvalid;               // page validity bytes (kWdMaxRows / 8 + 16)
    uint32_t tnn, trank, sh;       // per-tile counts and ranks, scalars
    uint32_t bytes;
};

__host__ __device__ inline uint32_t wd_al16(uint32_t x) { return (x + 15u) & ~15u; }

__host__ inline WideLayout wide_layout(uint32_t max_page) {
    WideLayout L{};
    uint32_t o = 0;
    L.stage = o; L.stage_bytes = wd_al16(max_page) + 32; o += L.stage_bytes;
    const uint32_t scr = kWdWaveScratch * kWdWaves;
    const uint32_t tab_min = 2 * wd_al16(max_page) + 16;
    const uint32_t rec_min = 8 * std::max<uint32_t>(1024u, wd_al16(max_page) / 4);
    L.tab_bytes = wd_al16(std::max(tab_min, rec_min + scr));
    L.tab = o; o += L.tab_bytes;
    L.scratch = L.tab + L.tab_bytes - scr;
    L.rcap = (L.scratch - L.tab) / 8;
    L.lcap = L.rcap / 16 + 24;  // both streams' lists (spec_runs2) fit
    L.list = o; o += wd_al16(4 * L.lcap);
    L.esum = o; o += wd_al16(4 * L.lcap);
    L.pvalid = o; o += wd_al16(kWdMaxRows / 8 + 16);
    L.tnn = o; o += 4 * kWdTiles;
    L.trank = o; o += 4 * kWdTiles;
    L.sh = o; o += 64;
    L.bytes = o;
    return L;
}

// First record of rec[0 .. nrec) whose start (x & 0xFFFF) is <= v, searched
// from `from` (records are sorted by start; v never lies before rec[from]).
__device__ __forceinline__ uint32_t wd_find(const uint2* rec, uint32_t nrec, uint32_t from, uint32_t v) {
    uint32_t c = from;
    for (uint32_t k0 = from + 1; k0 < nrec; k0 += kWave) {
        const uint32_t k = k0 + lane();
        const uint64_t le = __ballot(k < nrec && (rec[k].x & 0xFFFFu) <= v);
        c += __popcll(le);
        if (le != ~0ull) break;
    }
    return c;
}

// Values [v0, v0 + m) (m <= kTileRows) of a stream with records rec: lane l
// produces values v0 + 8l .. 8l + 7 into out[8l ..] (a max-scan over the
// record starts marked in `mark`).  Returns the record holding v0.
template <class F>
__device__ __forceinline__ uint32_t wd_expand(const uint2* rec, uint32_t nrec, uint32_t rd_from, uint32_t v0,
                                              uint32_t m, uint16_t* mark, F&& value) {
    const uint32_t rd0 = wd_find(rec, nrec, rd_from, v0);
    const uint32_t l8 = lane() * 8;
    if (l8 < kTileRows) *reinterpret_cast<uint4*>(mark + l8) = make_uint4(0u, 0u, 0u, 0u);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    for (uint32_t k = rd0 + 1 + lane(); k < nrec; k += kWave) {
        const uint32_t st = rec[k].x & 0xFFFFu;
        if (st >= v0 + m) break;
        mark[st - v0] = static_cast<uint16_t>(k - rd0);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint4 mk = *reinterpret_cast<const uint4*>(mark + l8);
    const uint32_t mw[4] = {mk.x, mk.y, mk.z, mk.w};
    uint32_t rm[8], run = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        run = max(run, (mw[k >> 1] >> (16 * (k & 1))) & 0xFFFFu);
        rm[k] = run;
    }
    const uint32_t ex = static_cast<uint32_t>(
        __builtin_amdgcn_update_dpp(0, static_cast<int>(wave_incl_max(run)), 0x138, 0xf, 0xf, true));
    // the eight records first (unconditional: past m the scan still names a
    // record of the tile), then the values, branch-free
    uint2 R[8];
#pragma unroll
    for (int k = 0; k < 8; k++) R[k] = rec[rd0 + max(ex, rm[k])];
#pragma unroll
    for (int k = 0; k < 8; k++) value(l8 + k, R[k], v0 + l8 + k - (R[k].x & 0xFFFFu));
    __builtin_amdgcn_wave_barrier();
    return rd0;
}

// Value of run record R at `off` values into it: the RLE value, or bw bits of
// the staged page (words past `nwords` read as zero, like bytes past the
// page), with clamped unconditional LDS reads and selects.
__device__ __forceinline__ uint32_t wd_value(const uint32_t* stage, uint32_t nwords, const uint2& R, uint32_t off,
                                             uint32_t bw) {
    const uint64_t b = static_cast<uint64_t>(R.y & 0x7FFFFFFFu) + static_cast<uint64_t>(off) * bw;
    const uint32_t wi = static_cast<uint32_t>(min(b >> 5, static_cast<uint64_t>(0x7FFFFFF0u)));
    const uint32_t lo = stage[min(wi, nwords - 1)], hi = stage[min(wi + 1, nwords - 1)];
    const uint64_t v = (static_cast<uint64_t>(wi + 1 < nwords ? hi : 0u) << 32) | (wi < nwords ? lo : 0u);
    const uint32_t x = static_cast<uint32_t>(v >> (b & 31)) & ((bw >= 32 ? 0u : (1u << bw)) - 1u);
    return (R.y >> 31) ? x : (R.y & 0x7FFFFFFFu);
}

__global__ void __launch_bounds__(kWdThreads) k_wide_rows(const uint8_t* __restrict__ bytes,
                                                         const DevPage* __restrict__ pages,
                                                         const DevDict* __restrict__ dicts,
                                                         const uint64_t* __restrict__ entries,
                                                         const int32_t* __restrict__ dict_count, ColumnParams cp,
                                                         uint64_t* __restrict__ row_codes,
                                                         int64_t* __restrict__ tile_chars,
                                                         const int32_t* __restrict__ page_tile0,
                                                         DevErr* __restrict__ page_err, int32_t* __restrict__ err_any,
                                                         uint32_t big_plain_min, WideLayout Lo,
                                                         uint64_t* __restrict__ prof) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    // "fused_prof": thread 0's shader-clock time per phase (slots 0-5), fallback
    // pages (6) and pages (7), summed over workgroups
    uint64_t tprev = prof ? __builtin_amdgcn_s_memtime() : 0;
    auto pmark = [&](int slot) {
        if (prof && threadIdx.x == 0) {
            const uint64_t now = __builtin_amdgcn_s_memtime();
            atomicAdd(reinterpret_cast<unsigned long long*>(prof + slot), now - tprev);
            tprev = now;
        }
    };
    uint32_t* stage = reinterpret_cast<uint32_t*>(smem + Lo.stage);
    uint16_t* tab = reinterpret_cast<uint16_t*>(smem + Lo.tab);
    uint2* rec = reinterpret_cast<uint2*>(smem + Lo.tab);
    uint32_t* list = reinterpret_cast<uint32_t*>(smem + Lo.list);
    uint32_t* esum = reinterpret_cast<uint32_t*>(smem + Lo.esum);
    uint8_t* pvalid = smem + Lo.pvalid;
    uint32_t* tnn = reinterpret_cast<uint32_t*>(smem + Lo.tnn);
    uint32_t* trank = reinterpret_cast<uint32_t*>(smem + Lo.trank);
    uint32_t* sh = reinterpret_cast<uint32_t*>(smem + Lo.sh);
    const uint32_t wv = threadIdx.x / kWave;
    uint8_t* wscr = smem + Lo.scratch + wv * kWdWaveScratch;
    uint16_t* mark = reinterpret_cast<uint16_t*>(wscr);
    uint32_t* ixv = reinterpret_cast<uint32_t*>(wscr + 2 * kTileRows);

    const int p = blockIdx.x;
    const DevPage pg = pages[p];
    if (big_plain_page(pg, cp, big_plain_min)) return;
    const uint32_t size = static_cast<uint32_t>(max(pg.size, 0));
    const uint32_t n = static_cast<uint32_t>(max(pg.nvals, 0));
    const bool staged = size + 32 <= Lo.stage_bytes;
    if (staged) copy_blocks(reinterpret_cast<uint4*>(stage), reinterpret_cast<const uint4*>(bytes + pg.off),
                            (size + 15) / 16 + 1, threadIdx.x, kWdThreads);
    if (threadIdx.x == 0) {  // prologue (column_reader.cpp:146-182): sh = fast, def len, index base, index bw
        uint32_t fast = staged && pg.mode == MODE_DICT && pg.dict >= 0 && n <= kWdMaxRows && cp.max_rep == 0 &&
                        cp.max_def <= 1;
        uint32_t pos = 0, dlen = 0, ibw = 0;
        if (fast && cp.max_def == 1) {
            if (4 > size) fast = 0;
            else {
                dlen = static_cast<uint32_t>(gld8(bytes + pg.off, 0));
                if (4ull + dlen > size || size - 5 > kWdThreads * kWdPer) fast = 0;  // both streams in one table
                else pos = 4 + dlen;
            }
        }
        if (fast) {
            if (pos + 1 > size) fast = 0;
            else {
                ibw = bytes[pg.off + pos];
                pos += 1;
                if (ibw > 24 || size - pos > kWdThreads * kWdPer) fast = 0;
            }
        }
        sh[4] = fast;
        sh[5] = dlen;
        sh[6] = pos;
        sh[7] = ibw;
    }
    __syncthreads();
    pmark(0);
    uint32_t fast = sh[4];
    const uint32_t dlen = sh[5], ibase = sh[6], ibw = sh[7];
    const uint32_t swords = (size + 16) / 4;  // staged words: the payload, then slot padding (zeros)
    const uint32_t ntiles = (n + kTileRows - 1) / kTileRows;
    // 2. run records of both streams in one pass (spec_runs2: def levels at
    //    [4, 4 + dlen), indices from ibase to the page end, the latter over
    //    all n rows as an upper bound of num_non_null: only ranks < nn are
    //    read), then def records -> validity bytes, tile counts
    uint2* irec = rec;
    uint32_t ni = 0;
    if (fast && cp.max_def == 1) {
        constexpr uint32_t kJ = 1u << kWdJumpLog;
        const uint32_t rc0 = min(Lo.rcap / 2, (dlen / 2 + 3 * kJ + 15) & ~15u);  // def runs <= dlen / 2 + 1
        const uint32_t base2[2] = {4u, ibase}, len2[2] = {dlen, size - ibase}, bw2[2] = {1u, ibw}, n2[2] = {n, n};
        const uint32_t rcap2[2] = {rc0, Lo.rcap - rc0};
        const uint32_t lcap2[2] = {rc0 / kJ + 8, (Lo.rcap - rc0) / kJ + 8};
        uint2* const rec2[2] = {rec, rec + rc0};
        uint32_t cnt2[2];
        spec_runs2<kWdThreads, kWdPer, kWdJumpLog>(stage, base2, len2, bw2, n2, tab, list, esum, lcap2, rec2, rcap2,
                                                   sh + 8, cnt2);
        irec = rec + rc0;
        ni = cnt2[1];
        if (ni == ~0u) fast = 0;
        const uint32_t nd = fast ? cnt2[0] : ~0u;
        pmark(1);
        if (nd == ~0u) fast = 0;
        else {
            uint32_t rd = 0;
            for (uint32_t ti = wv; ti < ntiles; ti += kWdWaves) {
                const uint32_t r0 = ti * kTileRows, m = min(n - r0, static_cast<uint32_t>(kTileRows));
                uint32_t vb = 0;
                rd = wd_expand(rec, nd, rd, r0, m, mark, [&](uint32_t j, const uint2& R, uint32_t off) {
                    vb |= (j < m && wd_value(stage, swords, R, off, 1) == 1u ? 1u : 0u) << (j & 7);
                });
                pvalid[(r0 >> 3) + lane()] = static_cast<uint8_t>(vb);
                const uint32_t c = bcast_last(wave_incl_scan(__popc(vb)));
                if (lane() == 0) tnn[ti] = c;
            }
        }
    } else if (fast) {
        for (uint32_t i = threadIdx.x; i < (n + 7) / 8; i += kWdThreads) {
            const uint32_t r = i * 8;
            pvalid[i] = static_cast<uint8_t>(n - r >= 8 ? 0xFFu : ((1u << (n - r)) - 1u));
        }
        for (uint32_t ti = threadIdx.x; ti < ntiles; ti += kWdThreads) tnn[ti] = min(n - ti * kTileRows, kTileRows);
    }
    __syncthreads();
    pmark(2);
    if (fast && wv == 0) {  // tile ranks
        uint32_t carry = 0;
        for (uint32_t i0 = 0; i0 < ntiles; i0 += kWave) {
            const uint32_t i = i0 + lane();
            const uint32_t v = i < ntiles ? tnn[i] : 0u;
            const uint32_t inc = wave_incl_scan(v);
            if (i < ntiles) trank[i] = carry + inc - v;
            carry += bcast_last(inc);
        }
        if (lane() == 0) sh[8] = carry;
    }
    __syncthreads();
    pmark(3);
    // 3. index records (num_non_null values; column_reader.cpp:180-182):
    //    REQUIRED chunks here (all rows non-null), OPTIONAL ones above
    const uint32_t nn = fast ? sh[8] : 0u;
    if (fast && cp.max_def == 0 && nn > 0) {
        ni = spec_runs<kWdThreads, kWdPer, true, kWdJumpLog>(stage, ibase, size - ibase, ibw, nn, tab, list, esum, Lo.lcap, rec, Lo.rcap,
                                           sh);
        if (ni == ~0u) fast = 0;
    }
    pmark(4);
    if (prof && threadIdx.x == 0) {
        atomicAdd(reinterpret_cast<unsigned long long*>(prof + 7), 1ull);
        if (!fast) atomicAdd(reinterpret_cast<unsigned long long*>(prof + 6), 1ull);
    }
    if (!fast) {  // the exact per-page walk (reports the reference's errors)
        if (wv == 0) {
            uint32_t* scr = reinterpret_cast<uint32_t*>(smem + Lo.scratch);
            ba_rows_page(bytes, pg, p, staged ? stage : nullptr, scr, scr + kTileRows, scr + 2 * kTileRows, dicts,
                         entries, dict_count, cp, row_codes, tile_chars, page_tile0, page_err, err_any);
        }
        return;
    }
    // 4. rows
    const uint32_t dict_n = static_cast<uint32_t>(max(dict_count[pg.dict], 0));
    const uint64_t* ent = entries + dicts[pg.dict].entry_base;
    const int32_t tile0 = page_tile0[p];
    uint32_t rd = 0;
    for (uint32_t ti = wv; ti < ntiles; ti += kWdWaves) {
        const uint32_t r0 = ti * kTileRows, m = min(n - r0, static_cast<uint32_t>(kTileRows));
        const uint32_t cnt = tnn[ti];
        if (cnt) {
            rd = wd_expand(irec, ni, rd, trank[ti], cnt, mark, [&](uint32_t j, const uint2& R, uint32_t off) {
                ixv[j] = wd_value(stage, swords, R, off, ibw);
            });
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        // every row group's dictionary load is issued before any is used
        // (one L2/HBM latency per tile, not one per 64 rows)
        uint32_t run = 0;
        uint64_t code[kTileRows / kWave];
#pragma unroll
        for (uint32_t u = 0; u < kTileRows / kWave; u++) {
            const uint32_t j = u * kWave + lane();
            const bool v = j < m && ((pvalid[(r0 + j) >> 3] >> (j & 7)) & 1u);
            const uint64_t vm = __ballot(v);
            code[u] = ~0ull;
            if (v) {
                const uint32_t idx = ixv[run + popc_below(vm)];
                if (idx < dict_n) code[u] = ent[idx];
            }
            run += __popcll(vm);
        }
        uint64_t sum = 0;
        uint64_t* out = row_codes + pg.first_row + r0;
#pragma unroll
        for (uint32_t u = 0; u < kTileRows / kWave; u++) {
            const uint32_t j = u * kWave + lane();
            if (j < m) out[j] = code[u];
            sum += code[u] == ~0ull ? 0u : (code[u] >> 32);
        }
#pragma unroll
        for (int dd = 32; dd >= 1; dd >>= 1) sum += __shfl_xor(sum, dd, kWave);
        if (lane() == 0) tile_chars[tile0 + ti] = static_cast<int64_t>(sum);
        __builtin_amdgcn_wave_barrier();
    }
    if (prof) {
        __syncthreads();
        pmark(5);
    }
}

// ── exclusive scan of int64 (3 phases) ─────────────────────────────────────
constexpr int kScanBlock = 1024;
constexpr int kScanItems = 8;  // per thread

__device__ int64_t block_excl_scan(int64_t v, int64_t* sh, int64_t* total) {
    // sh: kScanBlock/64 slots
    int64_t x = v;
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        int64_t t = __shfl_up(x, d, kWave);
        if (lane() >= static_cast<uint32_t>(d)) x += t;
    }
    const int w = threadIdx.x / kWave;
    if (lane() == kWave - 1) sh[w] = x;
    __syncthreads();
    if (w == 0) {
        int64_t y = lane() < blockDim.x / kWave ? sh[lane()] : 0;
#pragma unroll
        for (int d = 1; d < kWave; d <<= 1) {
            int64_t t = __shfl_up(y, d, kWave);
            if (lane() >= static_cast<uint32_t>(d)) y += t;
        }
        if (lane() < blockDim.x / kWave) sh[lane()] = y;
    }
    __syncthreads();
    int64_t base = w ? sh[w - 1] : 0;
    *total = sh[blockDim.x / kWave - 1];
    __syncthreads();
    return base + x - v;
}

__global__ void __launch_bounds__(kScanBlock) k_scan_reduce(const int64_t* __restrict__ in, int64_t n,
                                                            int64_t* __restrict__ block_sums) {
    __shared__ int64_t sh[kScanBlock / kWave];
    int64_t base = static_cast<int64_t>(blockIdx.x) * kScanBlock * kScanItems;
    int64_t acc = 0;
    for (int i = 0; i < kScanItems; i++) {
        int64_t idx = base + static_cast<int64_t>(i) * kScanBlock + threadIdx.x;
        if (idx < n) acc += in[idx];
    }
    int64_t tot;
    block_excl_scan(acc, sh, &tot);
    if (threadIdx.x == 0) block_sums[blockIdx.x] = tot;
}

__global__ void __launch_bounds__(kScanBlock) k_scan_blocks(int64_t* __restrict__ sums, int64_t nb,
                                                            int64_t* __restrict__ total) {
    __shared__ int64_t sh[kScanBlock / kWave];
    int64_t carry = 0;
    for (int64_t b0 = 0; b0 < nb; b0 += kScanBlock) {
        int64_t idx = b0 + threadIdx.x;
        int64_t v = idx < nb ? sums[idx] : 0;
        int64_t tot;
        int64_t ex = block_excl_scan(v, sh, &tot);
        if (idx < nb) sums[idx] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) *total = carry;
}

__global__ void __launch_bounds__(kScanBlock) k_scan_apply(const int64_t* __restrict__ in, int64_t n,
                                                           const int64_t* __restrict__ block_off,
                                                           int64_t* __restrict__ out) {
    __shared__ int64_t sh[kScanBlock / kWave];
    // each thread owns kScanItems consecutive elements
    int64_t base = static_cast<int64_t>(blockIdx.x) * kScanBlock * kScanItems +
                   static_cast<int64_t>(threadIdx.x) * kScanItems;
    int64_t v[kScanItems];
    int64_t acc = 0;
    for (int i = 0; i < kScanItems; i++) {
        v[i] = base + i < n ? in[base + i] : 0;
        acc += v[i];
    }
    int64_t tot;
    int64_t ex = block_excl_scan(acc, sh, &tot) + block_off[blockIdx.x];
    for (int i = 0; i < kScanItems; i++) {
        if (base + i < n) out[base + i] = ex;
        ex += v[i];
    }
}

// One workgroup scans up to kScanBlock * kScanSingle elements in one launch.
// Wave w owns a contiguous range; every load and store is 64 consecutive
// elements across the lanes (a per-thread run of 32 elements made each load
// instruction touch 64 cache lines).  Pass 1 sums the range, a scan over the
// waves' sums gives each range its base, pass 2 re-reads (L2) and scans 64
// elements per step with a carry.
constexpr int kScanSingle = 32;
__device__ __forceinline__ int64_t wave_incl_scan64(int64_t x) {
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        const int64_t t = __shfl_up(x, d, kWave);
        if (lane() >= static_cast<uint32_t>(d)) x += t;
    }
    return x;
}
__global__ void __launch_bounds__(kScanBlock) k_scan_single(const int64_t* __restrict__ in, int64_t n,
                                                            int64_t* __restrict__ out,
                                                            int64_t* __restrict__ total) {
    __shared__ int64_t sh[kScanBlock / kWave];
    constexpr int kW = kScanBlock / kWave;
    const int w = static_cast<int>(threadIdx.x / kWave);
    const int64_t per = (n + kW - 1) / kW;
    const int64_t lo = min(n, w * per), hi = min(n, lo + per);
    constexpr int kB = 8;  // 64-element groups loaded per batch (one latency per batch)
    int64_t acc = 0;
    for (int64_t b0 = lo; b0 < hi; b0 += kB * kWave) {
        int64_t v[kB];
#pragma unroll
        for (int u = 0; u < kB; u++) {
            const int64_t i = b0 + u * kWave + lane();
            v[u] = i < hi ? in[i] : 0;
        }
#pragma unroll
        for (int u = 0; u < kB; u++) acc += v[u];
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) acc += __shfl_xor(acc, d, kWave);
    if (lane() == 0) sh[w] = acc;
    __syncthreads();
    int64_t carry = 0;
    for (int k = 0; k < w; k++) carry += sh[k];
    if (threadIdx.x == 0) {
        int64_t t = 0;
        for (int k = 0; k < kW; k++) t += sh[k];
        *total = t;
    }
    for (int64_t b0 = lo; b0 < hi; b0 += kB * kWave) {
        int64_t v[kB];
#pragma unroll
        for (int u = 0; u < kB; u++) {
            const int64_t i = b0 + u * kWave + lane();
            v[u] = i < hi ? in[i] : 0;
        }
#pragma unroll
        for (int u = 0; u < kB; u++) {
            const int64_t i = b0 + u * kWave + lane();
            const int64_t inc = wave_incl_scan64(v[u]);
            if (i < hi) out[i] = carry + inc - v[u];
            carry += __shfl(inc, kWave - 1, kWave);
        }
    }
}

// ── BYTE_ARRAY gather: offsets, validity, chars ────────────────────────────
constexpr int kGatherWindow = 2048;  // 16-byte output blocks per window (32 KiB)
struct GatherLds {
    uint32_t loff[kTileRows + 1];
    uint32_t src[kTileRows];
    uint16_t blockrow[kGatherWindow];
};

// The byte-wise form (option "gather_rows" 0): 16-byte output blocks, each
// assembled from the rows that cover it.
__device__ void gather_bytes(GatherLds& L, const uint8_t* __restrict__ srcbase, uint32_t n, int64_t G0, int64_t G1,
                             int64_t B0, int64_t nb, uint8_t* __restrict__ chars) {
    for (int64_t w0 = 0; w0 < nb; w0 += kGatherWindow) {
        const int64_t w1 = min(nb, w0 + static_cast<int64_t>(kGatherWindow));
        // scatter: row r owns the blocks whose first in-tile byte lies in it
        for (uint32_t r = lane(); r < n; r += kWave) {
            uint32_t s = L.loff[r], e = L.loff[r + 1];
            if (e <= s) continue;
            int64_t blo = s == 0 ? 0 : ((s + G0 + 15) >> 4) - B0;
            int64_t bhi = ((e + G0 + 15) >> 4) - B0 - 1;
            blo = max(blo, w0);
            bhi = min(bhi, w1 - 1);
            for (int64_t b = blo; b <= bhi; b++) L.blockrow[b - w0] = static_cast<uint16_t>(r);
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        for (int64_t b = w0 + lane(); b < w1; b += kWave) {
            const int64_t blk = (B0 + b) << 4;
            const int64_t gs = max(blk, G0), ge = min(blk + 16, G1);
            uint32_t r = L.blockrow[b - w0];
            uint32_t q = static_cast<uint32_t>(gs - G0);
            uint32_t p = q - L.loff[r];
            uint32_t outw[4] = {0, 0, 0, 0};
            const uint32_t cnt = static_cast<uint32_t>(ge - gs);
            const uint32_t first = static_cast<uint32_t>(gs - blk);
            for (uint32_t k = 0; k < cnt; k++) {
                while (r + 1 < n && p >= L.loff[r + 1] - L.loff[r]) { r++; p = 0; }
                uint32_t byte = srcbase[L.src[r] + p];
                p++;
                uint32_t at = first + k;
                outw[at >> 2] |= byte << (8 * (at & 3));
            }
            if (cnt == 16) {
                *reinterpret_cast<uint4*>(chars + blk) = make_uint4(outw[0], outw[1], outw[2], outw[3]);
            } else {
                for (uint32_t k = 0; k < cnt; k++) {
                    uint32_t at = first + k;
                    chars[blk + at] = static_cast<uint8_t>(outw[at >> 2] >> (8 * (at & 3)));
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    }
}


__global__ void __launch_bounds__(256) k_ba_gather(const uint8_t* __restrict__ bytes,
                                                   const DevPage* __restrict__ pages,
                                                   const DevTile* __restrict__ tiles, int ntiles,
                                                   const DevDict* __restrict__ dicts,
                                                   const uint64_t* __restrict__ row_codes,
                                                   const int64_t* __restrict__ tile_base,
                                                   int64_t nrows_total,
                                                   const int64_t* __restrict__ total_ptr,
                                                   int64_t capacity, int32_t* __restrict__ overflow,
                                                   uint32_t* __restrict__ validity,
                                                   int64_t* __restrict__ offsets,
                                                   uint8_t* __restrict__ chars, bool byte_gather) {
    __shared__ GatherLds lds_all[kWavesPerBlock];
    const int wv = threadIdx.x / kWave;
    const int t = blockIdx.x * kWavesPerBlock + wv;
    if (t >= ntiles) return;
    GatherLds& L = lds_all[wv];
    const DevTile tl = tiles[t];
    const DevPage pg = pages[tl.page];
    const uint8_t* srcbase = bytes + (pg.mode == MODE_DICT ? dicts[pg.dict].off : pg.off);
    const int64_t R0 = pg.first_row + tl.row0;
    const uint32_t n = static_cast<uint32_t>(tl.nrows);
    const int64_t G0 = tile_base[t];

    // lengths -> local offsets, validity bits, global offsets
    uint32_t run = 0;
    for (uint32_t j0 = 0; j0 < n; j0 += kWave) {
        uint32_t j = j0 + lane();
        bool in = j < n;
        uint64_t code = in ? row_codes[R0 + j] : 0xFFFFFFFFFFFFFFFFull;
        bool valid = code != 0xFFFFFFFFFFFFFFFFull;
        uint32_t len = valid ? static_cast<uint32_t>(code >> 32) : 0u;
        uint32_t inc = wave_incl_scan(len);
        uint32_t ex = run + inc - len;
        if (in) {
            L.loff[j] = ex;
            L.src[j] = valid ? static_cast<uint32_t>(code) : 0u;
            offsets[R0 + j] = G0 + ex;
        }
        run += bcast_last(inc);
        uint64_t vm = __ballot(valid);
        int64_t R = R0 + j0;
        uint32_t w = static_cast<uint32_t>(R >> 5), sh = static_cast<uint32_t>(R & 31);
        // bits [R, R+64) -> up to three 32-bit words
        if (lane() < 3) {
            uint32_t part;
            if (lane() == 0) part = static_cast<uint32_t>(vm << sh);
            else if (lane() == 1) part = static_cast<uint32_t>((sh ? (vm >> (32 - sh)) : (vm >> 32)));
            else part = sh ? static_cast<uint32_t>(vm >> (64 - sh)) : 0u;
            if (part) atomicOr(&validity[w + lane()], part);
        }
    }
    if (lane() == 0) L.loff[n] = run;
    if (R0 + n == nrows_total && lane() == 0) offsets[nrows_total] = *total_ptr;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");

    const uint32_t total = run;
    if (total == 0) return;
    if (G0 + total > capacity) {  // output buffer too small: host grows it and re-runs
        if (lane() == 0) atomicOr(overflow, 1);
        return;
    }
    // characters: row per lane, unaligned 16-byte moves (row_copy.hpp); the
    // rows of neighbouring lanes are adjacent in the output
    if (byte_gather) {
        const int64_t G1 = G0 + total;
        const int64_t B0 = G0 >> 4;
        const int64_t nb = ((G1 - 1) >> 4) - B0 + 1;
        gather_bytes(L, srcbase, n, G0, G1, B0, nb, chars);
        return;
    }
    uint8_t* out = chars + G0;
    for (uint32_t r = lane(); r < n; r += kWave) {
        const uint32_t s = L.loff[r], e = L.loff[r + 1];
        rc::copy_row_g(out + s, srcbase + L.src[r], e - s);
    }
}

// ── fixed-width values (INT32/INT64/FLOAT/DOUBLE/INT96/BOOLEAN) ─────────────
struct FixedLds {
    uint32_t stage[kStageWords];
    uint32_t lv[kTileRows];
    uint32_t a[kTileRows];
};

__global__ void __launch_bounds__(256) k_fixed(const uint8_t* __restrict__ bytes,
                                               const DevPage* __restrict__ pages, int npages,
                                               const DevDict* __restrict__ dicts,
                                               const int32_t* __restrict__ dict_count,
                                               ColumnParams cp, uint32_t* __restrict__ validity,
                                               uint8_t* __restrict__ values,
                                               DevErr* __restrict__ page_err,
                                               int32_t* __restrict__ err_any) {
    __shared__ FixedLds lds_all[kWavesPerBlock];
    const int wv = threadIdx.x / kWave;
    const int p = blockIdx.x * kWavesPerBlock + wv;
    if (p >= npages) return;
    FixedLds& L = lds_all[wv];
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
    const uint32_t W = static_cast<uint32_t>(cp.width);
    const uint32_t PW = static_cast<uint32_t>(cp.plain_width);
    PagePrologue pp;
    if (page_prologue(s, cp, pp, err, err_any)) return;
    uint32_t pos = pp.pos;
    const int mode = pg.mode;
    Rle ix;
    uint32_t dict_n = 0;
    Src ds{nullptr, nullptr, 0};
    if (mode == MODE_BOOL_RLE) {  // [u32 len][hybrid RLE/bit-packed, bit width 1]
        if (pos + 4 > size) { set_err(err, err_any, PQ_ERR_BUFFER, pos, 4, size); return; }
        const uint32_t bl = src_u32(s, pos);
        pos += 4;
        if (static_cast<uint64_t>(pos) + bl > size) { set_err(err, err_any, PQ_ERR_BUFFER, pos, bl, size); return; }
        rle_init(ix, pos, bl, 1);
    }
    if (mode == MODE_DICT) {
        if (pos + 1 > size) { set_err(err, err_any, PQ_ERR_BUFFER, pos, 1, size); return; }
        uint32_t bw = src_byte(s, pos);
        pos += 1;
        rle_init(ix, pos, size - pos, bw);
        dict_n = static_cast<uint32_t>(dict_count[pg.dict]);
        const DevDict dd = dicts[pg.dict];
        ds = Src{nullptr, bytes + dd.off, static_cast<uint32_t>(dd.size)};
    }
    uint32_t rank_base = 0;  // non-null values before this tile (PLAIN / BOOLEAN)
    for (int32_t r0 = 0; r0 < nv; r0 += kTileRows) {
        const uint32_t m = min(static_cast<uint32_t>(nv - r0), static_cast<uint32_t>(kTileRows));
        int rc = 0;
        if (pp.has_def) {
            rc = rle_decode(pp.def, s, m, [&](uint32_t j, uint32_t v) { L.lv[j] = v & 0xFFFFu; });
        } else {
            for (uint32_t j = lane(); j < m; j += kWave) L.lv[j] = static_cast<uint32_t>(cp.max_def);
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        uint32_t nn = 0, above = 0;
        const bool dict = mode == MODE_DICT;
        for (uint32_t j0 = 0; j0 < m; j0 += kWave) {
            uint32_t j = j0 + lane();
            int32_t d = j < m ? static_cast<int16_t>(L.lv[j]) : -32768;
            bool isnn = dict ? d == cp.max_def : d >= cp.max_def;
            nn += __popcll(__ballot(isnn));
            above |= __ballot(d > cp.max_def) != 0;
        }
        if (rc == 0 && dict && above) rc = PQ_ERR_UNSUPPORTED;
        if (rc) { set_err(err, err_any, rc, 0, 0, size); return; }
        if (dict || mode == MODE_BOOL_RLE) {
            rc = rle_decode(ix, s, nn, [&](uint32_t j, uint32_t v) { L.a[j] = v; });
            if (rc) { set_err(err, err_any, rc, 0, 0, size); return; }
        } else if (nn > 0) {
            // PLAIN bounds: the first rank whose read overruns (ByteBuffer::check)
            if (cp.type == PQ_FIXED_LEN_BYTE_ARRAY) { set_err(err, err_any, PQ_ERR_FLBA, 0, 0, size); return; }
            if (PW == 0 && mode != MODE_BOOL) { set_err(err, err_any, PQ_ERR_TYPE, 0, 0, size); return; }
            if (mode == MODE_BOOL) {
                uint64_t last = rank_base + nn - 1;  // bytes needed: floor(last/8)+1
                uint64_t need_end = pos + last / 8 + 1;
                if (need_end > size) {
                    uint64_t k = static_cast<uint64_t>(size - pos) * 8;  // first rank without a byte
                    set_err(err, err_any, PQ_ERR_BUFFER, static_cast<uint32_t>(pos + k / 8), 1, size);
                    return;
                }
            } else {
                uint64_t need_end = pos + static_cast<uint64_t>(rank_base + nn) * PW;
                if (need_end > size) {
                    uint64_t k = (size - pos) / PW;
                    set_err(err, err_any, PQ_ERR_BUFFER, static_cast<uint32_t>(pos + k * PW), PW, size);
                    return;
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        uint32_t rank = 0;
        for (uint32_t j0 = 0; j0 < m; j0 += kWave) {
            uint32_t j = j0 + lane();
            bool in = j < m;
            int32_t d = in ? static_cast<int16_t>(L.lv[j]) : -32768;
            bool isnn = in && (dict ? d == cp.max_def : d >= cp.max_def);
            uint64_t mask = __ballot(isnn);
            uint32_t k = rank + popc_below(mask);
            rank += __popcll(mask);
            bool valid = isnn;
            uint32_t w[3] = {0, 0, 0};
            if (isnn) {
                if (dict) {
                    uint32_t idx = L.a[k];
                    valid = static_cast<int32_t>(idx) >= 0 && idx < dict_n;
                    if (valid) {
                        uint32_t at = idx * PW;
                        if (cp.type == PQ_BOOLEAN) w[0] = src_byte(ds, at) != 0;
                        else for (uint32_t q = 0; q < (W + 3) / 4; q++) w[q] = src_u32(ds, at + 4 * q);
                    }
                } else if (mode == MODE_BOOL_RLE) {
                    w[0] = L.a[k] & 1u;
                } else if (mode == MODE_BOOL) {
                    uint32_t kk = rank_base + k;
                    w[0] = (src_byte(s, pos + kk / 8) >> (kk % 8)) & 1u;
                } else {
                    uint32_t at = pos + (rank_base + k) * PW;
                    if (cp.type == PQ_BOOLEAN) w[0] = src_byte(s, at) != 0;
                    else for (uint32_t q = 0; q < (W + 3) / 4; q++) w[q] = src_u32(s, at + 4 * q);
                }
            }
            const int64_t R = pg.first_row + r0 + j;
            if (in) {
                uint8_t* o = values + R * W;
                if (W == 4) *reinterpret_cast<uint32_t*>(o) = w[0];
                else if (W == 8) *reinterpret_cast<uint2*>(o) = make_uint2(w[0], w[1]);
                else if (W == 1) *o = static_cast<uint8_t>(w[0]);
                else for (uint32_t q = 0; q < W / 4; q++) reinterpret_cast<uint32_t*>(o)[q] = w[q];
            }
            uint64_t vm = __ballot(valid && in);
            const int64_t RB = pg.first_row + r0 + j0;
            uint32_t wi = static_cast<uint32_t>(RB >> 5), sh = static_cast<uint32_t>(RB & 31);
            if (lane() < 3) {
                uint32_t part;
                if (lane() == 0) part = static_cast<uint32_t>(vm << sh);
                else if (lane() == 1) part = static_cast<uint32_t>(sh ? (vm >> (32 - sh)) : (vm >> 32));
                else part = sh ? static_cast<uint32_t>(vm >> (64 - sh)) : 0u;
                if (part) atomicOr(&validity[wi + lane()], part);
            }
        }
        if (!dict) rank_base += nn;
        __builtin_amdgcn_wave_barrier();
    }
}

}  // namespace

void launch_dict_entries(hipStream_t s, const uint8_t* bytes, const DevDict* dicts, int ndicts,
                         uint64_t* entries, int32_t* dict_count, DevErr* dict_err, int32_t* err_any,
                         int32_t type, int32_t plain_width) {
    if (ndicts <= 0) return;
    hipLaunchKernelGGL(k_dict_entries, dim3(ndicts), dim3(64), 0, s, bytes, dicts, entries,
                       dict_count, dict_err, err_any, type, plain_width);
}

void launch_ba_rows(hipStream_t s, const uint8_t* bytes, const DevPage* pages, int npages,
                    const DevDict* dicts, const uint64_t* entries, const int32_t* dict_count,
                    ColumnParams cp, uint64_t* row_codes, int64_t* tile_chars,
                    const int32_t* page_tile0, DevErr* page_err, int32_t* err_any, uint32_t big_plain_min,
                    uint32_t max_page, bool wide, uint64_t* prof) {
    if (npages <= 0) return;
    if (wide && cp.max_rep == 0 && cp.max_def <= 1) {
        const WideLayout Lo = wide_layout(max_page);
        if (Lo.bytes <= 160 * 1024 && ensure_dyn_lds(reinterpret_cast<const void*>(k_wide_rows), Lo.bytes)) {
            hipLaunchKernelGGL(k_wide_rows, dim3(npages), dim3(kWdThreads), Lo.bytes, s, bytes, pages, dicts, entries,
                               dict_count, cp, row_codes, tile_chars, page_tile0, page_err, err_any, big_plain_min, Lo,
                               prof);
            return;
        }
    }
    if (max_page > kStageWords * 4) {  // pages up to 32 KiB decode from LDS too
        hipLaunchKernelGGL((k_ba_rows<8192, 1>), dim3(npages), dim3(64), 0, s, bytes, pages, npages, dicts,
                           entries, dict_count, cp, row_codes, tile_chars, page_tile0, page_err, err_any,
                           big_plain_min);
        return;
    }
    int blocks = (npages + kWavesPerBlock - 1) / kWavesPerBlock;
    hipLaunchKernelGGL((k_ba_rows<kStageWords, kWavesPerBlock>), dim3(blocks), dim3(256), 0, s, bytes, pages,
                       npages, dicts, entries, dict_count, cp, row_codes, tile_chars, page_tile0, page_err,
                       err_any, big_plain_min);
}

uint32_t ba_rows_stage_bytes() { return kStageWords * 4; }

void launch_scan_i64(hipStream_t s, const int64_t* in, int64_t* out_excl, int64_t n,
                     int64_t* total, int64_t* scratch) {
    if (n <= 0) {
        (void)hipMemsetAsync(total, 0, sizeof(int64_t), s);
        return;
    }
    if (n <= static_cast<int64_t>(kScanBlock) * kScanSingle) {
        hipLaunchKernelGGL(k_scan_single, dim3(1), dim3(kScanBlock), 0, s, in, n, out_excl, total);
        return;
    }
    const int64_t per = static_cast<int64_t>(kScanBlock) * kScanItems;
    int64_t nb = (n + per - 1) / per;
    hipLaunchKernelGGL(k_scan_reduce, dim3(static_cast<uint32_t>(nb)), dim3(kScanBlock), 0, s, in,
                       n, scratch);
    hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(kScanBlock), 0, s, scratch, nb, total);
    hipLaunchKernelGGL(k_scan_apply, dim3(static_cast<uint32_t>(nb)), dim3(kScanBlock), 0, s, in,
                       n, scratch, out_excl);
}

void launch_ba_gather(hipStream_t s, const uint8_t* bytes, const DevPage* pages,
                      const DevTile* tiles, int ntiles, const DevDict* dicts,
                      const uint64_t* entries, const uint64_t* row_codes,
                      const int64_t* tile_base, int64_t nrows_total, const int64_t* total,
                      int64_t capacity, int32_t* overflow, uint32_t* validity, int64_t* offsets,
                      uint8_t* chars, bool byte_gather) {
    (void)entries;
    if (ntiles <= 0) return;
    int blocks = (ntiles + kWavesPerBlock - 1) / kWavesPerBlock;
    hipLaunchKernelGGL(k_ba_gather, dim3(blocks), dim3(256), 0, s, bytes, pages, tiles, ntiles,
                       dicts, row_codes, tile_base, nrows_total, total, capacity, overflow,
                       validity, offsets, chars, byte_gather);
}

void launch_fixed(hipStream_t s, const uint8_t* bytes, const DevPage* pages, int npages,
                  const DevDict* dicts, const int32_t* dict_count, ColumnParams cp,
                  uint32_t* validity, uint8_t* values, DevErr* page_err, int32_t* err_any) {
    if (npages <= 0) return;
    int blocks = (npages + kWavesPerBlock - 1) / kWavesPerBlock;
    hipLaunchKernelGGL(k_fixed, dim3(blocks), dim3(256), 0, s, bytes, pages, npages, dicts,
                       dict_count, cp, validity, values, page_err, err_any);
}

}  // namespace pqk
