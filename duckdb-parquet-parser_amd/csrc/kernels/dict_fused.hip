// dict_fused.hip — fast path for BYTE_ARRAY column chunks (SURVEY §8a
// R-DICT-PAGE / R-DICT-EXPAND / R-PLAIN / R-LEVELS / R-RLE) on gfx950.
//
// k_dict_index   dictionary page -> entry table (column_reader.cpp:128-138,
//                249-253).  The u32 length chain is serial, so one workgroup
//                walks it speculatively.  First in 256-byte slices with a
//                parallel link (dict_index_fine below: C4 c6's 4096-entry
//                page 0.079 -> 0.020 ms); when that does not resolve, the
//                coarse slices: the page sits in LDS, each of 16
//                waves owns a 1/16 slice and each of its lanes walks the chain
//                from one of the slice's first 64 byte offsets.  One thread
//                then links the slices (the true chain enters slice w at the
//                exit of slice w-1: pick that lane's result), and the chosen
//                lanes re-walk to write (len << 32 | pos) per entry.  Slices
//                whose entry point is not covered (an entry longer than 64
//                bytes, a malformed chain) fall back to a serial walk, which
//                also produces the exact reference error text.
// k_ba_fused     one launch per column chunk; persistent workgroups, one page
//                per wavefront at a time (ticket queue, pages in file order):
//                  1 page payload -> LDS (16-byte loads, issued first and
//                    landed after the level walk)
//                  2 def-level and index streams: run headers on the scalar
//                    unit (stream.hpp, SMEM), RLE runs expanded at once,
//                    bit-packed runs expanded lane-parallel from LDS
//                  3 per-row (source, length) + page-local prefix sum
//                  4 decoupled look-back over page totals -> the page's
//                    first output byte (no separate scan pass)
//                  5 int64 offsets, validity words, and the characters as
//                    16-byte aligned, fully coalesced stores assembled from
//                    the dictionary (or the page) held in LDS.
// The chunk's dictionary sits in LDS once per workgroup.
#include "kernels/device_common.hpp"
#include "kernels/dict_index.hpp"
#include "kernels/kernels.hpp"
#include "kernels/hybrid.hpp"
#include "kernels/stream.hpp"
#include "pq_gpu.h"

namespace pqk {
namespace {

using namespace dev;

constexpr uint64_t kAgg = 1ull << 62;
constexpr uint64_t kInc = 2ull << 62;
constexpr uint64_t kValMask = (1ull << 62) - 1;
constexpr uint32_t kGatherWin = 512;  // 16-byte blocks per gather window
constexpr uint32_t kLitCap = 16;      // recorded bit-packed runs per wave between expansions (serial walk)
constexpr uint32_t kRingBytes = 2048;  // writer's character ring (power of two, >= 2 * kGatherWin)
constexpr uint32_t kRingMaxRow = kRingBytes / 2 - 32;  // longer rows take the gather fallback

// ── dictionary entry table (dict_index.hpp) ─────────────────────────────────
constexpr int kDictWaves = 16;

__global__ void __launch_bounds__(kDictWaves * 64) k_dict_index(const uint8_t* __restrict__ bytes,
                                                                const DevDict* __restrict__ dicts,
                                                                uint64_t* __restrict__ entries,
                                                                int32_t* __restrict__ dict_count,
                                                                DevErr* __restrict__ dict_err,
                                                                int32_t* __restrict__ err_any,
                                                                uint32_t lds_cap) {
    extern __shared__ __attribute__((aligned(16))) uint32_t words[];
    dict_index_block<kDictWaves>(bytes, dicts, static_cast<int>(blockIdx.x), entries, dict_count, dict_err, err_any,
                                 lds_cap, words);
}

// ── dictionary pages larger than LDS (k_dict_index's serial walk) ───────────
// The fine-slice scheme of dict_index_fine over HBM, as two launches:
//   k_dict_slices  one wave per kLSlices 256-byte slices, staged in LDS with
//                  the slice before them: per slice the first kPCandD
//                  plausible entry starts among its first 64 bytes and the
//                  chain from each to the slice end; each slice is entered at
//                  the previous slice's exit (the exit of its first
//                  continuing candidate; slice 0 at 0) and must hold a
//                  candidate there leaving where it advertised.  Per slice
//                  (count | ok | chain error) and its entry; per wave the
//                  count sum and whether all its slices linked;
//   k_dict_fill    kFSlices slices per workgroup: every workgroup sums the
//                  wave words (all linked? entries before it?), stages its
//                  slices in LDS and re-walks the chosen chains writing
//                  (len << 32 | pos) entries.  Anything uncertain (a failed
//                  link, a bounds error in the last chain short of the
//                  count) is the serial walk of workgroup 0, which gives the
//                  reference's exact error (column_reader.cpp:128-138).
// scratch: slice words [nsl], slice entries [nsl], wave words [ceil(nsl / kLSlices)]
constexpr uint32_t kLSlices = 15;   // new slices per wave in k_dict_slices
constexpr uint32_t kFSlices = 240;  // slices per workgroup in k_dict_fill (16 k_dict_slices waves)

__global__ void __launch_bounds__(256) k_dict_slices(const uint8_t* __restrict__ page, uint32_t size, uint32_t nsl,
                                                     uint32_t* __restrict__ scr) {
    __shared__ uint32_t stw[4][(16 * kDSlice + 16) / 4 + 2];
    const uint32_t w = threadIdx.x / kWave, l = lane();
    const uint32_t wv = blockIdx.x * 4 + w;
    const uint32_t s0 = wv * kLSlices;  // first slice of this wave; slot j holds slice s0 - 1 + j
    if (s0 >= nsl) return;
    const uint32_t j0 = s0 == 0 ? 1u : 0u;   // wave 0 has no slice before its own
    const uint32_t base = (s0 - 1 + j0) * kDSlice;  // a multiple of 256: the page is 16-byte aligned in the image
    uint32_t* words = stw[w];
    {
        const uint32_t nb = min((16 - j0) * kDSlice + 16, (size - base + 15) / 16 * 16 + 16) / 16;
        const uint4* src = reinterpret_cast<const uint4*>(page + base);
        for (uint32_t i = l; i < nb; i += kWave) reinterpret_cast<uint4*>(words)[i] = src[i];
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint32_t jm = l / kPCandD, sl = l % kPCandD;
    uint64_t mk = 0;
#pragma unroll
    for (uint32_t j = 0; j < 16; j++) {
        const uint32_t sc = s0 - 1 + j, cs = sc * kDSlice;
        const bool sv = j >= j0 && sc < nsl;
        const uint32_t q = cs + l, ce = min(cs + kDSlice, size);
        bool plaus = sv && q < ce && q + 4 <= size &&
                     static_cast<uint64_t>(q) + 4 + lds_u32(words, min(q, size) - base) <= size;
        if (sv && sc == 0) plaus = l == 0;
        const uint64_t m = __ballot(plaus);
        if (j == jm) mk = m;
    }
    for (uint32_t i = 0; i < sl; i++) mk &= mk - 1;
    const uint32_t sc = s0 - 1 + jm;
    const bool sv = jm >= j0 && sc < nsl;
    uint32_t rx = kDNone, ry = kDNone;  // exit, count | entry << 8 | error << 31
    if (sv && mk) {
        const uint32_t cs = sc * kDSlice, ce = min(cs + kDSlice, size);
        const uint32_t e = static_cast<uint32_t>(__builtin_ctzll(mk));
        uint32_t q = cs + e, cnt = 0, bad = 0;
        while (q < ce) {
            if (q + 4 > size) { bad = 1; break; }
            const uint32_t len = lds_u32(words, q - base);
            if (static_cast<uint64_t>(q) + 4 + len > size) { bad = 1; break; }
            q += 4 + len;
            cnt++;
        }
        rx = q;
        ry = cnt | (e << 8) | (bad << 31);
    }
    // the slot's four candidates (every lane of the slot holds them all)
    uint32_t cx[kPCandD], cy[kPCandD];
#pragma unroll
    for (uint32_t k = 0; k < kPCandD; k++) {
        cx[k] = __shfl(rx, static_cast<int>(jm * kPCandD + k));
        cy[k] = __shfl(ry, static_cast<int>(jm * kPCandD + k));
    }
    // the slot's advertised exit: its first continuing candidate
    const uint32_t se = (sc + 1) * kDSlice;
    uint32_t cexit = kDNone;
#pragma unroll
    for (int k = static_cast<int>(kPCandD) - 1; k >= 0; k--)
        if (cx[k] != kDNone && !(cy[k] >> 31) && cx[k] >= se && cx[k] < se + 64) cexit = cx[k];
    const uint32_t prev = __shfl(cexit, static_cast<int>((jm == 0 ? 0u : jm - 1) * kPCandD));
    const uint32_t e = sc == 0 ? 0u : prev;
    uint32_t px = kDNone, py = kDNone;
#pragma unroll
    for (uint32_t k = 0; k < kPCandD; k++)
        if (cx[k] != kDNone && sc * kDSlice + ((cy[k] >> 8) & 0x3Fu) == e) { px = cx[k]; py = cy[k]; }
    const bool mine = jm >= 1 && sv;  // this wave's own slices
    const bool lastc = sc + 1 == nsl;
    const bool ok = px != kDNone && (lastc || (!(py >> 31) && px == cexit));
    const uint32_t c = (mine && sl == 0 && ok) ? (py & 0xFFu) : 0u;
    if (mine && sl == 0) {
        scr[sc] = c | ((py >> 31) << 30) | (ok ? 0x80000000u : 0u);
        scr[nsl + sc] = e;
    }
    const uint32_t tot = __shfl(wave_incl_scan(c), kWave - 1);
    const bool wok = __ballot(mine && sl == 0 && !ok) == 0;
    if (l == 0) scr[2 * nsl + wv] = tot | (wok ? 0x80000000u : 0u);
}

__global__ void __launch_bounds__(256) k_dict_fill(const uint8_t* __restrict__ page, uint32_t size, uint32_t n,
                                                   uint32_t nsl, const uint32_t* __restrict__ scr,
                                                   uint64_t* __restrict__ out, uint8_t* __restrict__ lens8,
                                                   uint4* __restrict__ pad16, int32_t* __restrict__ count,
                                                   DevErr* __restrict__ err, int32_t* __restrict__ err_any) {
    __shared__ __attribute__((aligned(16))) uint32_t words[(kFSlices * kDSlice + 48) / 4];
    __shared__ uint32_t red[3][4];
    __shared__ uint32_t wsum[4];
    const uint32_t t0 = threadIdx.x, w = t0 / kWave, l = lane();
    const uint32_t nwv = (nsl + kLSlices - 1) / kLSlices;
    const uint32_t wb = blockIdx.x * (kFSlices / kLSlices);  // first k_dict_slices wave of this workgroup
    uint32_t tot = 0, bef = 0, bad = 0;
    for (uint32_t v = t0; v < nwv; v += blockDim.x) {
        const uint32_t x = scr[2 * nsl + v];
        tot += x & 0x7FFFFFFFu;
        bef += v < wb ? (x & 0x7FFFFFFFu) : 0u;
        bad |= (x >> 31) ^ 1u;
    }
    tot = __shfl(wave_incl_scan(tot), kWave - 1);
    bef = __shfl(wave_incl_scan(bef), kWave - 1);
    bad = __ballot(bad != 0) != 0;
    if (l == 0) { red[0][w] = tot; red[1][w] = bef; red[2][w] = bad; }
    __syncthreads();
    tot = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    bef = red[1][0] + red[1][1] + red[1][2] + red[1][3];
    bad = red[2][0] | red[2][1] | red[2][2] | red[2][3];
    const bool last_bad = nsl > 0 && ((scr[nsl - 1] >> 30) & 1u);
    const bool fine = n > 0 && size > 0 && nsl > 0 && !bad && !(tot < n && last_bad);
    if (!fine) {
        // serial walk (workgroup 0, wave 0, scalar loads): the reference's order and errors
        if (blockIdx.x != 0 || w != 0) return;
        uint32_t pos = 0, k = 0;
        for (; k < n; k++) {
            if (static_cast<uint64_t>(pos) + 4 > size) { set_err(err, err_any, PQ_ERR_BUFFER, pos, 4, size); break; }
            const uint32_t len = suni(sload_u32(page, pos));
            pos += 4;
            if (static_cast<uint64_t>(pos) + len > size) { set_err(err, err_any, PQ_ERR_BUFFER, pos, len, size); break; }
            if (l == 0) {
                out[k] = entry_code(len, pos);
                if (lens8) lens8[k] = static_cast<uint8_t>(min(len, 255u));
                if (pad16) pad16[k] = make_uint4(0u, 0u, 0u, 0xFF000000u);  // (the entry word's path)
            }
            pos += len;
        }
        if (l == 0) *count = static_cast<int32_t>(k);
        return;
    }
    if (blockIdx.x == 0 && w == 0) {
        // the chain reached the page end with entries still declared
        if (tot < n) set_err(err, err_any, PQ_ERR_BUFFER, size, 4, size);
        if (l == 0) *count = static_cast<int32_t>(min(tot, n));
    }
    const uint32_t base = blockIdx.x * kFSlices * kDSlice;
    {
        // (+ 32: the characters of an entry starting at the last slice's end)
        const uint32_t nb = min(kFSlices * kDSlice + 32, (size - base + 15) / 16 * 16 + 16) / 16;
        const uint4* src = reinterpret_cast<const uint4*>(page + base);
        for (uint32_t i = t0; i < nb; i += blockDim.x) reinterpret_cast<uint4*>(words)[i] = src[i];
    }
    const uint32_t t = blockIdx.x * kFSlices + t0;
    const bool has = t0 < kFSlices && t < nsl;
    const uint32_t c = has ? (scr[t] & 0xFFu) : 0u;
    uint32_t q = has ? scr[nsl + t] : 0u;
    const uint32_t inc = wave_incl_scan(c);
    if (l == kWave - 1) wsum[w] = inc;
    __syncthreads();
    uint32_t before = bef + inc - c;
    for (uint32_t v = 0; v < w; v++) before += wsum[v];
    if (!has || before >= n) return;
    const uint32_t m = min(c, n - before);
    for (uint32_t k = 0; k < m; k++) {
        const uint32_t len = lds_u32(words, q - base);
        out[before + k] = entry_code(len, q + 4);
        if (lens8) lens8[before + k] = static_cast<uint8_t>(min(len, 255u));
        if (pad16) {  // characters 0..14 and the length in byte 15 (0xFF: 16 or more, the entry word's path)
            uint4 v = make_uint4(0u, 0u, 0u, 0xFF000000u);
            if (len <= 15) {
                const uint32_t a = q + 4 - base, wi = a >> 2, sh = a & 3;
                const uint32_t w0 = words[wi], w1 = words[wi + 1], w2 = words[wi + 2], w3 = words[wi + 3],
                               w4 = words[wi + 4];
                v.x = __builtin_amdgcn_alignbyte(w1, w0, sh);
                v.y = __builtin_amdgcn_alignbyte(w2, w1, sh);
                v.z = __builtin_amdgcn_alignbyte(w3, w2, sh);
                v.w = (__builtin_amdgcn_alignbyte(w4, w3, sh) & 0x00FFFFFFu) | (len << 24);
            }
            pad16[before + k] = v;
        }
        q += 4 + len;
    }
}

// ── fused page decode + gather ──────────────────────────────────────────────
//
// On gfx9 vector loads and stores share one counter (vmcnt), so a wave that
// both loads and stores waits for its own earlier stores whenever it needs a
// load result.  A workgroup is therefore split into producer/writer pairs:
//   producer  tickets, page payload -> LDS, level/index decode, per-row
//             (source, length) and page-local offsets, look-back.  Its only
//             global stores are the look-back status words.
//   writer    int64 offsets, validity words and characters: LDS -> HBM
//             stores only; it never waits on memory.
// Each producer hands pages to its writer through two LDS slots.
struct FusedArgs {
    const uint8_t* bytes;
    const DevPage* pages;
    int32_t p0, np;              // this chunk's data pages
    const DevDict* dicts;
    int32_t dict_id;             // dictionary in force for DICT pages (or -1)
    const uint64_t* entries;
    const int32_t* dict_count;
    int32_t max_def, max_rep;
    uint32_t rows_cap;           // max rows of a page (multiple of 64)
    uint32_t stage_bytes;        // max payload bytes (multiple of 16, + 16)
    uint32_t pair_bytes;         // LDS bytes per producer/writer pair
    uint32_t dict_bytes;         // LDS bytes of the dictionary region
    uint32_t dict_chars_bytes;   // payload bytes region (multiple of 16)
    uint64_t* status;            // np look-back words (zeroed)
    int32_t* ticket;             // zeroed
    const int64_t* base_in;      // characters before this chunk
    int64_t* base_out;           // characters through this chunk
    int64_t nrows_total;
    uint32_t* validity;
    int64_t* offsets;
    uint8_t* chars;
    int64_t capacity;
    int32_t* overflow;
    DevErr* page_err;
    int32_t* err_any;
    int32_t debug;               // ablation switches (timing only; output invalid)
    uint64_t* prof;              // per-phase cycle sums (kProfSlots), or null
    int32_t claim;               // pages claimed per ticket (one atomic per claim)
};

enum {
    PH_STAGE = 0, PH_DEF, PH_LEVELS, PH_VALUES, PH_ROWS, PH_LOOKBACK, PH_SLOTWAIT, PH_PAGES,
    PH_W_WAIT, PH_W_OFFSETS, PH_W_GATHER, PH_W_PAGES, PH_HA, PH_HB, PH_HC, PH_HD, kProfSlots
};

enum : uint32_t { SLOT_FREE = 0, SLOT_FULL = 1, SLOT_DONE = 2 };

struct SlotMeta {
    int64_t G0;        // first output byte of the page
    int64_t first_row;
    uint32_t n;        // rows
    uint32_t total;    // characters
    uint32_t dict;     // characters come from the dictionary (else the page)
    uint32_t maxlen;   // longest row
    uint32_t state;    // SLOT_*
    uint32_t pad;
};

struct Slot {
    SlotMeta* meta;
    uint32_t* stage;   // page payload
    uint32_t* off;     // rows_cap + 1: page-local char offsets
    uint16_t* rsrc;    // rows_cap: source byte of each row
    uint64_t* vm;      // rows_cap / 64: validity ballots
};

struct ProdMem {
    uint8_t* lv;       // rows_cap: def levels
    uint16_t* ix;      // rows_cap: dict index / plain chars position per rank
    LitRun* lits;      // kLitCap (serial walk)
    HybScratch hyb;    // decode scratch ...
    uint16_t* il;      // ... reused: rows_cap plain lengths per rank
};

// LDS layout of one producer/writer pair (shared by kernel and host).
struct PairLayout {
    uint32_t hyb_pos, hyb_runs;
    uint32_t p_lv, p_ix, p_lits, p_union, p_il, prod;          // producer scratch
    uint32_t s_meta, s_stage, s_off, s_rsrc, s_vm, slot;       // one slot
    uint32_t w_brow, writer;                                   // writer scratch
    uint32_t bytes;
};
__host__ __device__ inline uint32_t al16(uint32_t x) { return (x + 15u) & ~15u; }
__host__ __device__ inline PairLayout pair_layout(uint32_t rows_cap, uint32_t stage_bytes) {
    PairLayout L;
    L.hyb_pos = stage_bytes < kHybMaxPos ? stage_bytes : kHybMaxPos;
    L.hyb_runs = L.hyb_pos < rows_cap ? L.hyb_pos : rows_cap;
    uint32_t o = 0;
    L.p_lv = o; o += al16(rows_cap);
    L.p_ix = o; o += al16(2 * rows_cap);
    L.p_lits = o; o += al16(static_cast<uint32_t>(sizeof(LitRun)) * kLitCap);
    L.p_union = o;
    L.p_il = o;
    const uint32_t h = hyb_scratch_bytes(L.hyb_pos, L.hyb_runs), il = 2 * rows_cap;
    o += al16(h > il ? h : il);
    L.prod = o;
    o = 0;
    L.s_meta = o; o += al16(static_cast<uint32_t>(sizeof(SlotMeta)));
    L.s_stage = o; o += al16(stage_bytes);
    L.s_off = o; o += al16(4 * (rows_cap + 1));
    L.s_rsrc = o; o += al16(2 * rows_cap);
    L.s_vm = o; o += al16(8 * (rows_cap / 64 + 1));
    L.slot = o;
    L.w_brow = 0;  // gather fallback: block -> row map, aliases the ring
    L.writer = kRingBytes > 2 * kGatherWin ? kRingBytes : 2 * kGatherWin;
    L.bytes = L.prod + 2 * L.slot + L.writer;
    return L;
}

__device__ __forceinline__ Slot slot_at(uint8_t* base, const PairLayout& L) {
    Slot s;
    s.meta = reinterpret_cast<SlotMeta*>(base + L.s_meta);
    s.stage = reinterpret_cast<uint32_t*>(base + L.s_stage);
    s.off = reinterpret_cast<uint32_t*>(base + L.s_off);
    s.rsrc = reinterpret_cast<uint16_t*>(base + L.s_rsrc);
    s.vm = reinterpret_cast<uint64_t*>(base + L.s_vm);
    return s;
}

__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, kWave);
    return v;
}

// Decoupled look-back (status[t]: kAgg|aggregate or kInc|inclusive).
__device__ uint64_t look_back(uint64_t* status, int32_t t, uint64_t total) {
    if (t == 0) {
        if (lane() == 0) __hip_atomic_store(&status[0], kInc | total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return 0;
    }
    if (lane() == 0) __hip_atomic_store(&status[t], kAgg | total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint64_t prefix = 0;
    int32_t q = t - 1;
    uint32_t nap = 1;
    for (;;) {
        int32_t i = q - static_cast<int32_t>(lane());
        uint64_t s = i >= 0 ? __hip_atomic_load(&status[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kInc;
        uint64_t incm = __ballot((s >> 62) == 2);
        uint64_t notready = __ballot((s >> 62) == 0);
        uint32_t first_inc = incm ? static_cast<uint32_t>(__builtin_ctzll(incm)) : 64u;
        uint64_t upto = first_inc >= 63 ? ~0ull : ((2ull << first_inc) - 1ull);
        if (notready & upto) {
            for (uint32_t k = 0; k < nap; k++) __builtin_amdgcn_s_sleep(8);
            nap = nap < 8 ? 2 * nap : 8;
            continue;
        }
        uint64_t c = lane() <= first_inc ? (s & kValMask) : 0ull;
        prefix += wave_sum64(c);
        if (first_inc < 64) break;
        q -= 64;
    }
    if (lane() == 0)
        __hip_atomic_store(&status[t], kInc | (prefix + total), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return prefix;
}

__device__ __forceinline__ uint64_t clk() { return __builtin_amdgcn_s_memtime(); }

// LDS hand-off flag.  A wave's LDS operations execute in issue order, so a
// flag written after the data is seen after the data; the asm barriers keep
// the compiler from moving LDS accesses across the flag.
__device__ __forceinline__ uint32_t flag_get(const SlotMeta* m) {
    __asm__ __volatile__("" ::: "memory");
    uint32_t v = __hip_atomic_load(&m->state, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __asm__ __volatile__("" ::: "memory");
    return __builtin_amdgcn_readfirstlane(v);
}
__device__ __forceinline__ void flag_set(SlotMeta* m, uint32_t v) {
    __asm__ __volatile__("" ::: "memory");
    if (lane() == 0) __hip_atomic_store(&m->state, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __asm__ __volatile__("" ::: "memory");
}
__device__ __forceinline__ void flag_wait(const SlotMeta* m, bool want_free) {
    for (;;) {
        const uint32_t v = flag_get(m);
        if (want_free ? v == SLOT_FREE : v != SLOT_FREE) return;
        __builtin_amdgcn_s_sleep(2);
    }
}

template <bool kProf>
struct Prof {
    uint64_t ph[kProfSlots];
    uint64_t tk;
    __device__ void start() {
        if (kProf) {
            for (int i = 0; i < kProfSlots; i++) ph[i] = 0;
            tk = clk();
        }
    }
    __device__ void mark(int slot) {
        if (kProf) {
            uint64_t now = clk();
            ph[slot] += now - tk;
            tk = now;
        }
    }
    __device__ void count(int slot) {
        if (kProf) ph[slot]++;
    }
    __device__ void flush(uint64_t* out) {
        if (kProf && lane() == 0)
            for (int i = 0; i < kProfSlots; i++)
                if (ph[i]) atomicAdd(reinterpret_cast<unsigned long long*>(&out[i]), ph[i]);
    }
};

// ── producer: one page per iteration ────────────────────────────────────────
template <bool kProf>
__device__ void produce(const FusedArgs& a, const PairLayout& L, uint8_t* pair, const uint32_t* dtab,
                        uint32_t dict_n) {
    ProdMem M;
    M.lv = pair + L.p_lv;
    M.ix = reinterpret_cast<uint16_t*>(pair + L.p_ix);
    M.lits = reinterpret_cast<LitRun*>(pair + L.p_lits);
    M.hyb = hyb_carve(pair + L.p_union, L.hyb_pos, L.hyb_runs);
    M.il = reinterpret_cast<uint16_t*>(pair + L.p_il);
    uint8_t* slots = pair + L.prod;
    const uint32_t bw_def = level_bw(a.max_def);
    Prof<kProf> P;
    P.start();
    uint32_t si = 0;
    // Same-address atomics serialise chip-wide, so a producer claims `claim`
    // consecutive pages per ticket; it still processes pages in ticket order,
    // which keeps the look-back deadlock-free.
    int32_t tnext = 0, tend = 0;
    // debug bit 64 (with bit 1, no look-back): static page assignment, to
    // time the ticket atomics
    const bool stat = kProbes && (a.debug & 65) == 65;
    const int32_t nprod = static_cast<int32_t>(gridDim.x * (blockDim.x / (2 * kWave)));
    int32_t sp = static_cast<int32_t>(blockIdx.x * (blockDim.x / (2 * kWave)) + threadIdx.x / kWave);
    for (;;) {
        if (stat) {
            tnext = sp;
            tend = sp + 1;
            sp += nprod;
        } else if (tnext == tend) {
            int32_t c = 0;
            if (lane() == 0) c = atomicAdd(a.ticket, a.claim);
            tnext = static_cast<int32_t>(suni(static_cast<uint32_t>(c)));
            tend = tnext + a.claim;
        }
        const int32_t t = tnext++;
        Slot S = slot_at(slots + si * L.slot, L);
        flag_wait(S.meta, true);
        P.mark(PH_SLOTWAIT);
        if (t >= a.np) {
            flag_set(S.meta, SLOT_DONE);
            break;
        }
        P.count(PH_PAGES);
        const int32_t p = a.p0 + t;
        const DevPage pg = a.pages[p];
        const uint8_t* page = a.bytes + pg.off;
        const uint32_t size = static_cast<uint32_t>(pg.size);
        const uint32_t n = static_cast<uint32_t>(pg.nvals);
        // 1. payload -> LDS (slots are 16-byte aligned with >= 16 bytes of
        //    zero padding, so the extra block stays inside the image)
        {
            const uint4* gsrc = reinterpret_cast<const uint4*>(page);
            uint4* sdst = reinterpret_cast<uint4*>(S.stage);
            const uint32_t n16 = (size + 15) / 16 + 1;
            for (uint32_t i = lane(); i < n16; i += kWave) sdst[i] = gsrc[i];
        }
        __builtin_amdgcn_wave_barrier();
        P.mark(PH_STAGE);
        const uint32_t* pw = S.stage;
        int code = 0;
        uint32_t epos = 0, eneed = 0, nl = 0;
        // 2. levels (column_reader.cpp:146-170)
        uint32_t pos = 0, def_base = 0, dl = 0;
        if (a.max_def > 0) {
            if (pos + 4 > size) { code = PQ_ERR_BUFFER; epos = pos; eneed = 4; }
            else {
                dl = suni(lds_u32(pw, pos));
                pos += 4;
                if (static_cast<uint64_t>(pos) + dl > size) { code = PQ_ERR_BUFFER; epos = pos; eneed = dl; }
                else { def_base = pos; pos += dl; }
            }
        }
        if (!code && a.max_rep > 0) {
            if (pos + 4 > size) { code = PQ_ERR_BUFFER; epos = pos; eneed = 4; }
            else {
                uint32_t rl2 = suni(lds_u32(pw, pos));
                pos += 4;
                if (static_cast<uint64_t>(pos) + rl2 > size) { code = PQ_ERR_BUFFER; epos = pos; eneed = rl2; }
                else pos += rl2;
            }
        }
        // def levels (stream 0), then dictionary indices (stream 1): one loop
        // so the decoder is instantiated once
        const bool dict = pg.mode == MODE_DICT;
        uint32_t nn = 0;
        uint32_t sbase = def_base, slen = dl, sbw = bw_def, scount = n;
        bool run_stream = !code && a.max_def > 0;
        if (!code && a.max_def == 0)
            for (uint32_t j = lane(); j < n; j += kWave) M.lv[j] = 0;
#pragma nounroll
        for (uint32_t st = 0; st < 2; st++) {
            if (run_stream) {
                auto put = [&](uint32_t j, uint32_t v) {
                    if (st == 0) M.lv[j] = static_cast<uint8_t>(v > 255 ? 255 : v);
                    else M.ix[j] = static_cast<uint16_t>(static_cast<int32_t>(v) >= 0 && v < dict_n ? v : 0xFFFFu);
                };
                auto hm = [&](int ph) { P.mark(PH_HA + ph); };
                if (hyb_decode(pw, size, sbase, slen, sbw, scount, M.hyb, L.hyb_runs, M.ix, put, hm)) {
                    SRle r;
                    srle_init(r, sbase, slen, sbw);
                    code = srle_walk(r, page, scount, put, M.lits, nl, kLitCap,
                                     [&]() { expand_lits(M.lits, nl, pw, size, sbw, put); });
                    if (!code) expand_lits(M.lits, nl, pw, size, sbw, put);
                    nl = 0;
                }
                __builtin_amdgcn_wave_barrier();
            }
            if (st == 1 || code) break;
            P.mark(PH_DEF);
            uint32_t above = 0;
            for (uint32_t j0 = 0; j0 < n; j0 += kWave) {
                uint32_t j = j0 + lane();
                uint32_t d = j < n ? M.lv[j] : 0u;
                bool isnn = j < n && (dict ? d == static_cast<uint32_t>(a.max_def) : d >= static_cast<uint32_t>(a.max_def));
                nn += __popcll(__ballot(isnn));
                above |= __ballot(j < n && d > static_cast<uint32_t>(a.max_def)) != 0;
            }
            if (dict && above) code = PQ_ERR_UNSUPPORTED;
            P.mark(PH_LEVELS);
            run_stream = false;
            if (!code && dict) {  // column_reader.cpp:196-214
                if (pos + 1 > size) { code = PQ_ERR_BUFFER; epos = pos; eneed = 1; }
                else {
                    sbw = suni(lds_u32(pw, pos) & 0xFFu);
                    pos += 1;
                    sbase = pos;
                    slen = size - pos;
                    scount = nn;
                    run_stream = true;
                }
            }
        }
        if (!code && !dict) {
            for (uint32_t k = 0; k < nn; k++) {  // column_reader.cpp:249-253
                if (static_cast<uint64_t>(pos) + 4 > size) { code = PQ_ERR_BUFFER; epos = pos; eneed = 4; break; }
                uint32_t len = suni(lds_u32(pw, pos));
                pos += 4;
                if (static_cast<uint64_t>(pos) + len > size) { code = PQ_ERR_BUFFER; epos = pos; eneed = len; break; }
                if (lane() == 0) { M.ix[k] = static_cast<uint16_t>(pos); M.il[k] = static_cast<uint16_t>(len); }
                pos += len;
            }
        }
        __builtin_amdgcn_wave_barrier();
        P.mark(PH_VALUES);
        // 3. per-row source/length, page-local offsets, validity ballots
        uint64_t total = 0;
        uint32_t maxlen = 0;
        if (!code) {
            uint32_t rank = 0, run = 0;
            for (uint32_t j0 = 0; j0 < n; j0 += kWave) {
                uint32_t j = j0 + lane();
                bool in = j < n;
                uint32_t d = in ? M.lv[j] : 0u;
                bool isnn = in && (dict ? d == static_cast<uint32_t>(a.max_def) : d >= static_cast<uint32_t>(a.max_def));
                uint64_t mask = __ballot(isnn);
                uint32_t k = rank + popc_below(mask);
                rank += __popcll(mask);
                uint32_t len = 0, src = 0;
                bool valid = false;
                if (isnn) {
                    if (dict) {
                        uint32_t idx = M.ix[k];
                        if (idx != 0xFFFFu) {
                            uint32_t e = dtab[idx];
                            src = e & 0xFFFFu;
                            len = e >> 16;
                            valid = true;
                        }
                    } else {
                        src = M.ix[k];
                        len = M.il[k];
                        valid = true;
                    }
                }
                uint32_t inc = wave_incl_scan(len);
                maxlen = max(maxlen, len);
                if (in) {
                    S.off[j] = run + inc - len;
                    S.rsrc[j] = static_cast<uint16_t>(src);
                }
                run += bcast_last(inc);
                const uint64_t vm = __ballot(valid);
                if (lane() == 0) S.vm[j0 / kWave] = vm;
            }
            if (lane() == 0) S.off[n] = run;
            total = run;
        } else {
            if (lane() == 0) {
                DevErr* err = a.page_err + p;
                err->code = code;
                err->pos = static_cast<int32_t>(epos);
                err->need = static_cast<int32_t>(eneed);
                err->size = static_cast<int32_t>(size);
                atomicOr(a.err_any, 1);
            }
        }
        __builtin_amdgcn_wave_barrier();
        P.mark(PH_ROWS);
        // 4. page start in the output
        const int64_t G0 = probe(a.debug, 1) ? static_cast<int64_t>(t) * 24 * n
                                         : *a.base_in + static_cast<int64_t>(look_back(a.status, t, total));
        if (t == a.np - 1 && lane() == 0) {
            *a.base_out = G0 + static_cast<int64_t>(total);
            if (pg.first_row + n == a.nrows_total) a.offsets[a.nrows_total] = G0 + total;
        }
        P.mark(PH_LOOKBACK);
        if (lane() == 0) {
            S.meta->G0 = G0;
            S.meta->first_row = pg.first_row;
            S.meta->n = code ? 0u : n;
            S.meta->total = static_cast<uint32_t>(total);
            S.meta->dict = dict;
        }
        {
            const uint32_t ml = wave_incl_max(maxlen);
            if (lane() == kWave - 1) S.meta->maxlen = ml;
        }
        flag_set(S.meta, SLOT_FULL);
        si ^= 1;
    }
    P.flush(a.prof);
}

// Store the bytes [lo, hi) of one 16-byte block (global byte blk) held in
// `v`: a whole block as one 16-byte store, a partial one byte by byte (the
// rest of that block belongs to the neighbouring page).
__device__ __forceinline__ void store_block(uint8_t* chars, int64_t blk, uint32_t lo, uint32_t hi, uint4 v) {
    if (lo == 0 && hi == 16) {
        *reinterpret_cast<uint4*>(chars + blk) = v;
    } else {
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
        for (uint32_t bb = lo; bb < hi; bb++) chars[blk + bb] = static_cast<uint8_t>(w[bb >> 2] >> (8 * (bb & 3)));
    }
}

// Characters of one page, input-driven: one row per lane copies its bytes
// into an LDS ring indexed by global byte address (so ring blocks line up
// with 16-byte output blocks); completed blocks are streamed out and zeroed.
__device__ void copy_chars(const FusedArgs& a, const Slot& S, uint32_t* ring, const uint32_t* srcw,
                           uint32_t srcw_last, uint32_t n, int64_t G0, int64_t G1) {
    constexpr uint32_t kRingMask = kRingBytes / 4 - 1;  // in words
    int64_t fb = G0 >> 4;  // first block not yet stored
    uint32_t r0 = 0;
    while (r0 < n) {
        // rows [r0, r1): at most one per lane, ending within the ring's reach
        const uint32_t r = r0 + lane();
        const uint32_t e = r < n ? S.off[r + 1] : 0xFFFFFFFFu;
        const int64_t limit = fb * 16 + kRingBytes - 16;
        const uint64_t fit = __ballot(r < n && G0 + static_cast<int64_t>(e) <= limit);
        const uint32_t k = fit == ~0ull ? kWave : static_cast<uint32_t>(__builtin_ctzll(~fit));
        const uint32_t cnt = k ? k : 1u;  // a row longer than the ring never reaches here
        if (lane() < cnt) {
            // destination dwords [d >> 2, (d + L - 1) >> 2]; all source dwords
            // of a 64-byte segment are read before any is written, so a row
            // costs one LDS round trip per segment
            const uint32_t s0 = S.off[r];
            const uint32_t L = e - s0;
            const uint32_t src = S.rsrc[r];
            const int64_t d = G0 + s0;
            const uint32_t lo0 = static_cast<uint32_t>(d & 3);
            const uint32_t nd = (lo0 + L + 3) >> 2;
            const uint32_t a0 = src - lo0;  // >= 1: every value follows a 4-byte length prefix
            const uint32_t sh = a0 & 3, i0 = a0 >> 2;
            const uint32_t lastb = (lo0 + L - 1) & 3;
            const uint32_t dw0 = static_cast<uint32_t>(d >> 2);
            for (uint32_t j0 = 0; j0 < nd && L; j0 += 16) {
                uint32_t x[17];
#pragma unroll
                for (uint32_t k = 0; k < 17; k++) x[k] = srcw[min(i0 + j0 + k, srcw_last)];
#pragma unroll
                for (uint32_t k = 0; k < 16; k++) {
                    const uint32_t j = j0 + k;
                    uint32_t v = __builtin_amdgcn_alignbyte(x[k + 1], x[k], sh);
                    if (j == 0) v &= 0xFFFFFFFFu << (8 * lo0);
                    if (j == nd - 1) v &= 0xFFFFFFFFu >> (8 * (3 - lastb));
                    if (j < nd) atomicOr(&ring[(dw0 + j) & kRingMask], v);
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
        const uint32_t r1 = r0 + cnt;
        const int64_t end = G0 + static_cast<int64_t>(S.off[r1]);
        const int64_t lb = r1 >= n ? ((end + 15) >> 4) : (end >> 4);  // blocks [fb, lb) are complete
        for (int64_t b = fb + lane(); b < lb; b += kWave) {
            uint4* rb = reinterpret_cast<uint4*>(ring + ((static_cast<uint32_t>(b) * 4) & kRingMask));
            const uint4 v = *rb;
            *rb = make_uint4(0, 0, 0, 0);
            const int64_t blk = b << 4;
            const uint32_t lo = blk < G0 ? static_cast<uint32_t>(G0 - blk) : 0u;
            const uint32_t hi = blk + 16 > G1 ? static_cast<uint32_t>(G1 - blk) : 16u;
            if (!probe(a.debug, 16)) store_block(a.chars, blk, lo, hi, v);
        }
        __builtin_amdgcn_wave_barrier();
        fb = lb;
        r0 = r1;
    }
}

// Output-driven fallback for pages with rows longer than the ring allows:
// each lane assembles one 16-byte block from the rows that cover it.
__device__ void gather_chars(const FusedArgs& a, const Slot& S, uint32_t* ringw, const uint32_t* srcw, uint32_t n,
                             int64_t G0, int64_t G1) {
    uint16_t* brow = reinterpret_cast<uint16_t*>(ringw);
    const int64_t B0 = G0 >> 4;
    const int64_t nb = ((G1 - 1) >> 4) - B0 + 1;
    for (int64_t w0 = 0; w0 < nb; w0 += kGatherWin) {
        const int64_t w1 = min(nb, w0 + static_cast<int64_t>(kGatherWin));
        for (uint32_t r = lane(); r < n; r += kWave) {
            uint32_t s0 = S.off[r], e0 = S.off[r + 1];
            if (e0 <= s0) continue;
            int64_t blo = s0 == 0 ? 0 : ((s0 + G0 + 15) >> 4) - B0;
            int64_t bhi = ((e0 + G0 + 15) >> 4) - B0 - 1;
            blo = max(blo, w0);
            bhi = min(bhi, w1 - 1);
            for (int64_t b = blo; b <= bhi; b++) brow[b - w0] = static_cast<uint16_t>(r);
        }
        __builtin_amdgcn_wave_barrier();
        for (int64_t b = w0 + lane(); b < w1; b += kWave) {
            const int64_t blk = (B0 + b) << 4;
            const int64_t gs = max(blk, G0), ge = min(blk + 16, G1);
            uint32_t r = brow[b - w0];
            uint32_t q = static_cast<uint32_t>(gs - G0);  // page-local output byte
            uint32_t o = static_cast<uint32_t>(gs - blk);
            const uint32_t oe = static_cast<uint32_t>(ge - blk);
            uint32_t rend = S.off[r + 1];
            uint32_t out[4] = {0, 0, 0, 0};
#pragma unroll
            for (uint32_t k = 0; k < 4; k++) {
                uint32_t lo = max(4 * k, o), hi = min(4 * k + 4, oe);
                if (lo >= hi) continue;
                for (uint32_t bb = lo; bb < hi; bb++) {
                    uint32_t qb = q + (bb - o);
                    while (qb >= rend && r + 1 < n) { r++; rend = S.off[r + 1]; }
                    uint32_t sa = S.rsrc[r] + (qb - S.off[r]);
                    out[k] |= lds_u8(srcw, sa) << (8 * (bb & 3));
                }
            }
            store_block(a.chars, blk, o, oe, make_uint4(out[0], out[1], out[2], out[3]));
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// ── writer: offsets, validity and characters of the pages handed over ──────
template <bool kProf>
__device__ void write_pages(const FusedArgs& a, const PairLayout& L, uint8_t* pair, const uint32_t* dwords) {
    uint8_t* slots = pair + L.prod;
    uint32_t* ring = reinterpret_cast<uint32_t*>(pair + L.prod + 2 * L.slot + L.w_brow);
    for (uint32_t i = lane(); i < kRingBytes / 16; i += kWave)
        reinterpret_cast<uint4*>(ring)[i] = make_uint4(0, 0, 0, 0);
    __builtin_amdgcn_wave_barrier();
    Prof<kProf> P;
    P.start();
    uint32_t si = 0;
    for (;;) {
        Slot S = slot_at(slots + si * L.slot, L);
        flag_wait(S.meta, false);
        P.mark(PH_W_WAIT);
        if (flag_get(S.meta) == SLOT_DONE) break;
        P.count(PH_W_PAGES);
        const int64_t G0 = S.meta->G0;
        const int64_t first_row = S.meta->first_row;
        const uint32_t n = __builtin_amdgcn_readfirstlane(S.meta->n);
        const uint32_t total = __builtin_amdgcn_readfirstlane(S.meta->total);
        const bool dict = __builtin_amdgcn_readfirstlane(S.meta->dict) != 0;
        // offsets (two rows per lane and store)
        if (!probe(a.debug, 4)) {
            for (uint32_t j = 2 * lane(); j < n; j += 2 * kWave) {
                const int64_t o0 = G0 + S.off[j];
                if (j + 1 < n) {
                    const int64_t o1 = G0 + S.off[j + 1];
                    int64_t* dst = a.offsets + first_row + j;
                    if (((first_row + j) & 1) == 0) {
                        *reinterpret_cast<longlong2*>(dst) = make_longlong2(o0, o1);
                    } else {
                        dst[0] = o0;
                        dst[1] = o1;
                    }
                } else {
                    a.offsets[first_row + j] = o0;
                }
            }
        }
        // validity words covering rows [first_row, first_row + n)
        if (n) {
            const int64_t w0 = first_row >> 5, w1 = (first_row + n - 1) >> 5;
            for (int64_t w = w0 + lane(); w <= w1; w += kWave) {
                const int64_t wr = w * 32;  // first row of this word
                uint32_t bits = 0;
                // rows [max(wr, first_row), min(wr + 32, first_row + n))
                const int64_t lo = max(wr, first_row), hi = min(wr + 32, first_row + static_cast<int64_t>(n));
                const uint32_t r0 = static_cast<uint32_t>(lo - first_row);
                const uint32_t cnt = static_cast<uint32_t>(hi - lo);
                const uint64_t m0 = S.vm[r0 >> 6];
                const uint64_t m1 = ((r0 >> 6) + 1) * kWave < n ? S.vm[(r0 >> 6) + 1] : 0ull;
                const uint32_t sh = r0 & 63;
                uint64_t x = sh ? ((m0 >> sh) | (m1 << (64 - sh))) : m0;
                x &= cnt >= 32 ? 0xFFFFFFFFull : ((1ull << cnt) - 1ull);
                bits = static_cast<uint32_t>(x) << static_cast<uint32_t>(lo - wr);
                if (cnt == 32) a.validity[w] = bits;
                else if (bits) atomicOr(&a.validity[w], bits);
            }
        }
        P.mark(PH_W_OFFSETS);
        const int64_t G1 = G0 + static_cast<int64_t>(total);
        const uint32_t* srcw = dict ? dwords : S.stage;
        if (total && !probe(a.debug, 2) && G1 > a.capacity) {
            if (lane() == 0) atomicOr(a.overflow, 1);
        } else if (total && !probe(a.debug, 2) && __builtin_amdgcn_readfirstlane(S.meta->maxlen) <= kRingMaxRow) {
            copy_chars(a, S, ring, srcw, (dict ? a.dict_chars_bytes : a.stage_bytes) / 4 - 1, n, G0, G1);
        } else if (total && !probe(a.debug, 2)) {
            gather_chars(a, S, ring, srcw, n, G0, G1);
            for (uint32_t i = lane(); i < kRingBytes / 16; i += kWave)
                reinterpret_cast<uint4*>(ring)[i] = make_uint4(0, 0, 0, 0);
            __builtin_amdgcn_wave_barrier();
        }
        P.mark(PH_W_GATHER);
        flag_set(S.meta, SLOT_FREE);
        si ^= 1;
    }
    P.flush(a.prof);
}

template <bool kProf>
__global__ void __launch_bounds__(1024) k_ba_fused(FusedArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t wv = threadIdx.x / kWave;
    const uint32_t npairs = blockDim.x / (2 * kWave);
    const PairLayout L = pair_layout(a.rows_cap, a.stage_bytes);

    // dictionary -> LDS: raw payload words, then (pos | len << 16) per entry
    uint32_t* dwords = reinterpret_cast<uint32_t*>(smem);
    uint32_t* dtab = reinterpret_cast<uint32_t*>(smem + a.dict_chars_bytes);
    uint32_t dict_n = 0;
    if (a.dict_id >= 0) {
        const DevDict d = a.dicts[a.dict_id];
        dict_n = static_cast<uint32_t>(a.dict_count[a.dict_id]);
        const uint4* src = reinterpret_cast<const uint4*>(a.bytes + d.off);
        uint4* dst = reinterpret_cast<uint4*>(dwords);
        copy_blocks(dst, src, a.dict_chars_bytes / 16, threadIdx.x, blockDim.x);
        for (uint32_t k = threadIdx.x; k < dict_n; k += blockDim.x) {
            uint64_t e = a.entries[d.entry_base + k];
            dtab[k] = static_cast<uint32_t>(e & 0xFFFFu) | (static_cast<uint32_t>(e >> 32) << 16);
        }
    }
    const uint32_t pi = wv < npairs ? wv : wv - npairs;
    uint8_t* pair = smem + a.dict_bytes + pi * a.pair_bytes;
    if (wv < npairs && lane() == 0) {
        slot_at(pair + L.prod, L).meta->state = SLOT_FREE;
        slot_at(pair + L.prod + L.slot, L).meta->state = SLOT_FREE;
    }
    __syncthreads();
    if (wv < npairs) produce<kProf>(a, L, pair, dtab, dict_n);
    else write_pages<kProf>(a, L, pair, dwords);
}

}  // namespace

void launch_dict_index(hipStream_t s, const uint8_t* bytes, const DevDict* dicts, int ndicts,
                       uint64_t* entries, int32_t* dict_count, DevErr* dict_err, int32_t* err_any,
                       uint32_t max_dict_bytes) {
    if (ndicts <= 0) return;
    constexpr uint32_t kCap = kDictLdsCap;  // + 18.2 KiB static tables < 160 KiB
    ensure_dyn_lds(reinterpret_cast<const void*>(k_dict_index), kCap);
    uint32_t lds = std::min<uint32_t>(kCap, (max_dict_bytes + 15) / 16 * 16 + 32);
    hipLaunchKernelGGL(k_dict_index, dim3(ndicts), dim3(kDictWaves * kWave), lds, s, bytes, dicts, entries,
                       dict_count, dict_err, err_any, lds);
}

namespace {
void set_fused_attrs() {
    ensure_dyn_lds(reinterpret_cast<const void*>(k_ba_fused<false>), 160 * 1024);
    ensure_dyn_lds(reinterpret_cast<const void*>(k_ba_fused<true>), 160 * 1024);
}
}  // namespace

uint32_t dict_big_slices(uint32_t size) { return (size + kDSlice - 1) / kDSlice; }

uint32_t dict_big_scratch(uint32_t size) {
    const uint32_t nsl = dict_big_slices(size);
    return (2 * nsl + (nsl + kLSlices - 1) / kLSlices) * static_cast<uint32_t>(sizeof(uint32_t));
}

void launch_dict_big(hipStream_t s, const uint8_t* page, uint32_t size, uint32_t nvals, uint64_t* entries,
                     uint8_t* lens8, uint4* pad16, int32_t* count, DevErr* err, int32_t* err_any, uint32_t* scr) {
    const uint32_t nsl = dict_big_slices(size);
    const uint32_t nwv = (nsl + kLSlices - 1) / kLSlices;
    if (nwv) hipLaunchKernelGGL(k_dict_slices, dim3((nwv + 3) / 4), dim3(256), 0, s, page, size, nsl, scr);
    hipLaunchKernelGGL(k_dict_fill, dim3(std::max<uint32_t>(1, (nsl + kFSlices - 1) / kFSlices)), dim3(256), 0, s, page,
                       size, nvals, nsl, scr, entries, lens8, pad16, count, err, err_any);
}

int fused_occupancy_waves(uint32_t lds_bytes_per_block, int waves_per_block) {
    int blocks = 0;
    set_fused_attrs();
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, k_ba_fused<false>, waves_per_block * kWave,
                                                     lds_bytes_per_block) != hipSuccess)
        return 0;
    return blocks;
}

void launch_ba_fused(hipStream_t s, const FusedLaunch& L) {
    FusedArgs a;
    a.bytes = L.bytes; a.pages = L.pages; a.p0 = L.p0; a.np = L.np; a.dicts = L.dicts;
    a.dict_id = L.dict_id; a.entries = L.entries; a.dict_count = L.dict_count;
    a.max_def = L.max_def; a.max_rep = L.max_rep; a.rows_cap = L.rows_cap;
    a.stage_bytes = L.stage_bytes; a.pair_bytes = L.wave_bytes; a.dict_bytes = L.dict_bytes;
    a.dict_chars_bytes = L.dict_chars_bytes; a.status = L.status; a.ticket = L.ticket;
    a.base_in = L.base_in; a.base_out = L.base_out; a.nrows_total = L.nrows_total;
    a.validity = L.validity; a.offsets = L.offsets; a.chars = L.chars; a.capacity = L.capacity;
    a.overflow = L.overflow; a.page_err = L.page_err; a.err_any = L.err_any; a.debug = L.debug;
    a.prof = L.prof;
    a.claim = L.claim > 0 ? L.claim : 1;
    const uint32_t lds = L.dict_bytes + (L.waves_per_block / 2) * L.wave_bytes;
    set_fused_attrs();
    if (a.prof)
        hipLaunchKernelGGL(k_ba_fused<true>, dim3(L.grid), dim3(L.waves_per_block * kWave), lds, s, a);
    else
        hipLaunchKernelGGL(k_ba_fused<false>, dim3(L.grid), dim3(L.waves_per_block * kWave), lds, s, a);
}

// LDS bytes of one producer/writer pair (FusedLaunch::wave_bytes).
uint32_t fused_wave_bytes(uint32_t rows_cap, uint32_t stage_bytes) {
    return pair_layout(rows_cap, stage_bytes).bytes;
}

int fused_prof_slots() { return kProfSlots; }

}  // namespace pqk
