// capi_state.hpp — the C ABI's context and device-chunk state (pq_ctx,
// pq_chunk) and the planning functions that size a chunk's launches
// (host/plan.cpp), shared by capi.hip (entry points, uploads, launches).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <thread>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "host/format.hpp"
#include "kernels/kernels.hpp"
#include "pq_gpu.h"
#include "regex/regex.hpp"
#include "stage.hpp"

using pqk::DevDict;
using pqk::DevErr;
using pqk::DevPage;
using pqk::DevTile;

// host tables filled by index from several threads: no zero fill on resize
template <class T>
using HVec = std::vector<T, pqfmt::NoInitAlloc<T>>;

// ... and in pinned memory: the page and tile tables go to HBM by DMA
// straight from where the plan wrote them (no staging copy)
template <class T>
struct PinnedAlloc : pqfmt::NoInitAlloc<T> {
    using value_type = T;
    template <class U>
    struct rebind { using other = PinnedAlloc<U>; };
    PinnedAlloc() = default;
    template <class U>
    PinnedAlloc(const PinnedAlloc<U>&) noexcept {}
    T* allocate(size_t n) {
        void* p = nullptr;
        if (hipHostMalloc(&p, std::max<size_t>(n, 1) * sizeof(T), hipHostMallocDefault) != hipSuccess) throw std::bad_alloc();
        return static_cast<T*>(p);
    }
    void deallocate(T* p, size_t) noexcept { (void)hipHostFree(p); }
};
template <class A, class B>
bool operator==(const PinnedAlloc<A>&, const PinnedAlloc<B>&) { return true; }
template <class A, class B>
bool operator!=(const PinnedAlloc<A>&, const PinnedAlloc<B>&) { return false; }
template <class T>
using PVec = std::vector<T, PinnedAlloc<T>>;

struct PendingTimer {
    std::string name;
    hipEvent_t a, b;
};

struct pq_ctx {
    int device = 0;
    int cus = 256;                         // compute units (queried once: the property call costs ms)
    hipStream_t stream = nullptr;
    hipStream_t copy = nullptr;            // uploads (pinned staging), beside the decode stream
    hipStream_t copy2 = nullptr;           // second DMA queue of the upload ring (option "stage_streams")
    int opt_stage_streams = 2;
    pqstage::Stager stager;
    uint8_t* d_raw = nullptr;              // raw chunk bytes of the current upload (relayout source)
    size_t raw_cap = 0;
    bool opt_dev_walk = false;             // "device_walk": uploads walk pages on the GPU (walk.hip) over d_raw
    uint8_t* d_walk = nullptr;             // the device walk's records, links and page table
    size_t walk_cap = 0;
    pq_page_desc* h_walk = nullptr;        // pinned: the page table back to the host
    size_t h_walk_cap = 0;
    pqk::RelayoutEntry* d_relay = nullptr; // relayout entries of the current upload
    size_t relay_cap = 0;
    pqk::CodecEntry* d_codec = nullptr;    // compressed / V2 pages of the current upload (codec.hip)
    size_t codec_cap = 0;
    uint32_t* d_codec_st = nullptr;        // their status words
    uint8_t* d_zsrc = nullptr;             // their payloads, when not in d_raw
    size_t zsrc_cap = 0;
    uint8_t* d_chunker = nullptr;          // pq_chunk_assign scratch and (no caller buffer) output
    size_t chunker_cap = 0;
    bool opt_raw = true;                   // "raw_upload": DMA raw chunk bytes during the walk, relayout on the GPU
    hipStream_t side = nullptr;            // dictionary decode beside the run-table pass
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    std::string err;
    bool timing = false;
    std::vector<PendingTimer> pending;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> free_events;
    std::map<std::string, std::pair<double, int64_t>> timers;
    // upload scratch (upload_walked): per-page host tables, reused
    PVec<pqk::DevPage> s_hpages;
    HVec<std::pair<int64_t, int64_t>> s_copies;
    HVec<int32_t> s_copy_size;
    PVec<int32_t> s_tile0;
    PVec<pqk::DevTile> s_htiles;
    PVec<pqk::RelayoutEntry> s_ents;
    bool opt_fused = true;  // pq_ctx_set_option("fused_ba", 0) forces the generic path
    bool opt_pipe_wide = true;   // "pipe_wide": dictionaries beyond the writer's LDS / 65,535 entries on the pipe (k_pipe_wwide)
    bool opt_wide_rows = true;  // "wide_rows": generic BYTE_ARRAY rows by a workgroup per page (k_wide_rows)
    bool opt_levels_small = true;  // "levels_small": k_fixed_levels2 in its 35 KB LDS form (4 workgroups per CU)
    bool opt_gather_rows = true;  // "gather_rows": k_ba_gather copies characters row per lane (0: byte-wise blocks)
    int opt_debug = 0;      // "fused_debug": ablation switches for timing studies
    int opt_waves = 0;      // "fused_waves": waves per workgroup override (0 = auto)
    uint64_t* d_prof = nullptr;  // "fused_prof": per-phase cycle sums of k_ba_fused
    int opt_claim = 1;           // "fused_claim": pages claimed per ticket by k_ba_fused producers (>1 serialises the look-back; diagnostics)
    bool opt_regex_dfa = true;   // "regex_dfa": DFA kernels (else the NFA kernel)
    bool opt_regex_plain = true; // "regex_plain": windowed kernel for chunks without dictionary pages
    bool opt_regex_codes = true; // "regex_codes": dictionary chunks on the pipe path: match bits over the decode's codes
    bool opt_regex_reuse = true; // "regex_reuse": ... reusing the codes of an earlier checked decode of the chunk
    int opt_regex_index = 1;     // "regex_index": REQUIRED PLAIN chunks keep the string index of their first scan;
                                 // 2: every scan is a first scan (files the index again: the cold-scan timing)
    int opt_regex_win = 8192;    // "regex_win": window bytes of the windowed kernel
    int opt_regex_debug = 0;     // "regex_debug": timing ablation of the windowed kernel (output invalid)
    bool opt_fixed_plain = true; // "fixed_plain": tile-parallel PLAIN fixed-width kernels (fixed_fast.hip)
    bool opt_fixed_fused = false; // "fixed_fused": OPTIONAL ones scatter their values in the levels launch (slower: DESIGN §5)
    bool opt_pipe = true;        // "dict_pipe": three-pass dictionary BYTE_ARRAY kernels (dict_pipe.hip)
    bool opt_plain = true;       // "plain_ba": two-pass PLAIN BYTE_ARRAY kernels for REQUIRED chunks (plain_ba.hip)
    bool opt_plain_fused = true; // "plain_fused": their one-pass form when the pages' character counts are known
    bool opt_zflip = true;       // "zflip": per-decode flags from the block the previous k_pipe_write cleared (else a fill)
    int opt_write_waves = 10;    // "write_waves": k_pipe_write writer waves per workgroup (1..16), set before upload
    bool opt_big_all = false;    // "big_all": every page of a pipe chunk takes k_pipe_big (set before upload)
    int opt_run_pages = 32;      // "pipe_run_pages": pages per wavefront of the run-table pass (1..32)
    bool opt_run_dict = true;    // "pipe_run_dict": the dictionary decodes in k_pipe_runs' leading workgroups
    int opt_write_bpc = 0;       // "write_bpc": cap on k_pipe_write workgroups per CU (0: as many as fit; set before upload)
    int opt_stage_bufs = 6;      // "stage_bufs" / "stage_piece_kb": pinned upload ring (stage.hpp)
};

struct pq_chunk {
    int32_t type = 0;
    int16_t max_def = 0, max_rep = 0;
    int32_t width = 0, plain_width = 0;
    int64_t nrows = 0;
    int64_t row_offset = 0;             // page-range uploads: global row of the first data page
    int64_t payload_bytes = 0;
    pqfmt::PageList walked;             // every walked page, all chunks, global rows
    HVec<int64_t> page_seq;             // walk sequence of each device data page
    std::vector<int64_t> dict_seq;      // walk sequence of each device dict page
    int walk_error = 0;
    std::string walk_message;
    int64_t walk_error_seq = 0;
    int first_error = 0;                // error detected at upload time
    // device
    uint8_t* d_bytes = nullptr;
    size_t nbytes = 0;
    DevPage* d_pages = nullptr;
    int npages = 0;
    DevDict* d_dicts = nullptr;
    int ndicts = 0;
    DevTile* d_tiles = nullptr;
    int ntiles = 0;
    int32_t* d_page_tile0 = nullptr;
    uint64_t* d_entries = nullptr;
    int64_t nentries = 0;
    uint32_t max_dict_bytes = 0;        // largest dictionary payload
    // dictionary pages too large for k_dict_index's LDS (launch_dict_big)
    struct BigDict { int di; pqk::DevDict d; size_t scr_off, lens_off, pad_off; };
    std::vector<BigDict> hbigd;
    uint8_t* d_bigd = nullptr;          // their scratch
    uint32_t max_page_bytes = 0;        // largest data-page payload
    int32_t* d_dict_count = nullptr;
    DevErr* d_page_err = nullptr;
    DevErr* d_dict_err = nullptr;
    int32_t* d_flags = nullptr;  // [0] err_any, [1] overflow
    uint64_t* d_row_codes = nullptr;
    int64_t* d_tile_chars = nullptr;
    // three-pass dictionary BYTE_ARRAY decode (dict_pipe.hip)
    bool pipe = false, pipe_count = false;
    int32_t pipe_dict = -1;
    uint32_t pipe_dict_chars_bytes = 0, pipe_dict_bytes = 0, pipe_lds = 0, pipe_ecap = 0;
    int pipe_cus = 256;
    int pipe_grid = 0;
    uint2* d_runs = nullptr;
    uint32_t* d_info = nullptr;
    uint16_t* d_codes = nullptr;
    // the per-row codes (and dictionary entry table) depend only on the
    // chunk's bytes: once a pipe pass that wrote them was checked error-free
    // (collect), regex scans read them instead of recomputing
    bool codes_pending = false, codes_ok = false;
    bool entries_pending = false, entries_ok = false;  // the same for the dictionary entry table
    // pq_decode_regex_async: the decode about to launch also runs the page
    // filter (k_regex_dict before k_pipe_write, match bits in the writer)
    bool arm = false;
    int arm_neg = 0;
    // string index of a REQUIRED PLAIN chunk (u16 window offset per row),
    // filed by the first error-free windowed scan, read by the later ones
    uint16_t* d_rx_index = nullptr;
    bool rx_index_ok = false, rx_index_pending = false;
    uint32_t rx_index_win = 0;
    uint32_t pipe_dict_payload = ~0u;  // payload bytes of the pipe's dictionary (arming bound)
    int32_t* d_tile_nn = nullptr;
    unsigned long long* d_bsum = nullptr;
    int32_t* d_flist = nullptr;
    bool pipe_small = false;            // some pages take k_pipe_runs (<= kPipeSmallRows rows)
    uint32_t pipe_small_bytes = 0;      // the largest payload of those pages
    bool pipe_wide = false;             // 32-bit codes, dictionary in HBM (k_pipe_big<true> -> k_pipe_wwide)
    int pipe_wpw = 10;                  // k_pipe_write writer waves per workgroup (planned)
    std::vector<int32_t> hbig;          // pages of more than kPipeSmallRows rows (k_pipe_big)
    int32_t* d_bigp = nullptr;
    uint32_t big_max_bytes = 0;
    int32_t pipe_entry_base = 0;        // entry-table slot of the pipe dictionary's first entry
    size_t z_bsum = 0, z_flist = 0;  // offsets in a zero block: bsum, flist
    uint8_t* d_zero = nullptr;          // pipe chunks: two blocks of [flags][bsum][flist], alternating per decode
    size_t zfull = 0;                   // bytes per block
    int zsel = 0;                       // block of the current decode
    bool next_zeroed = false;           // the other block is clear (the last k_pipe_write cleared it)
    int32_t* d_dflag = nullptr;         // the side-stream dictionary decode's error flag (sticky, cleared at upload)
    size_t zero_bytes = 4 * sizeof(int32_t);  // bytes of d_flags cleared per decode (flags, bsum, flist[0])
    bool tiles_aligned32 = false;       // every tile starts on a 32-row boundary: k_pipe_write owns whole validity words
    // PLAIN BYTE_ARRAY, REQUIRED (plain_ba.hip)
    bool plain = false;
    std::vector<pqk::DevBatch> hpwins;
    pqk::DevBatch* d_pwins = nullptr;
    std::vector<int64_t> hpwbase;      // k_plain_fused: first output byte per window (+ total), or empty
    int64_t* d_pwbase = nullptr;
    uint32_t* d_rowinfo = nullptr;
    int64_t* d_wchars = nullptr;
    unsigned long long* d_pbsum = nullptr;
    int plain_grid = 0;
    // pages larger than a window: speculative chunk chains (plain_ba.hip k_plain_spec)
    bool plain_spec = false, spec_failed = false;
    bool pfused_failed = false;          // k_plain_fused gave up on this chunk: two passes from now on
    // OPTIONAL chunks on the PLAIN kernels (plain_ba.hip OptLaunch): levels,
    // value-section pages, dense offsets spread over the rows
    bool plain_opt = false, popt_failed = false;
    bool opt_lane_levels = false;       // every page <= kOptLaneRows rows: lane-per-page levels
    int32_t* d_page_nn = nullptr;
    int64_t* d_onnv = nullptr;          // per page: non-null values | characters
    int64_t* d_ochv = nullptr;
    int64_t* d_opdense = nullptr;       // their exclusive scans
    int64_t* d_opbase = nullptr;
    int64_t* d_otot = nullptr;          // [0] non-null values, [1] characters
    DevPage* d_vpages = nullptr;
    int64_t* d_doffs = nullptr;         // dense offsets (nrows + 1)
    DevErr* d_operr = nullptr;          // level / chain errors of this path (not reported: the general path re-runs)
    std::vector<int32_t> hpwpage;       // spec windows: their real page
    int32_t* d_pwpage = nullptr;
    std::vector<int32_t> hchunk_base;
    std::vector<uint2> hchunks;
    int32_t* d_chunk_base = nullptr;
    uint2* d_chunks = nullptr;
    uint4* d_cand = nullptr;
    DevPage* d_ppages = nullptr;
    DevErr* d_perr = nullptr;
    pq_column* last_out = nullptr;      // output of the last pq_decode_async (collect re-runs into it)
    // tile-parallel PLAIN fixed-width decode (fixed_fast.hip)
    bool fixed_plain = false;
    int32_t* d_tile_rank = nullptr;
    int32_t* d_page_pos = nullptr;
    int64_t* d_tile_base = nullptr;
    int64_t* d_total = nullptr;
    int64_t* d_scan_scratch = nullptr;
    int64_t char_estimate = 0;
    // fused BYTE_ARRAY path (dict_fused.hip): one launch per input chunk
    struct Range {
        int32_t p0 = 0, np = 0, dict_id = -1;
        uint32_t rows_cap = 0, stage_bytes = 0, wave_bytes = 0, dict_bytes = 0, dict_chars_bytes = 0;
        int waves = 0, grid = 0;
    };
    std::vector<Range> ranges;
    bool fused = false;
    uint64_t* d_status = nullptr;
    int32_t* d_tickets = nullptr;
    int64_t* d_bases = nullptr;
    // regex
    uint8_t* d_page_flags = nullptr;
    uint8_t* d_dict_match = nullptr;
    uint8_t* d_dfa = nullptr;           // regex DFA image (regex.hpp DevDfa)
    std::vector<pqk::DevBatch> hrwins;  // windowed PLAIN regex scan: page windows
    pqk::DevBatch* d_rwins = nullptr;
    int32_t* d_rwin_ticket = nullptr;
    uint32_t rwin_bytes = 0, rwin_for_dfa = 0;
    int rwin_grid = 0;
    int rwin_opt = 0;                   // regex_win the windows were planned with
    uint32_t dfa_bytes = 0;
    bool dfa_full = false;               // the DFA image has full 256-column rows
    bool dfa_sink = false;               // full rows of an anchored pattern (k_regex_plain<.., true>)
    std::string prog_pattern;           // pattern of d_prog / d_dfa
    int64_t dict_match_cap = 0;
    pqre::DeviceProgram* d_prog = nullptr;
};

namespace pqcapi {

template <class T>
int dalloc(T** p, size_t n) {
    *p = nullptr;
    if (n == 0) n = 1;
    return hipMalloc(reinterpret_cast<void**>(p), n * sizeof(T)) == hipSuccess ? 0 : PQ_ERR_HIP;
}
template <class T>
void dfree(T*& p) {
    if (p) (void)hipFree(p);
    p = nullptr;
}

// host/plan.cpp
void plan_pipe(pq_ctx* ctx, pq_chunk* c, const PVec<DevPage>& pages, const std::vector<DevDict>& dicts);
void plan_plain(pq_ctx* ctx, pq_chunk* c, const PVec<DevPage>& pages);
void plan_fused(pq_ctx* ctx, pq_chunk* c, const PVec<DevPage>& pages, const std::vector<DevDict>& dicts);
bool plan_pages_parallel(pq_chunk* c, const pq_chunk_desc& desc, const pqfmt::WalkResult& w, bool keep_walk, int hw,
                         int64_t seq, int64_t& row_base, int64_t& img, PVec<DevPage>& hpages,
                         std::vector<DevDict>& hdicts, HVec<std::pair<int64_t, int64_t>>& copies,
                         HVec<int32_t>& copy_size);
bool plan_regex_windows(pq_ctx* ctx, pq_chunk* c);

}  // namespace pqcapi
