// kernels.hpp — device-side data layout shared by the HIP kernels and the
// C-ABI host code (capi.hip).  See DESIGN.md "Data layout in HBM".
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "pq_gpu.h"

namespace pqk {

constexpr int kWave = 64;
constexpr int kTileRows = 512;        // rows per decode tile (ref-layout page = 1 tile)
constexpr uint32_t kNullCode = 0xFFFFFFFFu;

// MODE_BOOL_RLE: BOOLEAN values in the RLE encoding ([u32 len][hybrid stream,
// bit width 1]; DATA_PAGE_V2 writers use it), extended walks only
enum PageMode : int32_t { MODE_DICT = 0, MODE_PLAIN = 1, MODE_BOOL = 2, MODE_BOOL_RLE = 3 };

// One data page, as the kernels see it (32 B, HBM-resident).
struct DevPage {
    uint64_t off;       // payload offset in the device byte image
    int32_t size;       // payload bytes (compressed_page_size)
    int32_t nvals;      // DataPageHeader.num_values (= rows produced)
    int64_t first_row;  // output row of the first value
    int32_t mode;       // PageMode
    int32_t dict;       // DevDict index or -1
};

// One dictionary page (column_reader.cpp:128-138).
struct DevDict {
    uint64_t off;        // payload offset in the device byte image
    int32_t size;        // payload bytes
    int32_t nvals;       // entries declared by the header
    int32_t entry_base;  // first slot in the entry table
    int32_t pad;
};

// A tile = up to kTileRows consecutive rows of one page.
struct DevTile {
    int32_t page;
    int32_t row0;    // first row within the page
    int32_t nrows;
    int32_t pad;
};

// Error record: code 0 = ok; BUFFER errors carry (pos, need, size) so the host
// can rebuild the reference message "ByteBuffer: read beyond end (...)".
struct DevErr {
    int32_t code;
    int32_t pos;
    int32_t need;
    int32_t size;
};

// One payload of the raw-bytes → slot-image relayout (relayout.hip).
struct RelayoutEntry {
    uint64_t src;    // offset of the payload in the raw byte buffer
    uint64_t dst;    // slot offset in the image (16-byte aligned)
    uint32_t avail;  // payload bytes present (compressed_page_size, cut at EOF)
    uint32_t slot;   // slot bytes (multiple of 16): avail..slot are zero-filled
};
void launch_relayout(hipStream_t s, const uint8_t* raw, uint8_t* img, const RelayoutEntry* ent, int32_t n);

// One compressed or DATA_PAGE_V2 payload → its slot (codec.hip).
enum : uint32_t { kCodecV2 = 1, kCodecDefPrefix = 2, kCodecRepPrefix = 4 };
struct CodecEntry {
    uint64_t src;      // payload offset in the source buffer (raw chunk bytes)
    uint64_t dst;      // slot offset in the image (16-byte aligned)
    uint32_t src_len;  // compressed_page_size (cut at EOF)
    uint32_t out_len;  // payload bytes the slot receives (V1 layout)
    uint32_t def_len;  // V2: definition / repetition level bytes
    uint32_t rep_len;
    uint32_t codec;    // 0: values stored as is (V2, is_compressed = false), else CompressionCodec
    uint32_t flags;    // kCodec*
};
size_t codec_lds_bytes();
// status[i]: 0 ok, 1 corrupt input, 2 size mismatch, 3 unsupported.  kind:
// 1 the entries include GZIP pages (the CRC-32 instantiation; it takes codec
// 0 and 2 only), 2 they include ZSTD pages (codecs 0 and 6 only: a 32 KiB
// history ring and the decode tables in LDS), 0 neither
void launch_codec(hipStream_t s, const uint8_t* src, uint8_t* img, const CodecEntry* ent, int32_t n,
                  uint32_t* status, int cus, int kind, int32_t nsmall);
// entries with out_len under this take the small-page layout (nsmall counts them)
uint32_t codec_small_bytes();

// 4 KiB chunker (chunker.hip, src/main.cpp:17-32): device scratch bytes for
// n rows, and the launch sequence (synchronises the stream; 0 = OK).
size_t chunk_assign_scratch(int64_t n);
int chunk_assign(hipStream_t st, const uint32_t* validity, const int64_t* offsets, int64_t n, int64_t chunk_bytes,
                 int64_t* out, uint8_t* scratch, int64_t* num_chunks);

// Per-device launch facts (host/launch_attr.cpp), thread-safe and keyed by
// the current device: the dynamic-LDS limit of a kernel (raised when needed;
// false if the device refuses), resident workgroups per CU for (kernel,
// block threads, dynamic LDS), and the device's compute units.
bool ensure_dyn_lds(const void* fn, uint32_t bytes);
int resident_blocks(const void* fn, int threads, uint32_t lds);
int device_cus();

struct ColumnParams {
    int32_t type;
    int16_t max_def;
    int16_t max_rep;
    int32_t width;      // fixed-width output bytes (BOOLEAN 1, INT96 12)
    int32_t plain_width;// bytes per PLAIN value in the page
};

// ── launch wrappers (decode.hip) ────────────────────────────────────────────
void launch_dict_entries(hipStream_t s, const uint8_t* bytes, const DevDict* dicts, int ndicts,
                         uint64_t* entries, int32_t* dict_count, DevErr* dict_err, int32_t* err_any,
                         int32_t type, int32_t plain_width);

void launch_ba_rows(hipStream_t s, const uint8_t* bytes, const DevPage* pages, int npages,
                    const DevDict* dicts, const uint64_t* entries, const int32_t* dict_count,
                    ColumnParams cp, uint64_t* row_codes, int64_t* tile_chars,
                    const int32_t* page_tile0, DevErr* page_err, int32_t* err_any, uint32_t big_plain_min,
                    uint32_t max_page, bool wide, uint64_t* prof = nullptr);
uint32_t ba_rows_stage_bytes();

void launch_scan_i64(hipStream_t s, const int64_t* in, int64_t* out_excl, int64_t n,
                     int64_t* total, int64_t* scratch);

void launch_ba_gather(hipStream_t s, const uint8_t* bytes, const DevPage* pages,
                      const DevTile* tiles, int ntiles, const DevDict* dicts,
                      const uint64_t* entries, const uint64_t* row_codes,
                      const int64_t* tile_base, int64_t nrows_total, const int64_t* total,
                      int64_t capacity, int32_t* overflow, uint32_t* validity, int64_t* offsets,
                      uint8_t* chars, bool byte_gather);

void launch_fixed(hipStream_t s, const uint8_t* bytes, const DevPage* pages, int npages,
                  const DevDict* dicts, const int32_t* dict_count, ColumnParams cp,
                  uint32_t* validity, uint8_t* values, DevErr* page_err, int32_t* err_any);

// ── three-pass dictionary BYTE_ARRAY path (dict_pipe.hip) ──────────────────
constexpr uint32_t kPipeRunCap = 128;  // run records per stream per page
constexpr int32_t kPipeSmallRows = 2048;   // larger pages take k_pipe_big (one workgroup per page)
constexpr uint32_t kBigSegBytes = 24576;   // k_pipe_big: payload bytes one jump-table segment covers (at most)
constexpr uint32_t kBigOneSeg = 18432;     // k_pipe_big: larger pages take two segments (two workgroups per CU up to ~26 KiB)
constexpr uint32_t kBigMaxBytes = 49152;   // k_pipe_big: payload bytes per page (staged; two segments past kBigSegBytes)
constexpr uint32_t kBigLens = 8192;        // k_pipe_big: dictionary entry lengths held in LDS
constexpr int32_t kBigTiles = 64;          // k_pipe_big: 512-row tiles per page

struct PipeLaunch {
    const uint8_t* bytes;
    const DevPage* pages;
    int32_t npages;
    const DevTile* tiles;
    int32_t ntiles;
    const int32_t* page_tile0;
    int32_t max_def, max_rep;
    const DevDict* dicts;
    int32_t dict_id;
    const uint64_t* entries;
    const int32_t* dict_count;
    const uint2* runs;          // npages x 2 x kPipeRunCap
    const uint32_t* info;       // per page: run counts, index bit width, fallback flag
    const int32_t* flist;       // [count, pages...] marked for the exact decoder
    int32_t* tile_nn;           // per tile non-null rows (pages > 512 rows with def levels)
    uint16_t* codes;            // per row dictionary index, 0xFFFF = NULL
    int64_t* tile_chars;
    unsigned long long* bsum;   // per k_pipe_write workgroup characters (zeroed, P.grid entries)
    int64_t* total;
    int64_t nrows_total;
    int64_t capacity;
    int32_t* overflow;
    uint32_t* validity;
    int64_t* offsets;
    uint8_t* chars;
    DevErr* page_err;
    int32_t* err_any;
    uint32_t dict_chars_bytes, dict_bytes, lds;
    int grid;
    int debug;  // ablation bits (k_pipe_write)
    uint32_t dict_entries_cap;  // entry-table capacity of the dictionary (k_pipe_codes length table)
    int cus;
    bool has_small;             // some pages of <= kPipeSmallRows rows (k_pipe_runs / k_pipe_codes3)
    int write_waves;            // writer waves per k_pipe_write workgroup (planned with P.lds / P.grid)
    uint32_t* znext;            // cleared by k_pipe_write (the next decode's flags/bsum/flist[0]), or null
    uint32_t znext_words;
    const uint8_t* match = nullptr;  // armed page filter (k_pipe_write), dictionary payloads < kArmDictBytes
    int match_neg = 0;
    uint8_t* page_flags = nullptr;
    // wide dictionaries (k_pipe_big<true> -> k_pipe_wwide): 32-bit codes
    // here (0xFFFFFFFF = NULL) instead of `codes`; P.lds / P.grid are then
    // plan_pipe_wide's
    uint32_t* codes32 = nullptr;
    // the wide dictionary's entry lengths as bytes (255: 255 or more; from
    // launch_dict_big) and their capacity, or null: k_wide_chars then reads
    // the entry table
    const uint8_t* lens8 = nullptr;
    uint32_t lens8_cap = 0;
    // the same dictionary as 16-byte slots (launch_dict_big's pad16), or
    // null: k_pipe_wwide then reads entry words and characters
    const uint4* pad16 = nullptr;
};
constexpr uint32_t kArmDictBytes = 32768;  // every entry length < 2^15: the match bit rides in the entry word
struct PipePlan {
    uint32_t lds;       // dynamic LDS bytes of k_pipe_write
    int blocks_per_cu;  // 0: the dictionary does not fit
};
PipePlan plan_pipe_lds(uint32_t dict_bytes, int wpw);
// k_pipe_wwide (dictionary in HBM): per-wave scratch only (pad: + the rows'
// 16-byte entry slots, k_pipe_wwide<true>)
PipePlan plan_pipe_wide(int wpw, bool pad);
// Dictionary pages for k_pipe_runs' leading workgroups (4 waves each; pages
// up to kRunDictMax bytes), so the dictionary decodes inside the run-table
// launch instead of a k_dict_index launch on a side stream.
struct RunDicts {
    const DevDict* dicts;
    int ndicts;
    uint64_t* entries;
    int32_t* dict_count;
    DevErr* dict_err;
    int32_t* err_any;
};
constexpr uint32_t kRunDictMax = 60 * 1024;
void launch_pipe_runs(hipStream_t s, const uint8_t* bytes, const DevPage* pages, int npages, int32_t max_def,
                      int32_t max_rep, uint2* runs, uint32_t* info, int pages_per_wave, int32_t* flist, int debug,
                      const RunDicts* dicts = nullptr, uint32_t stage_max = 0,  // 0: k_pipe_codes3's stage
                      uint32_t slot_max = 0, uint32_t dict_max = 0, int cus = 256);  // pages_per_wave 0: auto
void launch_pipe_codes(hipStream_t s, const PipeLaunch& P, bool count_pass);
struct DevBatch;
void launch_pipe_write(hipStream_t s, const PipeLaunch& P);
// The page walk on the GPU (walk.hip): one header record per page a
// segment's chain meets, the launch's buffers (nseg segments of `seg` bytes,
// `cap` records each; segs / links: walk_seg_bytes() / walk_link_bytes() per
// segment; base_pg / base_val / dict_in: nseg int64; out: 2 int64 (pages or
// -1 = refused, cut segment); pages: the page table, <= nseg * cap entries).
struct WalkRec {
    uint64_t pos;
    uint32_t hs;
    int32_t comp, uncomp, type, nv, enc;
    uint32_t flags;
    uint32_t pad;
};
struct WalkLaunch {
    const uint8_t* bytes;  // file bytes [base, base + len) in HBM
    uint64_t base, len;
    uint64_t start, end;   // the chain's first page and the extent's end (file offsets)
    uint64_t seg;
    uint32_t nseg, cap;
    int64_t num_values;
    WalkRec* recs;
    void* segs;
    void* links;
    int64_t *base_pg, *base_val, *dict_in, *out;
    pq_page_desc* pages;
};
size_t walk_seg_bytes();
size_t walk_link_bytes();
void launch_walk(hipStream_t s, const WalkLaunch& W);
// pages of more than kPipeSmallRows rows: run tables by speculative parse,
// then codes and tile characters (one workgroup per listed page)
uint32_t pipe_big_lds(uint32_t max_page_bytes, uint32_t nlens);
// the regex filter over the wide pipe's codes holds one match bit per entry in LDS
bool pipe_match_wide_ok(uint32_t entries_cap);
void launch_pipe_big(hipStream_t s, const PipeLaunch& P, const int32_t* big_pages, int nbig, uint32_t max_page_bytes);
// wide pipe: every tile's characters from the raw 32-bit codes k_pipe_big<true>
// wrote (after the dictionary decode), filed for k_pipe_wwide
void launch_wide_chars(hipStream_t s, const PipeLaunch& P);
// regex page filter on the codes: page_flags[p] = 1 unless a non-null row of
// page p matches (neg: fails to match); match = dictionary match bits
void launch_pipe_match(hipStream_t s, const PipeLaunch& P, const uint8_t* match, int neg, uint8_t* page_flags,
                       bool flags_set = false);  // flags_set: page_flags already 1 (k_regex_dict set them)

// ── tile-parallel PLAIN fixed-width path (fixed_fast.hip) ──────────────────
// OPTIONAL columns' def levels alone (k_fixed_levels2): validity, per-tile
// ranks, value section start and non-null count of every page
void launch_fixed_levels(hipStream_t s, const uint8_t* bytes, const DevPage* pages, int npages,
                         const int32_t* page_tile0, ColumnParams cp, uint32_t* validity, int32_t* tile_rank,
                         int32_t* page_pos, int32_t* page_nn, DevErr* page_err, int32_t* err_any, bool small);
void launch_fixed_plain(hipStream_t s, const uint8_t* bytes, const DevPage* pages, int npages, const DevTile* tiles,
                        int ntiles, const int32_t* page_tile0, ColumnParams cp, uint32_t* validity,
                        uint8_t* values, int32_t* tile_rank, int32_t* page_pos, DevErr* page_err,
                        int32_t* err_any, bool fused, bool small);

// ── fused BYTE_ARRAY path (dict_fused.hip) ─────────────────────────────────
struct FusedLaunch {
    const uint8_t* bytes;
    const DevPage* pages;
    int32_t p0, np;
    const DevDict* dicts;
    int32_t dict_id;
    const uint64_t* entries;
    const int32_t* dict_count;
    int32_t max_def, max_rep;
    uint32_t rows_cap, stage_bytes, wave_bytes, dict_bytes, dict_chars_bytes;
    uint64_t* status;
    int32_t* ticket;
    const int64_t* base_in;
    int64_t* base_out;
    int64_t nrows_total;
    uint32_t* validity;
    int64_t* offsets;
    uint8_t* chars;
    int64_t capacity;
    int32_t* overflow;
    DevErr* page_err;
    int32_t* err_any;
    int grid;
    int waves_per_block;
    int debug;
    uint64_t* prof;  // per-phase cycle sums (fused_prof_slots()), or null
    int claim;       // pages per ticket
};

// A run of consecutive data pages whose payload slots form one contiguous
// image range [img_lo, img_lo + img_bytes).
struct DevBatch {
    int32_t p0, np;
    uint64_t img_lo;
    uint32_t img_bytes;
    uint32_t nrows;  // the pages' values (windows of the regex scan; else 0)
    int64_t row0;    // first row of page p0 (windows of the regex scan)
};


// Dictionary pages whose payload + 32 bytes exceed kDictLdsCap are skipped
// by k_dict_index and decoded by launch_dict_big (one call per such page:
// page = its payload in the image, entries/count/err = its slots, lens8
// (or null): min(length, 255) per entry, pad16 (or null): per entry its
// characters 0..14 and its length in byte 15 (0xFF: 16 or more); scratch:
// dict_big_scratch(size) bytes, no zeroing needed).
constexpr uint32_t kDictLdsCap = 128 * 1024;
constexpr uint32_t kPCandDHost = 4;  // candidates per slice (dict_index.hpp kPCandD)
void launch_dict_index(hipStream_t s, const uint8_t* bytes, const DevDict* dicts, int ndicts,
                       uint64_t* entries, int32_t* dict_count, DevErr* dict_err, int32_t* err_any,
                       uint32_t max_dict_bytes);
uint32_t dict_big_slices(uint32_t size);
uint32_t dict_big_scratch(uint32_t size);
void launch_dict_big(hipStream_t s, const uint8_t* page, uint32_t size, uint32_t nvals, uint64_t* entries,
                     uint8_t* lens8, uint4* pad16, int32_t* count, DevErr* err, int32_t* err_any, uint32_t* scr);
void launch_ba_fused(hipStream_t s, const FusedLaunch& L);
uint32_t fused_wave_bytes(uint32_t rows_cap, uint32_t stage_bytes);
int fused_occupancy_waves(uint32_t lds_bytes_per_block, int waves_per_block);
int fused_prof_slots();

// ── PLAIN BYTE_ARRAY, REQUIRED (plain_ba.hip) ────────────────────────────
constexpr uint32_t kPWin = 8192;  // window bytes (consecutive page slots)
struct PlainLaunch {
    const uint8_t* bytes;
    const DevPage* pages;
    const DevBatch* wins;        // windows: p0, np, img_lo, img_bytes
    int32_t nwins;
    uint32_t* rowinfo;           // per row: position in window | length << 16
    int64_t* wchars;             // per window characters
    unsigned long long* bsum;    // per k_plain_write workgroup characters
    int per, grid;
    int64_t nrows_total;
    int64_t* total;
    int64_t capacity;
    int32_t* overflow;
    uint32_t* validity;
    int64_t* offsets;
    uint8_t* chars;
    DevErr* page_err;
    int32_t* err_any;
    const int32_t* gate;         // non-null: skip everything when *gate != 0 (the spec path fell back)
    const int64_t* wbase;        // non-null: first output byte of every window (nwins + 1), the one-pass kernel runs
                                 // (pseudo pages: per window, the first output byte of its real page minus
                                 // its image offset plus 4 x its first row; the kernel adds its first string's)
    int32_t* redo;               // with wbase: set by the one-pass kernel when a page does not fit its
                                 // form (the host then decodes the chunk with the two passes)
    int32_t wmode;               // one-pass: kWinBase, kWinPseudo, kWinOpt, kWinOptPseudo
    // OPTIONAL chunks (kWinOpt*): the pages are value sections of the real
    // pages (k_opt_pages), rows are non-null rows; the one-pass kernel writes
    // their offsets to a dense array that k_opt_offsets spreads over the rows
    const int64_t* pbase;        // characters before each real page
    const int64_t* pdense;       // non-null rows before each real page
    const int32_t* ppos;         // value section start of each real page
    const int32_t* wpage;        // kWinOptPseudo: the real page of each window
    const DevPage* rpages;       // kWinOptPseudo: the real pages
};
enum : int32_t { kWinBase = 0, kWinPseudo = 1, kWinOpt = 2, kWinOptPseudo = 3 };
int plain_write_blocks_per_cu();

// PLAIN BYTE_ARRAY pages larger than a window (plain_ba.hip k_plain_spec /
// k_plain_link): each page is cut into kPChunk-byte chunks; the chunks' string
// chains are found speculatively and linked per page into pseudo pages (one
// per chunk, whole strings only) that k_plain_walk / k_plain_write decode in
// windows of kPChunkGroup chunks.  Anything the link cannot resolve sets
// *fallback and the host re-runs the chunk on the generic path.
// C4 c7 (10M strings of 10..44 bytes): 2048 B x 3 per window 0.74 ms, 1024 x 7
// 0.61 (0.54 with the speculative link), 512 x 15 0.51, 256 x 31 0.56.  A
// window's chunks plus one string of <= 60 bytes fit kPWin.
constexpr uint32_t kPChunk = 512;
constexpr uint32_t kPChunkGroup = 15;
constexpr uint32_t kPCand = 4;  // candidate chain starts kept per chunk
struct SpecLaunch {
    const uint8_t* bytes;
    const DevPage* pages;        // the real pages
    int32_t npages;
    const int32_t* chunk_base;   // per real page: its first chunk (npages + 1 entries)
    const uint2* chunks;         // per chunk: real page, chunk number in the page
    int32_t nchunks;
    uint4* cand;                 // per chunk kPCand candidate records
    DevPage* ppages;             // per chunk: the pseudo page
    DevErr* page_err;            // per real page
    int32_t* err_any;
    int32_t* fallback;
    // OPTIONAL chunks: the chain of real page p starts at ppos[p] (after its
    // levels) and reads vpages[p].nvals values, rows from vpages[p].first_row
    const int32_t* ppos;
    const DevPage* vpages;
};
void launch_plain_spec(hipStream_t s, const SpecLaunch& S);

// OPTIONAL PLAIN BYTE_ARRAY chunks on the PLAIN kernels (plain_ba.hip): after
// k_fixed_levels2 (validity, tile ranks, value section starts, non-null
// counts), the per-page value sections become REQUIRED-shaped pages of their
// non-null values; anything unusual (a level error, a section too short for
// its values) sets *redo and the host decodes the chunk on the general path.
struct OptLaunch {
    const DevPage* pages;        // the real pages
    int32_t npages;
    const int32_t* page_nn;      // non-null values per page (k_fixed_levels2)
    const int32_t* page_pos;     // value section start per page
    const DevErr* lerr;          // level errors per page
    int64_t* nnv;                // per page: non-null values, then (scan) values before it
    int64_t* chv;                // per page: characters, then (scan) characters before it
    int64_t* pdense;             // exclusive scans of nnv / chv
    int64_t* pbase;
    int64_t* scratch;            // scan scratch (npages / 8192 + 16)
    int64_t* tot_nn;             // scan totals
    int64_t* tot_ch;
    DevPage* vpages;             // out: value-section pages
    int64_t* doffs;              // dense offsets (their entry at the non-null total gets the character total)
    int32_t* redo;
};
void launch_opt_pages(hipStream_t s, const OptLaunch& O);
// def levels of pages of up to kOptLaneRows rows, one lane per page (the
// same outputs as launch_fixed_levels for the PLAIN kernels' OPTIONAL form)
constexpr int32_t kOptLaneRows = 2048;
void launch_opt_levels(hipStream_t s, const uint8_t* bytes, const DevPage* pages, int npages,
                       const int32_t* page_tile0, int32_t max_def, uint32_t* validity, int32_t* tile_rank,
                       int32_t* page_pos, int32_t* page_nn, DevErr* lerr, int32_t* redo);
// offsets of every row from the dense offsets: row R takes entry rank(R)
// (non-null rows before it), NULL rows included; offsets[nrows] = total
void launch_opt_offsets(hipStream_t s, const DevPage* pages, const DevTile* tiles, int ntiles,
                        const int32_t* tile_rank, const int64_t* pdense, const uint32_t* validity,
                        const int64_t* doffs, int64_t* offsets, const int32_t* redo);
// REQUIRED PLAIN BYTE_ARRAY pages larger than min_size bytes: row codes and
// tile characters for the generic gather (k_ba_rows skips these pages)
void launch_plain_big_rows(hipStream_t s, const uint8_t* bytes, const DevPage* pages, int npages, uint32_t min_size,
                           uint64_t* row_codes, int64_t* tile_chars, const int32_t* page_tile0, DevErr* page_err,
                           int32_t* err_any);
void launch_plain_ba(hipStream_t s, PlainLaunch P);

}  // namespace pqk
