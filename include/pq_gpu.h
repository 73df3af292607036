/*
 * pq_gpu.h — C ABI of the MI355X Parquet page-decode / regex page-scan path.
 *
 * This is the drop-in boundary behind the reference's C++ API
 * (sputnik89/duckdb-parquet-parser).  Plain C: pointers, sizes, status codes,
 * no C++ or torch types, and no exception ever crosses it.  Each entry point
 * names the reference interface it replaces:
 *
 *   pq_build_page_table  ColumnReader::read_all's page walk
 *                        (src/reader/column_reader.cpp:18-71, the header loop
 *                        and PageHeader::deserialize, src/reader/metadata.cpp:121-155)
 *   pq_chunk_upload      the ReadRangeFunc byte supply
 *                        (include/reader/column_reader.hpp:10; parquet_reader.cpp:173-178)
 *   pq_decode            ColumnReader::read_all / read_pages value decode
 *                        (column_reader.cpp:128-268, rle_decoder.hpp:6-108)
 *   pq_regex_pages       the README's --regex-column page filter (README.md:54-64;
 *                        no source in the reference — contract in SURVEY §8a R-REGEX)
 *   pq_file_*            ParquetReader::open footer/schema/page index
 *                        (parquet_reader.cpp:14-61, 495-605)
 *
 * Ownership: a context owns device memory it hands out; every pq_*_free
 * releases it.  A context is used from one host thread at a time (the
 * reference's ParquetReader is not thread-safe either, parquet_reader.cpp:189).
 * Status: 0 = OK, negative = error class below; pq_last_error() has the text,
 * which reproduces the reference's exception message where one exists.
 */
#ifndef PQ_GPU_H
#define PQ_GPU_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    PQ_OK = 0,
    PQ_ERR_CODEC = -1,        /* "Only uncompressed parquet files are supported" (column_reader.cpp:13-15) */
    PQ_ERR_BUFFER = -2,       /* "ByteBuffer: read beyond end (pos=P need=N size=S)" (common.hpp:162-168) */
    PQ_ERR_OPTIONAL = -3,     /* std::bad_optional_access (column_reader.cpp:50,57)                       */
    PQ_ERR_FLBA = -4,         /* "FIXED_LEN_BYTE_ARRAY not supported without type_length" (254-256)      */
    PQ_ERR_TYPE = -5,         /* "Unsupported type: N" (column_reader.cpp:265-266)                        */
    PQ_ERR_THRIFT = -6,       /* ThriftReader::skip unknown type / "varint too long"                      */
    PQ_ERR_ALLOC = -7,        /* negative sizes (std::vector length_error / bad_alloc)                    */
    PQ_ERR_UNSUPPORTED = -8,  /* input outside the parity scope (reference behaviour undefined)          */
    PQ_ERR_DECOMPRESS = -9,   /* extended mode: a compressed page failed to decompress (corrupt input)    */
    PQ_ERR_ARG = -20,         /* bad argument to this API                                                 */
    PQ_ERR_HIP = -21,         /* HIP runtime failure / no device                                          */
    PQ_ERR_REGEX = -22        /* pattern outside the supported RE2/Python-re subset                       */
};

enum { PQ_BOOLEAN = 0, PQ_INT32, PQ_INT64, PQ_INT96, PQ_FLOAT, PQ_DOUBLE, PQ_BYTE_ARRAY,
       PQ_FIXED_LEN_BYTE_ARRAY };
enum { PQ_DATA_PAGE = 0, PQ_INDEX_PAGE = 1, PQ_DICTIONARY_PAGE = 2, PQ_DATA_PAGE_V2 = 3 };

typedef struct pq_ctx pq_ctx;
typedef struct pq_chunk pq_chunk; /* device-resident column chunk(s) of one leaf column */

/* ColumnChunk.meta_data + ColumnInfo fields the decode needs
 * (include/reader/metadata.hpp:17-28, include/reader/column_info.hpp:6-20). */
typedef struct {
    int64_t num_values;
    int64_t data_page_offset;
    int64_t dictionary_page_offset;
    int32_t has_dictionary_page_offset;
    int32_t codec;
    int32_t type;           /* ParquetType of the leaf column */
    int16_t max_def_level;
    int16_t max_rep_level;
    int64_t total_compressed_size; /* ColumnMetaData.total_compressed_size, or 0 if unknown:
                                      only an extent hint (a chunk of >= kSpecMinBytes = 4 MiB
                                      whose pages are small walks its page chain speculatively
                                      on host threads, one per >= 1 MiB of extent;
                                      csrc/host/format.hpp) */
    int32_t ext_flags;      /* 0 (pq_file_chunk's default): the reference's format scope.
                               PQ_EXT_* bits widen it beyond the reference */
    int32_t ext_reserved;   /* 0 */
} pq_chunk_desc;

/* pq_chunk_desc.ext_flags.  The reference rejects every compression codec
 * ("Only uncompressed parquet files are supported", column_reader.cpp:13-15)
 * and walks past DATA_PAGE_V2 pages without counting them (56-67).  With
 *   PQ_EXT_CODECS   pages of SNAPPY (1), GZIP (2), LZ4 (5, Hadoop framing) and
 *                   LZ4_RAW (7) chunks are decompressed on the GPU at upload;
 *   PQ_EXT_PAGE_V2  DATA_PAGE_V2 pages count as data pages: their level
 *                   sections and (decompressed) values are rebuilt on the GPU
 *                   into the V1 layout the reference reads
 *                   ([u32 def_len][def][u32 rep_len][rep][values]).
 * Outputs are checked against pyarrow. */
enum { PQ_EXT_CODECS = 1, PQ_EXT_PAGE_V2 = 2 };

/* One page of the walk (dictionary, data and skipped pages alike). */
typedef struct {
    int64_t header_offset;   /* file offset of the Thrift page header              */
    int64_t payload_offset;  /* file offset of the payload (after the header)      */
    int32_t payload_size;    /* compressed_page_size                               */
    int32_t page_type;       /* PageType                                           */
    int32_t num_values;      /* data: DataPageHeader.num_values; dict: entries     */
    int32_t encoding;        /* data: DataPageHeader.encoding                      */
    int32_t page_num;        /* ColumnReader::read_pages page_num                  */
    int32_t dict_page;       /* index of the dictionary page in force, or -1       */
    int64_t first_row;       /* data pages: first output row                       */
    int32_t uncompressed_size; /* PageHeader.uncompressed_page_size                 */
    int32_t flags;           /* PQ_PAGE_* (extended walks only)                    */
    int32_t v2_def_len;      /* DATA_PAGE_V2 level section bytes                   */
    int32_t v2_rep_len;
} pq_page_desc;

/* pq_page_desc.flags.  PQ_PAGE_COMPRESSED: the payload (V2: its values
 * section) is compressed with the chunk's codec, held in bits 8..15.  PQ_PAGE_V2: a DATA_PAGE_V2
 * page of an extended walk; it is listed with page_type PQ_DATA_PAGE because
 * the device holds it in the V1 layout. */
enum { PQ_PAGE_COMPRESSED = 1, PQ_PAGE_V2 = 2 };

/* Device-resident columnar result (SURVEY §8b "pq_column_out"):
 *   validity  LSB-first bitmap, bit i = row i non-null; ceil(n/32) words
 *   values    fixed-width types: n * value_width bytes (NULL rows zeroed);
 *             BYTE_ARRAY: the concatenated chars
 *   offsets   BYTE_ARRAY: n + 1 int64 offsets into values
 * INT96 is returned raw (12 bytes); the C++ adapter renders the reference's
 * "INT96(hi:lo)" string (column_reader.cpp:257-264). BOOLEAN is 1 byte 0/1. */
typedef struct {
    int64_t num_rows;
    int32_t type;
    int32_t value_width;     /* 0 for BYTE_ARRAY */
    uint32_t* d_validity;
    uint8_t* d_values;
    int64_t* d_offsets;
    int64_t num_bytes;       /* bytes in d_values */
    int64_t capacity_rows;   /* allocation bookkeeping (reuse across calls) */
    int64_t capacity_bytes;
} pq_column;

/* ── context ─────────────────────────────────────────────────────────────── */
/* One context per device; several contexts (also on one device) may be
 * driven from different host threads at once, each from one thread at a
 * time.  pq_device_count: visible devices (0 without a GPU). */
int pq_device_count(void);
pq_ctx* pq_ctx_create(int device);
void pq_ctx_destroy(pq_ctx* ctx);
const char* pq_last_error(const pq_ctx* ctx);
void* pq_ctx_stream(pq_ctx* ctx);              /* the hipStream_t kernels run on */
int pq_ctx_sync(pq_ctx* ctx);
/* Tuning switches (apply to chunks uploaded afterwards).  Every setting gives
 * the same outputs; they choose between kernels:
 *   "dict_pipe"   1 (default): three-pass dictionary BYTE_ARRAY kernels
 *   "write_waves" writer waves per workgroup of the pipe's write pass, 1..16 (10)
 *   "zflip"       1 (default): per-decode flags come pre-cleared by the previous
 *                 write pass, else a fill kernel per decode
 *   "big_all"     1: every page of a pipe chunk takes the large-page kernel
 *                 (k_pipe_big; coverage of that kernel on small pages), 0 (default)
 *   "pipe_run_pages" pages per wavefront of the run-table pass, 1..32 (32)
 *   "pipe_run_dict" 1 (default): dictionary pages up to 60 KiB decode in the
 *                 run-table launch (its leading workgroups), else in their own
 *                 launch on a side stream
 *   "pipe_wide"   1 (default): dictionaries beyond the writer's LDS (or of more
 *                 than 65,535 entries) take the wide pipe (32-bit codes, the
 *                 dictionary decoded beside the front); 0: the generic path
 *   "plain_ba"    1 (default): two-pass PLAIN BYTE_ARRAY kernels
 *   "plain_fused" 1 (default): their one-pass form when every page's strings
 *                 fill it exactly (checked on the device; else the two passes)
 *   "fixed_plain" 1 (default): tile-parallel PLAIN fixed-width kernels
 *   "fixed_fused" 0 (default): OPTIONAL PLAIN fixed-width chunks scatter their
 *                 values in a second launch; 1: inside the def-level launch
 *   "fused_ba"    1 (default): per-page fused BYTE_ARRAY kernel for chunks the
 *                 pipe does not take; 0 forces the generic rows/scan/gather kernels
 *   "wide_rows"   1 (default): generic BYTE_ARRAY chunks with dictionary pages
 *                 resolve rows by a workgroup per page (k_wide_rows); 0: one wave
 *                 per page (k_ba_rows)
 *   "gather_rows" 1 (default): the generic gather copies characters row per
 *                 lane; 0: byte-wise 16-byte blocks
 *   "levels_small" 1 (default): OPTIONAL fixed-width def levels in the 35 KB LDS
 *                 form (four workgroups per CU); 0: the 58 KB form
 *   "fused_waves" waves per workgroup cap (0 = automatic)
 *   "stage_bufs" pinned buffers of the upload ring, 2..16 (6); "stage_piece_kb"
 *                 bytes per buffer / H2D piece in KiB, 64..65536 (8192);
 *                 "stage_streams" DMA queues the pieces alternate over, 1..2 (2);
 *                 "raw_upload" 1 (default): chunks with a known byte extent go to
 *                 HBM as raw file bytes while the host walks, the slot image is
 *                 then built on the GPU (0: the host builds it);
 *                 "device_walk" 0 (default) / 1: with the raw upload, the page
 *                 walk runs on the GPU (pq_build_page_table_device) once the
 *                 raw bytes are in HBM; a chunk it refuses walks on the host
 *   "regex_dfa", "regex_plain", "regex_codes" 1 (default): DFA kernels, the
 *                 windowed kernel for dictionary-free chunks, match bits over
 *                 the pipe's codes; "regex_win" window bytes (1024..32768,
 *                 multiple of 16; 8192); "regex_reuse" 1 (default): a scan
 *                 of a chunk whose earlier pipe decode was checked error-free
 *                 (pq_decode / pq_decode_check) reads that decode's codes
 *                 instead of recomputing them; "regex_index" 1 (default): a
 *                 REQUIRED PLAIN chunk's first error-free windowed scan keeps
 *                 every string's window offset (2 B per row) for later scans
 * Diagnostics (timing studies only; outputs are not valid with bits set):
 *   "fused_debug", "regex_debug" ablation bits, "fused_prof"
 *   per-phase clocks (k_ba_fused; k_wide_rows: slots 0-5 phases, 6 fallback
 *   pages, 7 pages).
 * Unknown keys and out-of-range values return PQ_ERR_ARG. */
int pq_ctx_set_option(pq_ctx* ctx, const char* key, int64_t value);

/* ── host page walk (R-WALK / R-HDR) ────────────────────────────────────── */
/* Walks one chunk exactly like ColumnReader::read_all (256-byte header window,
 * zero padding past EOF).  Writes up to `cap` pages; *npages = pages walked.
 * Returns 0, or the error met by the walk after *npages good pages (the
 * message in err). */
int pq_build_page_table(const uint8_t* file, size_t file_len, const pq_chunk_desc* chunk,
                        pq_page_desc* pages, int64_t cap, int64_t* npages, char* err,
                        size_t errlen);

/* The same walk on the GPU (the device page table): the
 * chunk's bytes are already in HBM at d_bytes, holding file offsets
 * [base, base + len) (16-byte aligned; zeros are read past its end).  The
 * extent is cut into segments of seg_bytes (0: 8 KiB) walked speculatively,
 * one wavefront each, linked where each segment's chain leaves it
 * (csrc/kernels/walk.hip), with at most rec_cap pages per segment (0:
 * seg_bytes / 128).  Returns 0 with the same pages pq_build_page_table
 * lists (up to `cap` written to host `pages`, *npages = pages), or
 * PQ_ERR_UNSUPPORTED when the speculative chain cannot settle the walk
 * exactly (a page longer than a segment, an invalid header before the
 * value count, codecs / V2 flags): walk on the host then, which also reports
 * the reference's errors.  Replaces metadata.cpp:121-155's serial loop for
 * chunks already in device memory. */
int pq_build_page_table_device(pq_ctx* ctx, const uint8_t* d_bytes, size_t len, int64_t base,
                               const pq_chunk_desc* chunk, int64_t seg_bytes, int64_t rec_cap,
                               pq_page_desc* pages, int64_t cap, int64_t* npages);

/* A device copy of host bytes for pq_build_page_table_device (callers
 * without HIP headers): n bytes + 64 zero bytes, 256-byte aligned. */
int pq_device_buffer(pq_ctx* ctx, const uint8_t* host, size_t n, void** d_out);
void pq_device_buffer_free(pq_ctx* ctx, void* d);

/* ── device chunks ───────────────────────────────────────────────────────── */
/* Upload `nchunks` column chunks of ONE leaf column (e.g. every row group's
 * chunk of that column) from a host file image; the walk runs on the host,
 * the page bytes go to HBM once.  Rows of chunk k follow chunk k-1
 * (ParquetReader::read_column concatenation, parquet_reader.cpp:133-144). */
int pq_chunk_upload(pq_ctx* ctx, const uint8_t* file, size_t file_len, const pq_chunk_desc* chunks,
                    int nchunks, pq_chunk** out);
/* Page-range shard (the decode-a-page-list entry point; §8e):
 * uploads data pages [data_begin, data_end) of ONE chunk — ordinals among the
 * chunk's data pages in walk order — plus every dictionary page they use,
 * taken from `table`, the chunk's page table as pq_build_page_table returned
 * it (no re-walk).  Pages decode independently given their dictionary
 * (column_reader.cpp:140-225), so a shard's decode equals rows
 * [first_row, first_row + num_rows) of the whole chunk's decode; the unit of
 * sharding is the global data-page id of build_page_index
 * (parquet_reader.cpp:559-605).  Output rows start at 0; pq_chunk_first_row
 * gives the chunk row of the shard's first row. */
int pq_chunk_upload_range(pq_ctx* ctx, const uint8_t* file, size_t file_len, const pq_chunk_desc* chunk,
                          const pq_page_desc* table, int64_t ntable, int64_t data_begin,
                          int64_t data_end, pq_chunk** out);
/* Page-range plan for N shards: `world` contiguous ranges of the
 * chunk's DATA pages (ordinals in walk order, as pq_chunk_upload_range takes
 * them) balanced by payload bytes: range k ends where the running payload
 * total first reaches k/world of the chunk's sum (dictionary pages are not
 * counted; every shard that needs one gets it).  ranges[2k], ranges[2k + 1]
 * = [begin, end) of shard k.  Host only; the order is the reference's global
 * page order within a chunk (build_page_index, parquet_reader.cpp:559-605). */
int pq_plan_page_ranges(const pq_page_desc* table, int64_t ntable, int world, int64_t* ranges);
void pq_chunk_free(pq_ctx* ctx, pq_chunk* chunk);
int64_t pq_chunk_num_rows(const pq_chunk* chunk);
int64_t pq_chunk_first_row(const pq_chunk* chunk);     /* 0 unless a page-range upload */
int64_t pq_chunk_num_pages(const pq_chunk* chunk);       /* data pages */
int64_t pq_chunk_payload_bytes(const pq_chunk* chunk);   /* Σ data + dictionary payload bytes */
int pq_chunk_pages(const pq_chunk* chunk, pq_page_desc* pages, int64_t cap, int64_t* npages);

/* ── decode (ColumnReader::read_all on the GPU) ─────────────────────────── */
/* Decodes every data page of `chunk` into `out` (device memory; buffers are
 * reused when out->capacity_* suffice, so a caller can loop without
 * allocation).  Synchronous by default; pq_decode_async leaves the work on
 * the context stream. */
int pq_decode(pq_ctx* ctx, pq_chunk* chunk, pq_column* out);
int pq_decode_async(pq_ctx* ctx, pq_chunk* chunk, pq_column* out);
/* sync + error collection after _async; also completes the column the
 * chunk's last async decode wrote (its num_bytes; a column whose characters
 * outgrew the estimate is grown and decoded again), which must still be live */
int pq_decode_check(pq_ctx* ctx, pq_chunk* chunk);
int pq_column_copy_out(pq_ctx* ctx, const pq_column* col, uint32_t* validity, uint8_t* values,
                       int64_t* offsets);
void pq_column_free(pq_ctx* ctx, pq_column* col);

/* ── 4 KiB string chunker (the example driver's loop, src/main.cpp:17-32) ── */
/* Over a decoded BYTE_ARRAY column (pq_decode output; its non-NULL strings in
 * row order, as StringColumnIterator yields them, parquet_reader.cpp:282-473):
 * a chunk is closed before a string once it holds >= chunk_bytes bytes, each
 * string adding to_string(len).size() + len bytes.  Writes the chunk id of
 * every row (NULL rows 0: the zero-initialised std::vector<size_t>) to
 * d_tuple_to_chunk (device, num_rows int64; NULL = a context buffer) and,
 * when h_tuple_to_chunk is not NULL, copies it there; *num_chunks =
 * chunk_id + 1 as main.cpp prints it.  Synchronous. */
int pq_chunk_assign(pq_ctx* ctx, const pq_column* col, int64_t chunk_bytes, int64_t* d_tuple_to_chunk,
                    int64_t* h_tuple_to_chunk, int64_t* num_chunks);

/* ── regex page filter (README.md:54-64, SURVEY §8a R-REGEX) ───────────── */
/* page_flags[i] = 1 iff data page i of the chunk is REPORTED: no non-null
 * value matches (neg = 0) / no non-null value fails to match (neg = 1). */
int pq_regex_compile_check(const char* pattern, char* err, size_t errlen);
int pq_regex_pages(pq_ctx* ctx, pq_chunk* chunk, const char* pattern, int neg,
                   uint8_t* page_flags);
int pq_regex_pages_async(pq_ctx* ctx, pq_chunk* chunk, const char* pattern, int neg);
int pq_regex_pages_result(pq_ctx* ctx, pq_chunk* chunk, uint8_t* page_flags);
/* ColumnReader::read_all and the --regex-column filter of the same chunk in
 * one pass (the C5 shape: decode + filter): on dictionary chunks the pipe
 * takes (dictionary payload < 32 KiB), the pattern runs once per dictionary
 * entry and k_pipe_write tests every row's entry while it writes the column;
 * otherwise the decode, then
 * pq_regex_pages_async over its codes.  Results: pq_regex_pages_result for
 * the flags, pq_decode_check then pq_column_copy_out for the column. */
int pq_decode_regex_async(pq_ctx* ctx, pq_chunk* chunk, pq_column* out, const char* pattern, int neg);

/* ── kernel timing (HIP events on the context stream) ───────────────────── */
void pq_timing_enable(pq_ctx* ctx, int enable);
void pq_timing_reset(pq_ctx* ctx);
/* total milliseconds and launch count of kernel `name` since the last reset
 * (names: see DESIGN.md).  Returns 0 if unknown. */
int pq_timing_get(pq_ctx* ctx, const char* name, double* total_ms, int64_t* launches);
/* Per-phase shader-clock sums of the fused BYTE_ARRAY kernel, collected while
 * option "fused_prof" is 1 (diagnostics).  Copies up to n
 * counters into out, zeroes them, returns the number of counters. */
int pq_fused_prof_read(pq_ctx* ctx, uint64_t* out, int n);

/* ── file-level helpers (ParquetReader::open) ───────────────────────────── */
typedef struct pq_file pq_file;
int pq_file_open(const uint8_t* file, size_t file_len, pq_file** out, char* err, size_t errlen);
void pq_file_close(pq_file* f);
int64_t pq_file_num_rows(const pq_file* f);
int pq_file_num_row_groups(const pq_file* f);
int pq_file_num_columns(const pq_file* f);
int pq_file_column_name(const pq_file* f, int col, char* buf, size_t buflen);
int pq_file_find_column(const pq_file* f, const char* name);
/* ColumnInfo (column_info.hpp:6-20): physical type, max levels, repetition
 * and converted type (-1 when the schema element has none). */
int pq_file_column_info(const pq_file* f, int col, int32_t* type, int16_t* max_def,
                        int16_t* max_rep, int32_t* repetition, int32_t* converted_type);
int pq_file_chunk(const pq_file* f, int row_group, int col, pq_chunk_desc* out);
int64_t pq_file_row_group_rows(const pq_file* f, int row_group);
/* build_page_index (parquet_reader.cpp:559-605): global data-page ids,
 * rg-major then column then page order; 4 int64 per page:
 * data_offset, data_size, row_group_idx, column_idx. */
int64_t pq_file_num_pages(const pq_file* f);
int pq_file_page_index(const pq_file* f, int64_t* entries, int64_t cap);

#ifdef __cplusplus
}
#endif
#endif
