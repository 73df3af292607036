/*
 * pq_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C restatement of the reference's column-chunk decode path
 * (sputnik89/duckdb-parquet-parser `ColumnReader::read_all` / `read_pages`,
 * src/reader/column_reader.cpp:18-276, and `RleDecoder`,
 * include/reader/rle_decoder.hpp:6-108).  It is the parity CHECKER for the
 * HIP product path: only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.  The product library never links it.
 *
 * Pinning: checked against the compiled reference (oracle/_ref, built from
 * the reference sources where they lie) on every fixture in tests/golden/.
 */
#ifndef PQ_ORACLE_H
#define PQ_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ColumnMetaData fields the decode path reads (metadata.hpp:17-28). */
typedef struct {
    int64_t num_values;             /* ColumnMetaData.num_values            */
    int64_t data_page_offset;       /* ColumnMetaData.data_page_offset      */
    int64_t dictionary_page_offset; /* valid when has_dictionary_page_offset */
    int32_t has_dictionary_page_offset;
    int32_t codec;                  /* CompressionCodec                     */
    int32_t type;                   /* ParquetType of the leaf column       */
    int16_t max_def_level;
    int16_t max_rep_level;
} pqo_chunk;

/* One entry per PageResult of read_pages() (column_reader.hpp:12-17). */
typedef struct {
    int32_t page_num;
    int32_t page_type;   /* PageType */
    int32_t num_values;  /* header num_values (dict header for dict pages) */
    int64_t first_row;   /* first output row of this page (data pages)    */
    int64_t nrows;       /* values produced (0 for dictionary pages)      */
} pqo_page;

/*
 * Columnar result.  Every type lands in the same shape:
 *   valid[i]      1 = non-null, 0 = NULL
 *   offsets[i]    byte offset of row i's payload in data[] (nrows+1 entries)
 *   data          concatenated payload: fixed-width types as their LE bytes
 *                 (BOOLEAN one byte 0/1), BYTE_ARRAY / INT96 as the string
 *                 bytes the reference's Value would hold.  NULL rows are empty.
 */
typedef struct {
    int64_t nrows;
    int32_t type;
    uint8_t* valid;
    int64_t* offsets;
    uint8_t* data;
    int64_t data_len;
    pqo_page* pages;
    int32_t npages;
} pqo_column;

/* Error codes (negative).  Messages follow the reference's exception text. */
enum {
    PQO_OK = 0,
    PQO_ERR_CODEC = -1,        /* "Only uncompressed parquet files are supported" */
    PQO_ERR_BUFFER = -2,       /* "ByteBuffer: read beyond end (...)"             */
    PQO_ERR_OPTIONAL = -3,     /* std::bad_optional_access                        */
    PQO_ERR_FLBA = -4,         /* FIXED_LEN_BYTE_ARRAY not supported ...          */
    PQO_ERR_TYPE = -5,         /* "Unsupported type: N"                           */
    PQO_ERR_THRIFT = -6,       /* ThriftReader::skip: unknown type / varint       */
    PQO_ERR_ALLOC = -7,        /* negative sizes / allocation failure             */
    PQO_ERR_UNSUPPORTED = -8   /* outside the parity scope (documented UB)        */
};

/* file[0..file_len) is the whole Parquet file; reads past its end see zeros
 * (the in-memory, zero-padding ReadRangeFunc of SURVEY §8c). */
int pqo_read_all(const uint8_t* file, size_t file_len, const pqo_chunk* c,
                 pqo_column* out, char* err, size_t errlen);
void pqo_free(pqo_column* col);

/* Canonical dump (SURVEY §8 header): per row u8 is_null, then for non-null
 * fixed-width types the raw LE bytes, for BYTE_ARRAY/INT96 u32 len + bytes. */
int pqo_dump(const pqo_column* col, uint8_t** out, size_t* out_len);
void pqo_free_buf(void* p);

/* Standalone hybrid RLE/bit-packed decoder (rle_decoder.hpp:17-34).  Writes
 * `count` values, zero-filling after exhaustion, truncated like the
 * reference's static_cast<int32_t>. */
int pqo_rle_decode(const uint8_t* data, uint32_t size, uint32_t bit_width,
                   int32_t* out, uint32_t count);

/* The example driver's 4 KiB chunker (src/main.cpp:17-32) over a decoded
 * BYTE_ARRAY column: non-NULL strings in row order, a chunk closed before a
 * string once it holds >= chunk_size bytes, each string adding
 * to_string(len).size() + len bytes.  out[row] = chunk id (NULL rows 0);
 * *num_chunks = chunk_id + 1 as main.cpp prints it. */
void pqo_chunk_assign(const uint8_t* valid, const int64_t* offsets, int64_t nrows,
                      int64_t chunk_size, int64_t* out, int64_t* num_chunks);

#ifdef __cplusplus
}
#endif
#endif
