// format.hpp — host-side Parquet format layer (C++17, clean-room).
//
// Thrift compact decoding, footer structures, schema -> leaf columns with
// max levels, the column-chunk page walk and the global data-page index.
// Behaviour (not code) follows the reference:
//   ByteBuffer checks/messages     include/common.hpp:110-173
//   ThriftReader                   src/reader/thrift.cpp:6-119
//   footer structs                 src/reader/metadata.cpp:5-242
//   leaf columns / max levels      src/reader/parquet_reader.cpp:495-543
//   chunk walk                     src/reader/column_reader.cpp:18-71
//   data-page index                src/reader/parquet_reader.cpp:559-605
#pragma once
#include <array>
#include <cstddef>
#include <cstdint>
#include <functional>
#include <optional>
#include <stdexcept>
#include <string>
#include <memory>
#include <utility>
#include <vector>

#include "pq_gpu.h"

namespace pqfmt {

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

// Bounds-checked cursor; the message text matches the reference exception.
class Cursor {
public:
    Cursor(const uint8_t* d, size_t n) : d_(d), n_(n) {}
    void need(size_t k) const {
        if (p_ + k > n_)
            throw Error(PQ_ERR_BUFFER, "ByteBuffer: read beyond end (pos=" + std::to_string(p_) +
                                           " need=" + std::to_string(k) +
                                           " size=" + std::to_string(n_) + ")");
    }
    uint8_t byte() { need(1); return d_[p_++]; }
    const uint8_t* bytes(size_t k) { need(k); const uint8_t* q = d_ + p_; p_ += k; return q; }
    uint64_t varint();
    int64_t zigzag() { uint64_t u = varint(); return static_cast<int64_t>((u >> 1) ^ (~(u & 1) + 1)); }
    size_t pos() const { return p_; }
    size_t size() const { return n_; }

private:
    const uint8_t* d_;
    size_t n_, p_ = 0;
};

class Thrift {
public:
    Thrift(const uint8_t* d, size_t n) : c_(d, n) {}
    // returns false at STOP
    bool field(int16_t& id, uint8_t& type);
    int32_t i32() { return static_cast<int32_t>(c_.zigzag()); }
    int64_t i64() { return c_.zigzag(); }
    std::string str();
    void list(uint8_t& et, int32_t& n);
    void push() { stack_.push_back(last_); last_ = 0; }
    void pop() { last_ = stack_.back(); stack_.pop_back(); }
    void skip(uint8_t type);
    size_t pos() const { return c_.pos(); }

private:
    Cursor c_;
    int16_t last_ = 0;
    std::vector<int16_t> stack_;
};

struct SchemaElement {
    std::optional<int32_t> type, type_length, repetition, num_children, converted_type, scale,
        precision, field_id;
    std::string name;
};
struct ColumnMeta {
    int32_t type = PQ_INT32;
    std::vector<int32_t> encodings;
    std::vector<std::string> path;
    int32_t codec = 0;
    int64_t num_values = 0, total_uncompressed = 0, total_compressed = 0, data_page_offset = 0;
    std::optional<int64_t> index_page_offset, dictionary_page_offset;
};
struct ColumnChunkMeta {
    std::optional<std::string> file_path;
    int64_t file_offset = 0;
    std::optional<ColumnMeta> meta;
};
struct RowGroupMeta {
    std::vector<ColumnChunkMeta> columns;
    int64_t total_byte_size = 0, num_rows = 0;
};
struct FileMeta {
    int32_t version = 0;
    std::vector<SchemaElement> schema;
    int64_t num_rows = 0;
    std::vector<RowGroupMeta> row_groups;
    std::optional<std::string> created_by;
};
struct LeafColumn {
    std::string name;
    int32_t type = PQ_BYTE_ARRAY;
    int column_index = 0;
    int16_t max_def = 0, max_rep = 0;
    std::optional<int32_t> repetition, converted_type;
};

// Parses "PAR1 ... footer len PAR1" (parquet_reader.cpp:14-61).
FileMeta parse_footer(const uint8_t* file, size_t len);
std::vector<LeafColumn> leaf_columns(const FileMeta& fm);

struct PageHeader {
    int32_t type = 0, uncompressed = 0, compressed = 0;
    bool has_data = false, has_dict = false;
    int32_t data_num_values = 0, data_encoding = 0;
    int32_t dict_num_values = 0;
    // DataPageHeaderV2 (field 8; the reference skips it): read for extended walks
    bool has_v2 = false, v2_compressed = true;
    int32_t v2_num_values = 0, v2_encoding = 0, v2_def_len = 0, v2_rep_len = 0;
    size_t header_size = 0;
};
// Parses a header from the 256-byte window at `off` (zeros past EOF).
PageHeader read_page_header(const uint8_t* file, size_t len, size_t off);

// Allocator whose resize leaves trivially constructible elements
// uninitialised (page tables are filled in parallel right after; no serial
// zero fill of tens of MB).
template <class T>
struct NoInitAlloc : std::allocator<T> {
    template <class U>
    struct rebind { using other = NoInitAlloc<U>; };
    NoInitAlloc() = default;
    template <class U>
    NoInitAlloc(const NoInitAlloc<U>&) noexcept {}
    template <class U>
    void construct(U* p) noexcept { ::new (static_cast<void*>(p)) U; }
    template <class U, class... A>
    void construct(U* p, A&&... a) { ::new (static_cast<void*>(p)) U(std::forward<A>(a)...); }
};
using PageList = std::vector<pq_page_desc, NoInitAlloc<pq_page_desc>>;

struct WalkResult {
    PageList pages;
    int error = 0;            // first error met by the walk (after `pages`)
    std::string message;
};
// ColumnReader::read_all's walk (column_reader.cpp:18-71): every page until
// Σ DATA_PAGE num_values >= chunk num_values; unknown pages are skipped.
// pq_chunk_desc.ext_flags widen it (pq_gpu.h PQ_EXT_*): compressed chunks,
// and DATA_PAGE_V2 pages walked as data pages (flags PQ_PAGE_V2).
// Chunks of at least kSpecMinBytes (pq_chunk_desc.total_compressed_size)
// walk speculatively on `threads` host threads (0 = up to 16; at most one
// per MiB), with results
// identical to the serial walk.
constexpr int64_t kSpecMinBytes = 4 << 20;
// fn(0 .. n-1) on up to `threads` threads (the caller and a process-wide pool
// of host workers, created once, so a walk does not pay a thread spawn per
// call); a call that finds the pool busy (another host thread's walk) uses
// fresh threads instead.
void parallel_run(int n, int threads, const std::function<void(int)>& fn);
WalkResult walk_chunk(const uint8_t* file, size_t len, const pq_chunk_desc& c, int threads = 0);

// build_page_index: (data_offset, data_size, rg, col) per data page.
std::vector<std::array<int64_t, 4>> page_index(const uint8_t* file, size_t len, const FileMeta& fm);

}  // namespace pqfmt
