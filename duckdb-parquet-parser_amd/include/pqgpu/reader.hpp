// reader.hpp — C++17 mirror of the reference reader API, decoding on MI355X.
//
// Same class names, signatures, argument meaning and error behaviour as
// sputnik89/duckdb-parquet-parser (include/reader/*.hpp), in namespace
// pqgpu, implemented above the C ABI of include/pq_gpu.h:
//   ColumnReader(ReadRangeFunc, const ColumnChunk&, ParquetType, max_def, max_rep)
//       read_all() / read_pages()            column_reader.hpp:19-42
//   ParquetReader::open / schema / read_column / read_column_by_idx /
//       page index / PageIterator / read_pages_chunk / column_iterator
//                                            parquet_reader.hpp:12-138
// plus the README's regex page filter (README.md:54-64):
//   ParquetReader::regex_pages(column, pattern, neg)
// Errors are std::runtime_error carrying the reference's message text
// (std::bad_optional_access where the reference throws it).
#pragma once
#include <cstdint>
#include <functional>
#include <memory>
#include <optional>
#include <stdexcept>
#include <string>
#include <tuple>
#include <utility>
#include <variant>
#include <vector>

struct pq_ctx;
struct pq_chunk;
struct pq_file;

namespace pqgpu {

enum class ParquetType : int32_t {
    BOOLEAN = 0, INT32 = 1, INT64 = 2, INT96 = 3, FLOAT = 4, DOUBLE = 5, BYTE_ARRAY = 6,
    FIXED_LEN_BYTE_ARRAY = 7
};
enum class PageType : int32_t { DATA_PAGE = 0, INDEX_PAGE = 1, DICTIONARY_PAGE = 2, DATA_PAGE_V2 = 3 };
enum class CompressionCodec : int32_t { UNCOMPRESSED = 0, SNAPPY = 1, GZIP = 2, LZO = 3, BROTLI = 4,
                                        LZ4 = 5, ZSTD = 6, LZ4_RAW = 7 };
enum class FieldRepetitionType : int32_t { REQUIRED = 0, OPTIONAL = 1, REPEATED = 2 };

// common.hpp:177-201
struct Value {
    bool is_null = true;
    std::variant<bool, int32_t, int64_t, float, double, std::string> data;
    static Value null() { return Value{true, {}}; }
    static Value from_bool(bool v) { return Value{false, v}; }
    static Value from_i32(int32_t v) { return Value{false, v}; }
    static Value from_i64(int64_t v) { return Value{false, v}; }
    static Value from_float(float v) { return Value{false, v}; }
    static Value from_double(double v) { return Value{false, v}; }
    static Value from_string(std::string v) { return Value{false, std::move(v)}; }
    std::string to_string() const;
};

// metadata.hpp:17-40 (fields the decode path reads)
struct ColumnMetaData {
    ParquetType type = ParquetType::INT32;
    CompressionCodec codec = CompressionCodec::UNCOMPRESSED;
    int64_t num_values = 0;
    int64_t total_uncompressed_size = 0;
    int64_t total_compressed_size = 0;  // 0: unknown (the chunk is read header by header)
    int64_t data_page_offset = 0;
    std::optional<int64_t> dictionary_page_offset;
};
struct ColumnChunk {
    int64_t file_offset = 0;
    std::optional<ColumnMetaData> meta_data;
};

// column_reader.hpp:10-17
using ReadRangeFunc = std::function<std::vector<uint8_t>(size_t, size_t)>;
struct PageResult {
    int page_num;
    PageType type;
    int32_t num_values;
    std::vector<Value> values;
};

// Device context shared by readers (one per GPU; not thread-safe, like the
// reference's ParquetReader).
class Device {
public:
    explicit Device(int device = 0);
    ~Device();
    Device(const Device&) = delete;
    Device& operator=(const Device&) = delete;
    pq_ctx* ctx() const { return ctx_; }
    static Device& default_device();
    static int count();  // visible HIP devices

private:
    pq_ctx* ctx_;
};

// Decoded column as device-independent host arrays (the columnar fast path:
// no std::vector<Value> materialisation).
// Host arrays whose resize leaves new elements uninitialised (the device
// copy writes them; a zero fill first would touch every page on one thread).
template <class T>
struct NoInitAlloc : std::allocator<T> {
    template <class U> struct rebind { using other = NoInitAlloc<U>; };
    NoInitAlloc() = default;
    template <class U> NoInitAlloc(const NoInitAlloc<U>&) noexcept {}
    template <class U> void construct(U* p) noexcept { ::new (static_cast<void*>(p)) U; }
    template <class U, class... A> void construct(U* p, A&&... a) { ::new (static_cast<void*>(p)) U(std::forward<A>(a)...); }
};
template <class T>
using HostVec = std::vector<T, NoInitAlloc<T>>;

struct HostColumn {
    ParquetType type = ParquetType::INT32;
    int64_t num_rows = 0;
    HostVec<uint32_t> validity;  // LSB-first bitmap
    HostVec<uint8_t> values;     // fixed-width values or chars
    HostVec<int64_t> offsets;    // BYTE_ARRAY: num_rows + 1
    bool valid(int64_t i) const { return (validity[i >> 5] >> (i & 31)) & 1u; }
    Value value(int64_t i) const;    // reference Value semantics (INT96 -> "INT96(hi:lo)")
};

// The API-parity std::vector<Value> of rows [a, b) of a decoded column
// (the slow path, multithreaded): contiguous row ranges on
// `threads` host threads (0: hardware_concurrency, at most 16), each
// constructing its rows' Values in place.
std::vector<Value> to_values(const HostColumn& h, int64_t a, int64_t b, unsigned threads = 0);
// Wall ms of the calling thread's last to_values, by phase (bench / api_check
// accounting): the storage reserve, its pages faulted in by the workers, the
// default construction (resize), the parallel fill (strings allocated here).
struct ToValuesPhases {
    double reserve_ms = 0, fault_ms = 0, resize_ms = 0, fill_ms = 0;
    unsigned threads = 0;
};
ToValuesPhases last_to_values_phases();
inline std::vector<Value> to_values(const HostColumn& h, unsigned threads = 0) { return to_values(h, 0, h.num_rows, threads); }

class ColumnReader {
public:
    ColumnReader(ReadRangeFunc read_range, const ColumnChunk& chunk, ParquetType type,
                 int16_t max_def_level, int16_t max_rep_level, Device& dev = Device::default_device());
    std::vector<Value> read_all();
    std::vector<PageResult> read_pages();
    HostColumn read_columnar();  // same decode, columnar result

private:
    ReadRangeFunc read_range_;
    const ColumnMetaData* meta_;
    ParquetType type_;
    int16_t max_def_level_, max_rep_level_;
    Device& dev_;
};

struct ColumnInfo {  // column_info.hpp:6-20
    std::string name;
    ParquetType type;
    int column_index;
    int16_t max_def_level;
    int16_t max_rep_level;
    std::optional<FieldRepetitionType> repetition;
    std::optional<int32_t> converted_type;
    bool is_required() const { return repetition && *repetition == FieldRepetitionType::REQUIRED; }
    bool is_optional() const { return repetition && *repetition == FieldRepetitionType::OPTIONAL; }
    bool is_repeated() const { return repetition && *repetition == FieldRepetitionType::REPEATED; }
};

struct PageIndexEntry {  // parquet_reader.hpp:12-17
    size_t data_offset, data_size, row_group_idx, column_idx;
};
struct RawPage {  // parquet_reader.hpp:19-24
    size_t page_id, row_group_idx, column_idx;
    std::vector<uint8_t> data;
};

class ParquetReader;

class PageIterator {  // parquet_reader.hpp:64-77
public:
    PageIterator(ParquetReader& reader, size_t start, size_t end);
    bool has_next() const;
    RawPage next();
    void reset();

private:
    ParquetReader& reader_;
    size_t start_, end_, current_;
};

class StringColumnIterator {  // parquet_reader.hpp:28-62 (non-NULL strings + global row)
public:
    bool has_next() const;
    std::tuple<size_t, size_t, const char*> next();

private:
    friend class ParquetReader;
    explicit StringColumnIterator(HostColumn col);
    void skip_nulls();
    HostColumn col_;
    int64_t row_ = 0;
};

class ParquetReader {  // parquet_reader.hpp:79-138
public:
    explicit ParquetReader(Device& dev = Device::default_device());
    ~ParquetReader();
    bool open(const std::string& filename);
    bool open_buffer(std::vector<uint8_t> bytes);

    size_t num_columns() const;
    int64_t num_rows() const;
    size_t num_row_groups() const;
    std::vector<std::string> column_names() const;
    const ColumnInfo& column(size_t col_idx) const;
    const ColumnInfo& column(const std::string& name) const;
    int find_column(const std::string& name) const;
    std::string schema_string() const;

    std::vector<Value> read_column(const std::string& col_name, size_t row_group_idx);
    std::vector<Value> read_column(const std::string& col_name);
    std::vector<Value> read_column_by_idx(int row_group_idx, int col_idx);
    HostColumn read_column_columnar(const std::string& col_name);
    // Page-range sharding over several devices (the global page
    // order of build_page_index, parquet_reader.cpp:559-605): every row
    // group's chunk is cut into byte-balanced data-page ranges
    // (pq_plan_page_ranges), one per device; one host thread per device
    // uploads and decodes its ranges (pq_chunk_upload_range: the range's pages
    // plus their dictionary page, no collective); the shards are joined in
    // page order.  Same result and errors as the one-device calls.
    HostColumn read_column_columnar(const std::string& col_name, const std::vector<Device*>& devices);
    std::vector<Value> read_column(const std::string& col_name, const std::vector<Device*>& devices);

    StringColumnIterator column_iterator(const std::string& col_name);
    // The example driver's chunk assignment (src/main.cpp:17-32) over
    // column_iterator(col_name), on the GPU: (tuple_to_chunk, chunk_id + 1).
    std::pair<std::vector<size_t>, size_t> chunk_assign(const std::string& col_name, size_t chunk_size = 4096);

    size_t num_pages() const;
    std::vector<uint8_t> read_page_data(size_t global_page_id) const;
    const PageIndexEntry& page_index_entry(size_t global_page_id) const;
    std::vector<uint8_t> read_pages_chunk(size_t start_page_id, size_t end_page_id, size_t max_bytes) const;
    PageIterator page_iterator();
    PageIterator page_iterator(size_t start_page_id, size_t end_page_id);

    size_t file_size() const { return data_.size(); }
    std::vector<uint8_t> read_range(size_t offset, size_t length);

    // README.md:54-64: global page ids (page index order) of `col_name`'s data
    // pages with no value matching `pattern` (neg: no value failing it).
    std::vector<size_t> regex_pages(const std::string& col_name, const std::string& pattern,
                                    bool neg = false);
    // The same page filter sharded over devices: each row group's
    // chunk cut into byte-balanced data-page ranges (pq_plan_page_ranges), one
    // host thread per device uploading its ranges (pq_chunk_upload_range) and
    // scanning them; the per-shard page flags are concatenated in page order
    // (no collective).  Same ids and the same first error as the one-device call.
    std::vector<size_t> regex_pages(const std::string& col_name, const std::string& pattern, bool neg,
                                    const std::vector<Device*>& devices);
    // Decode and page filter in one call per shard (pq_decode_regex_async: one
    // pass over dictionary pages when the pipe takes the chunk): the column as
    // read_column_columnar(col_name, devices) returns it, and the page ids as
    // regex_pages returns them.
    HostColumn read_column_regex(const std::string& col_name, const std::string& pattern, bool neg,
                                 const std::vector<Device*>& devices, std::vector<size_t>* page_ids);

private:
    HostColumn decode_column(int col_idx, int rg_first, int rg_count);
    HostColumn decode_column_on(Device& dev, int col_idx);
    // page ids of column col_idx's data pages flagged in `flags`: data_offsets
    // holds the payload offset of every data page, in walk order
    std::vector<size_t> flagged_page_ids(int col_idx, const std::vector<int64_t>& data_offsets,
                                         const std::vector<uint8_t>& flags) const;
    // one call per device over every row group's range of the column: regex
    // (decode: also the column) of the shards, joined in page order
    HostColumn sharded_scan(int col_idx, const std::string& pattern, bool neg, const std::vector<Device*>& devices,
                            bool want_col, std::vector<size_t>* page_ids, bool* walk_failed);
    Device& dev_;
    std::vector<uint8_t> data_;
    pq_file* file_ = nullptr;
    std::vector<ColumnInfo> columns_;
    std::vector<PageIndexEntry> page_index_;
};

}  // namespace pqgpu
