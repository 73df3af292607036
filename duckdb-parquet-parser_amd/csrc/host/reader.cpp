// reader.cpp — the C++ reader API (include/pqgpu/reader.hpp) over the C ABI.
#include <sys/mman.h>
#include "pqgpu/reader.hpp"

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <thread>
#include <fstream>
#include <iostream>
#include <sstream>

#include "host/format.hpp"
#include "pq_gpu.h"

namespace pqgpu {

namespace {

[[noreturn]] void raise(int code, const std::string& msg) {
    if (code == PQ_ERR_OPTIONAL) throw std::bad_optional_access();
    throw std::runtime_error(msg);
}

const char* type_name(ParquetType t) {  // common.hpp:205-217
    switch (t) {
        case ParquetType::BOOLEAN: return "BOOLEAN";
        case ParquetType::INT32: return "INT32";
        case ParquetType::INT64: return "INT64";
        case ParquetType::INT96: return "INT96";
        case ParquetType::FLOAT: return "FLOAT";
        case ParquetType::DOUBLE: return "DOUBLE";
        case ParquetType::BYTE_ARRAY: return "BYTE_ARRAY";
        case ParquetType::FIXED_LEN_BYTE_ARRAY: return "FIXED_LEN_BYTE_ARRAY";
        default: return "UNKNOWN";
    }
}

// Storage of large host vectors on transparent huge pages: a 2 MiB fault
// instead of 512 4 KiB ones (and a faster unmap when freed); a no-op where
// THP is off or the range holds no whole huge page.
static void advise_huge(const void* p, size_t bytes) {
    constexpr uintptr_t kHuge = uintptr_t{2} << 20;
    const uintptr_t b = reinterpret_cast<uintptr_t>(p), e = b + bytes;
    const uintptr_t hb = (b + kHuge - 1) & ~(kHuge - 1), he = e & ~(kHuge - 1);
    if (he > hb) (void)madvise(reinterpret_cast<void*>(hb), he - hb, MADV_HUGEPAGE);
}
template <class V>
static void resize_huge(V& v, size_t n) {
    v.reserve(n);
    advise_huge(v.data(), n * sizeof(typename V::value_type));
    v.resize(n);
}

// Decode `descs` (chunks of one column) on `dev`; returns host arrays and
// optionally the walked page list.
HostColumn decode_chunks(Device& dev, const uint8_t* file, size_t len, const std::vector<pq_chunk_desc>& descs,
                         std::vector<pq_page_desc>* walked) {
    pq_ctx* ctx = dev.ctx();
    pq_chunk* ch = nullptr;
    int rc = pq_chunk_upload(ctx, file, len, descs.data(), static_cast<int>(descs.size()), &ch);
    if (rc) raise(rc, pq_last_error(ctx));
    pq_column out{};
    rc = pq_decode(ctx, ch, &out);
    if (rc) {
        std::string msg = pq_last_error(ctx);
        pq_column_free(ctx, &out);
        pq_chunk_free(ctx, ch);
        raise(rc, msg);
    }
    HostColumn h;
    h.type = static_cast<ParquetType>(out.type);
    h.num_rows = out.num_rows;
    h.validity.resize(static_cast<size_t>((out.num_rows + 31) / 32) + 1);
    h.validity.back() = 0;  // (the copy fills the others)
    resize_huge(h.values, static_cast<size_t>(std::max<int64_t>(out.num_bytes, 1)));
    if (out.type == PQ_BYTE_ARRAY) resize_huge(h.offsets, static_cast<size_t>(out.num_rows + 1));
    rc = pq_column_copy_out(ctx, &out, h.validity.data(), h.values.data(),
                            h.offsets.empty() ? nullptr : h.offsets.data());
    h.values.resize(static_cast<size_t>(out.num_bytes));
    if (walked) {
        int64_t n = 0;
        pq_chunk_pages(ch, nullptr, 0, &n);
        walked->resize(static_cast<size_t>(n));
        pq_chunk_pages(ch, walked->data(), n, &n);
    }
    pq_column_free(ctx, &out);
    pq_chunk_free(ctx, ch);
    if (rc) raise(rc, "device copy failed");
    return h;
}

// Shard `b`..`e` (data-page ordinals) of one chunk on `dev`.
HostColumn decode_range(Device& dev, const uint8_t* file, size_t len, const pq_chunk_desc& desc,
                        const std::vector<pq_page_desc>& table, int64_t b, int64_t e) {
    pq_ctx* ctx = dev.ctx();
    pq_chunk* ch = nullptr;
    int rc = pq_chunk_upload_range(ctx, file, len, &desc, table.data(), static_cast<int64_t>(table.size()), b, e, &ch);
    if (rc) raise(rc, pq_last_error(ctx));
    pq_column out{};
    rc = pq_decode(ctx, ch, &out);
    if (rc) {
        std::string msg = pq_last_error(ctx);
        pq_column_free(ctx, &out);
        pq_chunk_free(ctx, ch);
        raise(rc, msg);
    }
    HostColumn h;
    h.type = static_cast<ParquetType>(desc.type);
    h.num_rows = out.num_rows;
    h.validity.resize(static_cast<size_t>((out.num_rows + 31) / 32) + 1);
    h.validity.back() = 0;  // (the copy fills the others)
    h.values.resize(static_cast<size_t>(std::max<int64_t>(out.num_bytes, 1)));
    if (desc.type == PQ_BYTE_ARRAY) h.offsets.resize(static_cast<size_t>(out.num_rows + 1));
    rc = pq_column_copy_out(ctx, &out, h.validity.data(), h.values.data(),
                            h.offsets.empty() ? nullptr : h.offsets.data());
    h.values.resize(static_cast<size_t>(out.num_bytes));
    pq_column_free(ctx, &out);
    pq_chunk_free(ctx, ch);
    if (rc) raise(rc, "device copy failed");
    return h;
}

// Shard b..e of one chunk on `dev`: the page filter's flags of its data pages
// (`pattern` set), the decoded column (`col` set), or both in one call.
void scan_range(Device& dev, const uint8_t* file, size_t len, const pq_chunk_desc& desc,
                const std::vector<pq_page_desc>& table, int64_t b, int64_t e, const std::string* pattern, bool neg,
                HostColumn* col, std::vector<uint8_t>* flags) {
    pq_ctx* ctx = dev.ctx();
    pq_chunk* ch = nullptr;
    int rc = pq_chunk_upload_range(ctx, file, len, &desc, table.data(), static_cast<int64_t>(table.size()), b, e, &ch);
    if (rc) raise(rc, pq_last_error(ctx));
    pq_column out{};
    auto fail = [&](int code) {
        std::string msg = pq_last_error(ctx);
        pq_column_free(ctx, &out);
        pq_chunk_free(ctx, ch);
        raise(code, msg);
    };
    flags->assign(static_cast<size_t>(std::max<int64_t>(pq_chunk_num_pages(ch), 1)), 0);
    if (col) {
        if ((rc = pq_decode_regex_async(ctx, ch, &out, pattern->c_str(), neg ? 1 : 0))) fail(rc);
        if ((rc = pq_regex_pages_result(ctx, ch, flags->data()))) fail(rc);
        if ((rc = pq_decode_check(ctx, ch))) fail(rc);
        col->type = static_cast<ParquetType>(desc.type);
        col->num_rows = out.num_rows;
        col->validity.resize(static_cast<size_t>((out.num_rows + 31) / 32) + 1);
        col->validity.back() = 0;  // (the copy fills the others)
        col->values.resize(static_cast<size_t>(std::max<int64_t>(out.num_bytes, 1)));
        if (desc.type == PQ_BYTE_ARRAY) col->offsets.resize(static_cast<size_t>(out.num_rows + 1));
        rc = pq_column_copy_out(ctx, &out, col->validity.data(), col->values.data(),
                                col->offsets.empty() ? nullptr : col->offsets.data());
        col->values.resize(static_cast<size_t>(out.num_bytes));
        if (rc) fail(rc);
    } else if ((rc = pq_regex_pages(ctx, ch, pattern->c_str(), neg ? 1 : 0, flags->data()))) {
        fail(rc);
    }
    flags->resize(static_cast<size_t>(pq_chunk_num_pages(ch)));
    pq_column_free(ctx, &out);
    pq_chunk_free(ctx, ch);
}

// a followed by b (rows, validity bits, values; offsets rebased)
void append_column(HostColumn& a, const HostColumn& b) {
    const int64_t n0 = a.num_rows, n = n0 + b.num_rows;
    a.validity.resize(static_cast<size_t>((n + 31) / 32) + 1, 0);
    for (int64_t i = 0; i < b.num_rows; i++)
        if (b.valid(i)) a.validity[static_cast<size_t>((n0 + i) >> 5)] |= 1u << ((n0 + i) & 31);
    const int64_t base = static_cast<int64_t>(a.values.size());
    a.values.insert(a.values.end(), b.values.begin(), b.values.end());
    if (a.type == ParquetType::BYTE_ARRAY) {
        if (a.offsets.empty()) a.offsets.push_back(0);
        for (int64_t i = 1; i <= b.num_rows; i++) a.offsets.push_back(base + b.offsets[static_cast<size_t>(i)]);
    }
    a.num_rows = n;
}

}  // namespace

int Device::count() { return pq_device_count(); }

std::string Value::to_string() const {  // common.hpp:189-200
    if (is_null) return "NULL";
    return std::visit(
        [](auto&& a) -> std::string {
            using T = std::decay_t<decltype(a)>;
            if constexpr (std::is_same_v<T, bool>) return a ? "true" : "false";
            else if constexpr (std::is_same_v<T, std::string>) return a;
            else return std::to_string(a);
        },
        data);
}

Value HostColumn::value(int64_t i) const {
    if (!valid(i)) return Value::null();
    switch (type) {
        case ParquetType::BOOLEAN: return Value::from_bool(values[i] != 0);
        case ParquetType::INT32: { int32_t v; std::memcpy(&v, &values[4 * i], 4); return Value::from_i32(v); }
        case ParquetType::INT64: { int64_t v; std::memcpy(&v, &values[8 * i], 8); return Value::from_i64(v); }
        case ParquetType::FLOAT: { float v; std::memcpy(&v, &values[4 * i], 4); return Value::from_float(v); }
        case ParquetType::DOUBLE: { double v; std::memcpy(&v, &values[8 * i], 8); return Value::from_double(v); }
        case ParquetType::INT96: {  // column_reader.cpp:257-264
            int64_t lo;
            int32_t hi;
            std::memcpy(&lo, &values[12 * i], 8);
            std::memcpy(&hi, &values[12 * i + 8], 4);
            return Value::from_string("INT96(" + std::to_string(hi) + ":" + std::to_string(lo) + ")");
        }
        case ParquetType::BYTE_ARRAY:
            return Value::from_string(std::string(reinterpret_cast<const char*>(values.data()) + offsets[i],
                                                  static_cast<size_t>(offsets[i + 1] - offsets[i])));
        default: return Value::null();
    }
}

namespace {
thread_local ToValuesPhases g_tv_phases;
double ms_since(std::chrono::steady_clock::time_point& t) {
    const auto n = std::chrono::steady_clock::now();
    const double r = std::chrono::duration<double, std::milli>(n - t).count();
    t = n;
    return r;
}
}  // namespace

ToValuesPhases last_to_values_phases() { return g_tv_phases; }

namespace {
unsigned value_threads(unsigned threads, int64_t n) {
    unsigned t = threads ? threads : std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    // (below ~64k rows a thread costs more than it saves)
    return static_cast<unsigned>(std::min<int64_t>(t, std::max<int64_t>(1, n / 65536)));
}

// `out` sized to n rows: the storage reserved, its pages faulted in by the
// workers (the default construction then runs over mapped memory instead of
// taking every page fault on this thread), then default-constructed.
void prepare_values(std::vector<Value>& out, int64_t n, unsigned t, ToValuesPhases& P) {
    auto tp = std::chrono::steady_clock::now();
    out.clear();
    out.reserve(static_cast<size_t>(n));
    advise_huge(out.data(), static_cast<size_t>(n) * sizeof(Value));  // (hundreds of MB for 10M values)
    P.reserve_ms = ms_since(tp);
    if (t > 1) {
        volatile char* raw = reinterpret_cast<volatile char*>(out.data());
        const size_t bytes = static_cast<size_t>(n) * sizeof(Value);
        std::vector<std::thread> th;
        for (unsigned k = 0; k < t; k++)
            th.emplace_back([=] {
                for (size_t o = bytes * k / t / 4096 * 4096; o < bytes * (k + 1) / t; o += 4096) raw[o] = 0;
            });
        for (auto& x : th) x.join();
    }
    P.fault_ms = ms_since(tp);
    out.resize(static_cast<size_t>(n));
    P.resize_ms = ms_since(tp);
}

// Rows [a, a + out.size()) of h into the default-constructed `out`, each
// Value built in place (the string constructed inside the variant: no
// temporary, no moves), on t threads over contiguous ranges.
void fill_values(const HostColumn& h, int64_t a, std::vector<Value>& out, unsigned t, ToValuesPhases& P) {
    auto tp = std::chrono::steady_clock::now();
    const int64_t n = static_cast<int64_t>(out.size());
    const bool ba = h.type == ParquetType::BYTE_ARRAY;
    auto part = [&](unsigned k) {
        const int64_t r0 = n * k / t, r1 = n * (k + 1) / t;
        if (ba) {
            const char* chars = reinterpret_cast<const char*>(h.values.data());
            for (int64_t r = r0; r < r1; r++) {
                const int64_t i = a + r;
                Value& v = out[static_cast<size_t>(r)];
                if (!h.valid(i)) continue;  // (default: NULL)
                v.is_null = false;
                v.data.template emplace<std::string>(chars + h.offsets[i], static_cast<size_t>(h.offsets[i + 1] - h.offsets[i]));
            }
        } else {
            for (int64_t r = r0; r < r1; r++) out[static_cast<size_t>(r)] = h.value(a + r);
        }
    };
    if (t <= 1) {
        part(0);
    } else {
        std::vector<std::thread> th;
        th.reserve(t - 1);
        for (unsigned k = 1; k < t; k++) th.emplace_back(part, k);
        part(0);
        for (auto& x : th) x.join();
    }
    P.fill_ms = ms_since(tp);
}
}  // namespace

std::vector<Value> to_values(const HostColumn& h, int64_t a, int64_t b, unsigned threads) {
    ToValuesPhases& P = g_tv_phases;
    P = ToValuesPhases{};
    a = std::max<int64_t>(a, 0);
    b = std::min<int64_t>(b, h.num_rows);
    const int64_t n = std::max<int64_t>(b - a, 0);
    const unsigned t = value_threads(threads, n);
    P.threads = t;
    std::vector<Value> out;
    prepare_values(out, n, t, P);
    fill_values(h, a, out, t, P);
    return out;
}

// ── Device ─────────────────────────────────────────────────────────────────
Device::Device(int device) : ctx_(pq_ctx_create(device)) {
    if (!ctx_) throw std::runtime_error("pqgpu: no HIP device " + std::to_string(device));
}
Device::~Device() { pq_ctx_destroy(ctx_); }
Device& Device::default_device() {
    static Device d(0);
    return d;
}

// ── ColumnReader ───────────────────────────────────────────────────────────
ColumnReader::ColumnReader(ReadRangeFunc read_range, const ColumnChunk& chunk, ParquetType type,
                           int16_t max_def_level, int16_t max_rep_level, Device& dev)
    : read_range_(std::move(read_range)), type_(type), max_def_level_(max_def_level),
      max_rep_level_(max_rep_level), dev_(dev) {
    if (!chunk.meta_data) throw std::runtime_error("ColumnChunk has no metadata");  // column_reader.cpp:9-11
    meta_ = &*chunk.meta_data;
    if (meta_->codec != CompressionCodec::UNCOMPRESSED)
        throw std::runtime_error("Only uncompressed parquet files are supported");
}

HostColumn ColumnReader::read_columnar() {
    // Fetch exactly the bytes the reference's walk touches (256-byte header
    // windows + payloads) through the caller's ReadRangeFunc, then hand one
    // contiguous image to the GPU path.
    int64_t start = meta_->data_page_offset;
    if (meta_->dictionary_page_offset) start = std::min(start, *meta_->dictionary_page_offset);
    size_t cur = static_cast<size_t>(start), end = cur;
    int64_t values_read = 0;
    // the chunk's extent per its metadata (+ one header window) in one read;
    // header windows outside it (a chain longer than the metadata says) come
    // from read_range_ as before, so the image holds the same bytes either way
    std::vector<uint8_t> big;
    if (meta_->total_compressed_size > 0)
        big = read_range_(static_cast<size_t>(start), static_cast<size_t>(meta_->total_compressed_size) + 256);
    std::vector<uint8_t> hdr;
    while (values_read < meta_->num_values) {
        const uint8_t* win;
        if (cur - static_cast<size_t>(start) + 256 <= big.size()) {
            win = big.data() + (cur - static_cast<size_t>(start));
        } else {
            hdr = read_range_(cur, 256);
            hdr.resize(256, 0);
            win = hdr.data();
        }
        pqfmt::PageHeader h;
        try {
            h = pqfmt::read_page_header(win, 256, 0);
        } catch (const pqfmt::Error&) {
            end = std::max(end, cur + 256);
            break;  // the GPU-side walk reports it at the same place
        }
        end = std::max(end, cur + 256);
        cur += h.header_size;
        if (h.compressed < 0) break;
        end = std::max(end, cur + static_cast<size_t>(h.compressed));
        if (h.type == 0 && h.has_data) values_read += h.data_num_values;
        else if (h.type == 0 || (h.type == 2 && !h.has_dict)) break;
        cur += static_cast<size_t>(h.compressed);
    }
    std::vector<uint8_t> image;
    if (end - static_cast<size_t>(start) <= big.size()) {
        big.resize(end - static_cast<size_t>(start));
        image = std::move(big);
    } else {
        image = read_range_(static_cast<size_t>(start), end - static_cast<size_t>(start));
    }
    pq_chunk_desc d{};
    d.num_values = meta_->num_values;
    d.data_page_offset = meta_->data_page_offset - start;
    d.has_dictionary_page_offset = meta_->dictionary_page_offset.has_value();
    d.dictionary_page_offset = meta_->dictionary_page_offset.value_or(start) - start;
    d.codec = static_cast<int32_t>(meta_->codec);
    d.type = static_cast<int32_t>(type_);
    d.max_def_level = max_def_level_;
    d.max_rep_level = max_rep_level_;
    return decode_chunks(dev_, image.data(), image.size(), {d}, nullptr);
}

// The Value vector is sized (allocated, faulted in, default-constructed) on a
// host thread while the chunk uploads and decodes on the GPU; the decoded
// column then fills it in place (to_values' phases, overlapped).
std::vector<Value> ColumnReader::read_all() {
    ToValuesPhases& P = g_tv_phases;
    P = ToValuesPhases{};
    const int64_t guess = std::max<int64_t>(meta_->num_values, 0);  // a flat column's rows
    const unsigned t = value_threads(0, guess);
    std::vector<Value> out;
    ToValuesPhases prep{};
    std::thread pre([&] { prepare_values(out, guess, t, prep); });
    HostColumn h;
    try {
        h = read_columnar();
    } catch (...) {
        pre.join();
        throw;
    }
    pre.join();
    P.reserve_ms = prep.reserve_ms;
    P.fault_ms = prep.fault_ms;
    P.resize_ms = prep.resize_ms;
    P.threads = value_threads(0, h.num_rows);
    if (static_cast<int64_t>(out.size()) != h.num_rows) out.resize(static_cast<size_t>(std::max<int64_t>(h.num_rows, 0)));
    fill_values(h, 0, out, P.threads, P);
    return out;
}

std::vector<PageResult> ColumnReader::read_pages() {
    int64_t start = meta_->data_page_offset;
    if (meta_->dictionary_page_offset) start = std::min(start, *meta_->dictionary_page_offset);
    HostColumn h = read_columnar();
    // re-walk on the host for the page records (same walk as the device upload)
    std::vector<uint8_t> img;
    std::vector<PageResult> pages;
    size_t cur = static_cast<size_t>(start);
    int64_t values_read = 0, row = 0;
    int page_num = 0;
    while (values_read < meta_->num_values) {
        std::vector<uint8_t> hdr = read_range_(cur, 256);
        hdr.resize(256, 0);
        pqfmt::PageHeader ph = pqfmt::read_page_header(hdr.data(), hdr.size(), 0);
        cur += ph.header_size;
        if (ph.type == 2) {
            pages.push_back({page_num++, PageType::DICTIONARY_PAGE, ph.dict_num_values, {}});
        } else if (ph.type == 0) {
            PageResult pr{page_num++, PageType::DATA_PAGE, ph.data_num_values, {}};
            pr.values = to_values(h, row, row + std::max(ph.data_num_values, 0));
            row += ph.data_num_values;
            values_read += ph.data_num_values;
            pages.push_back(std::move(pr));
        } else {
            page_num++;
        }
        cur += static_cast<size_t>(ph.compressed);
    }
    return pages;
}

// ── PageIterator / StringColumnIterator ────────────────────────────────────
PageIterator::PageIterator(ParquetReader& r, size_t s, size_t e) : reader_(r), start_(s), end_(e), current_(s) {}
bool PageIterator::has_next() const { return current_ < end_; }
RawPage PageIterator::next() {  // parquet_reader.cpp:247-259
    if (!has_next()) throw std::runtime_error("PageIterator: no more pages");
    const auto& e = reader_.page_index_entry(current_);
    RawPage p{current_, e.row_group_idx, e.column_idx, reader_.read_page_data(current_)};
    current_++;
    return p;
}
void PageIterator::reset() { current_ = start_; }

StringColumnIterator::StringColumnIterator(HostColumn col) : col_(std::move(col)) { skip_nulls(); }
void StringColumnIterator::skip_nulls() {
    while (row_ < col_.num_rows && !col_.valid(row_)) row_++;
}
bool StringColumnIterator::has_next() const { return row_ < col_.num_rows; }
std::tuple<size_t, size_t, const char*> StringColumnIterator::next() {
    if (!has_next()) throw std::runtime_error("StringColumnIterator: no more strings");
    int64_t i = row_++;
    skip_nulls();
    return {static_cast<size_t>(i), static_cast<size_t>(col_.offsets[i + 1] - col_.offsets[i]),
            reinterpret_cast<const char*>(col_.values.data()) + col_.offsets[i]};
}

// ── ParquetReader ──────────────────────────────────────────────────────────
ParquetReader::ParquetReader(Device& dev) : dev_(dev) {}
ParquetReader::~ParquetReader() { pq_file_close(file_); }

bool ParquetReader::open(const std::string& filename) {  // parquet_reader.cpp:14-61
    std::ifstream f(filename, std::ios::binary | std::ios::ate);
    if (!f.is_open()) {
        std::cerr << "Error: cannot open file " << filename << std::endl;
        return false;
    }
    std::vector<uint8_t> bytes(static_cast<size_t>(f.tellg()));
    f.seekg(0);
    f.read(reinterpret_cast<char*>(bytes.data()), static_cast<std::streamsize>(bytes.size()));
    return open_buffer(std::move(bytes));
}

bool ParquetReader::open_buffer(std::vector<uint8_t> bytes) {
    data_ = std::move(bytes);
    char err[512] = {0};
    pq_file_close(file_);
    file_ = nullptr;
    int rc = pq_file_open(data_.data(), data_.size(), &file_, err, sizeof err);
    if (rc == PQ_ERR_ARG) {
        std::cerr << "Error: " << err << std::endl;
        return false;
    }
    if (rc) raise(rc, err);
    columns_.clear();
    for (int c = 0; c < pq_file_num_columns(file_); c++) {
        char name[1024];
        pq_file_column_name(file_, c, name, sizeof name);
        int32_t type, rep, conv;
        int16_t md, mr;
        pq_file_column_info(file_, c, &type, &md, &mr, &rep, &conv);
        ColumnInfo ci{name, static_cast<ParquetType>(type), c, md, mr, std::nullopt, std::nullopt};
        if (rep >= 0) ci.repetition = static_cast<FieldRepetitionType>(rep);
        if (conv >= 0) ci.converted_type = conv;
        columns_.push_back(ci);
    }
    int64_t np = pq_file_num_pages(file_);
    std::vector<int64_t> e(static_cast<size_t>(4 * np));
    pq_file_page_index(file_, e.data(), np);
    page_index_.clear();
    for (int64_t i = 0; i < np; i++)
        page_index_.push_back({static_cast<size_t>(e[4 * i]), static_cast<size_t>(e[4 * i + 1]),
                               static_cast<size_t>(e[4 * i + 2]), static_cast<size_t>(e[4 * i + 3])});
    return true;
}

size_t ParquetReader::num_columns() const { return columns_.size(); }
int64_t ParquetReader::num_rows() const { return pq_file_num_rows(file_); }
size_t ParquetReader::num_row_groups() const { return static_cast<size_t>(pq_file_num_row_groups(file_)); }
std::vector<std::string> ParquetReader::column_names() const {
    std::vector<std::string> n;
    for (const auto& c : columns_) n.push_back(c.name);
    return n;
}
const ColumnInfo& ParquetReader::column(size_t i) const {
    if (i >= columns_.size()) throw std::runtime_error("Column index " + std::to_string(i) + " out of range");
    return columns_[i];
}
const ColumnInfo& ParquetReader::column(const std::string& name) const {
    int i = find_column(name);
    if (i < 0) throw std::runtime_error("Column not found: " + name);
    return columns_[static_cast<size_t>(i)];
}
int ParquetReader::find_column(const std::string& name) const { return pq_file_find_column(file_, name.c_str()); }

std::string ParquetReader::schema_string() const {  // parquet_reader.cpp:99-121
    std::ostringstream ss;
    ss << "Schema:\n";
    for (size_t i = 0; i < columns_.size(); i++) {
        const auto& c = columns_[i];
        ss << "  " << i << ": " << c.name << " (" << type_name(c.type);
        if (c.repetition) {
            switch (*c.repetition) {
                case FieldRepetitionType::REQUIRED: ss << ", REQUIRED"; break;
                case FieldRepetitionType::OPTIONAL: ss << ", OPTIONAL"; break;
                case FieldRepetitionType::REPEATED: ss << ", REPEATED"; break;
            }
        }
        ss << ")\n";
    }
    ss << "Rows: " << num_rows() << "\n";
    ss << "Row groups: " << num_row_groups() << "\n";
    return ss.str();
}

HostColumn ParquetReader::decode_column(int col_idx, int rg_first, int rg_count) {
    std::vector<pq_chunk_desc> descs;
    for (int rg = rg_first; rg < rg_first + rg_count; rg++) {
        pq_chunk_desc d{};
        int rc = pq_file_chunk(file_, rg, col_idx, &d);
        if (rc) raise(rc == PQ_ERR_OPTIONAL ? 0 : rc, "ColumnChunk has no metadata");
        if (d.codec != 0) throw std::runtime_error("Only uncompressed parquet files are supported");
        descs.push_back(d);
    }
    return decode_chunks(dev_, data_.data(), data_.size(), descs, nullptr);
}

std::vector<Value> ParquetReader::read_column_by_idx(int rg, int col) {  // parquet_reader.cpp:146-165
    if (rg < 0 || rg >= static_cast<int>(num_row_groups())) throw std::runtime_error("Invalid row group index");
    if (col < 0 || col >= static_cast<int>(columns_.size())) throw std::runtime_error("Invalid column index");
    return to_values(decode_column(col, rg, 1));
}
std::vector<Value> ParquetReader::read_column(const std::string& name, size_t rg) {
    int c = find_column(name);
    if (c < 0) throw std::runtime_error("Column not found: " + name);
    return read_column_by_idx(static_cast<int>(rg), c);
}
HostColumn ParquetReader::read_column_columnar(const std::string& name) {
    int c = find_column(name);
    if (c < 0) throw std::runtime_error("Column not found: " + name);
    return decode_column(c, 0, static_cast<int>(num_row_groups()));
}
HostColumn ParquetReader::read_column_columnar(const std::string& name, const std::vector<Device*>& devices) {
    int c = find_column(name);
    if (c < 0) throw std::runtime_error("Column not found: " + name);
    const int nrg = static_cast<int>(num_row_groups());
    const int D = static_cast<int>(devices.size());
    if (D <= 1) return D == 1 ? decode_column_on(*devices[0], c) : read_column_columnar(name);
    std::vector<pq_chunk_desc> descs(static_cast<size_t>(nrg));
    std::vector<std::vector<pq_page_desc>> tables(static_cast<size_t>(nrg));
    std::vector<std::vector<int64_t>> plans(static_cast<size_t>(nrg), std::vector<int64_t>(2 * static_cast<size_t>(D)));
    for (int rg = 0; rg < nrg; rg++) {
        pq_chunk_desc& d = descs[static_cast<size_t>(rg)];
        int rc = pq_file_chunk(file_, rg, c, &d);
        if (rc) raise(rc == PQ_ERR_OPTIONAL ? 0 : rc, "ColumnChunk has no metadata");
        if (d.codec != 0) throw std::runtime_error("Only uncompressed parquet files are supported");
        // the chunk's page table (host walk), grown until it holds every page
        std::vector<pq_page_desc>& t = tables[static_cast<size_t>(rg)];
        int64_t n = 0;
        t.resize(1024);
        for (;;) {
            rc = pq_build_page_table(data_.data(), data_.size(), &d, t.data(), static_cast<int64_t>(t.size()), &n,
                                     nullptr, 0);
            if (n <= static_cast<int64_t>(t.size())) break;
            t.resize(static_cast<size_t>(n));
        }
        t.resize(static_cast<size_t>(n));
        // a walk error: the one-device path reports it exactly as the reference
        if (rc) return decode_column_on(*devices[0], c);
        pq_plan_page_ranges(t.data(), n, D, plans[static_cast<size_t>(rg)].data());
    }
    // one host thread per device: its range of every row group, in order
    std::vector<std::vector<HostColumn>> parts(static_cast<size_t>(D), std::vector<HostColumn>(static_cast<size_t>(nrg)));
    std::vector<std::exception_ptr> errs(static_cast<size_t>(D) * static_cast<size_t>(nrg));
    std::vector<std::thread> th;
    for (int k = 0; k < D; k++) {
        th.emplace_back([&, k]() {
            for (int rg = 0; rg < nrg; rg++) {
                const auto& pl = plans[static_cast<size_t>(rg)];
                try {
                    parts[static_cast<size_t>(k)][static_cast<size_t>(rg)] =
                        decode_range(*devices[static_cast<size_t>(k)], data_.data(), data_.size(),
                                     descs[static_cast<size_t>(rg)], tables[static_cast<size_t>(rg)],
                                     pl[2 * static_cast<size_t>(k)], pl[2 * static_cast<size_t>(k) + 1]);
                } catch (...) {
                    errs[static_cast<size_t>(rg) * D + k] = std::current_exception();
                    return;  // (later row groups of this device are never reached by the reference)
                }
            }
        });
    }
    for (auto& x : th) x.join();
    // the first error in page order (row group, then shard) is the reference's first error
    for (auto& e : errs)
        if (e) std::rethrow_exception(e);
    HostColumn out;
    out.type = columns_[static_cast<size_t>(c)].type;
    for (int rg = 0; rg < nrg; rg++)
        for (int k = 0; k < D; k++) append_column(out, parts[static_cast<size_t>(k)][static_cast<size_t>(rg)]);
    if (out.type == ParquetType::BYTE_ARRAY && out.offsets.empty()) out.offsets.push_back(0);
    out.validity.resize(static_cast<size_t>((out.num_rows + 31) / 32) + 1, 0);
    return out;
}

std::vector<Value> ParquetReader::read_column(const std::string& name, const std::vector<Device*>& devices) {
    return to_values(read_column_columnar(name, devices));
}

HostColumn ParquetReader::decode_column_on(Device& dev, int col_idx) {
    std::vector<pq_chunk_desc> descs;
    for (int rg = 0; rg < static_cast<int>(num_row_groups()); rg++) {
        pq_chunk_desc d{};
        int rc = pq_file_chunk(file_, rg, col_idx, &d);
        if (rc) raise(rc == PQ_ERR_OPTIONAL ? 0 : rc, "ColumnChunk has no metadata");
        if (d.codec != 0) throw std::runtime_error("Only uncompressed parquet files are supported");
        descs.push_back(d);
    }
    return decode_chunks(dev, data_.data(), data_.size(), descs, nullptr);
}

std::vector<Value> ParquetReader::read_column(const std::string& name) {  // parquet_reader.cpp:125-144
    return to_values(read_column_columnar(name));
}

StringColumnIterator ParquetReader::column_iterator(const std::string& name) {  // parquet_reader.cpp:282-295
    int c = find_column(name);
    if (c < 0) throw std::runtime_error("Column not found: " + name);
    if (columns_[c].type != ParquetType::BYTE_ARRAY)
        throw std::runtime_error("Column '" + name + "' is not BYTE_ARRAY (type: " + type_name(columns_[c].type) + ")");
    return StringColumnIterator(decode_column(c, 0, static_cast<int>(num_row_groups())));
}

// The example driver's 4 KiB chunker (main.cpp:17-32) over column_iterator's
// strings, on the device: tuple_to_chunk (num_rows, NULL rows 0) and the chunk
// count main.cpp prints (chunk_id + 1).
std::pair<std::vector<size_t>, size_t> ParquetReader::chunk_assign(const std::string& name, size_t chunk_size) {
    int c = find_column(name);
    if (c < 0) throw std::runtime_error("Column not found: " + name);
    if (columns_[c].type != ParquetType::BYTE_ARRAY)
        throw std::runtime_error("Column '" + name + "' is not BYTE_ARRAY (type: " + type_name(columns_[c].type) + ")");
    std::vector<pq_chunk_desc> descs;
    for (int rg = 0; rg < static_cast<int>(num_row_groups()); rg++) {
        pq_chunk_desc d{};
        int rc = pq_file_chunk(file_, rg, c, &d);
        if (rc) raise(rc == PQ_ERR_OPTIONAL ? 0 : rc, "ColumnChunk has no metadata");
        descs.push_back(d);
    }
    std::pair<std::vector<size_t>, size_t> res;
    if (descs.empty()) {
        res.second = 1;
        return res;
    }
    pq_ctx* ctx = dev_.ctx();
    pq_chunk* ch = nullptr;
    int rc = pq_chunk_upload(ctx, data_.data(), data_.size(), descs.data(), static_cast<int>(descs.size()), &ch);
    if (rc) raise(rc, pq_last_error(ctx));
    pq_column out{};
    rc = pq_decode(ctx, ch, &out);
    std::vector<int64_t> ids(static_cast<size_t>(std::max<int64_t>(out.num_rows, 0)));
    int64_t nchunks = 1;
    if (!rc) rc = pq_chunk_assign(ctx, &out, static_cast<int64_t>(chunk_size), nullptr, ids.data(), &nchunks);
    std::string msg = rc ? pq_last_error(ctx) : "";
    pq_column_free(ctx, &out);
    pq_chunk_free(ctx, ch);
    if (rc) raise(rc, msg);
    res.first.assign(ids.begin(), ids.end());
    res.second = static_cast<size_t>(nchunks);
    return res;
}

size_t ParquetReader::num_pages() const { return page_index_.size(); }
std::vector<uint8_t> ParquetReader::read_range(size_t off, size_t len) {
    std::vector<uint8_t> b(len, 0);
    if (off < data_.size()) std::memcpy(b.data(), data_.data() + off, std::min(len, data_.size() - off));
    return b;
}
const PageIndexEntry& ParquetReader::page_index_entry(size_t id) const {
    if (id >= page_index_.size()) throw std::runtime_error("Global page ID " + std::to_string(id) + " out of range");
    return page_index_[id];
}
std::vector<uint8_t> ParquetReader::read_page_data(size_t id) const {
    const auto& e = page_index_entry(id);
    return const_cast<ParquetReader*>(this)->read_range(e.data_offset, e.data_size);
}
std::vector<uint8_t> ParquetReader::read_pages_chunk(size_t s, size_t e, size_t max_bytes) const {  // 194-231
    if (s >= page_index_.size()) throw std::runtime_error("Start page ID " + std::to_string(s) + " out of range");
    if (e >= page_index_.size()) throw std::runtime_error("End page ID " + std::to_string(e) + " out of range");
    if (s > e) throw std::runtime_error("Start page ID must be <= end page ID");
    std::vector<uint8_t> out;
    for (size_t i = s; i <= e; i++) {
        size_t rem = max_bytes - out.size();
        if (rem == 0) break;
        const auto& en = page_index_[i];
        auto d = const_cast<ParquetReader*>(this)->read_range(en.data_offset, std::min(en.data_size, rem));
        out.insert(out.end(), d.begin(), d.end());
    }
    return out;
}
PageIterator ParquetReader::page_iterator() { return PageIterator(*this, 0, page_index_.size()); }
PageIterator ParquetReader::page_iterator(size_t s, size_t e) {  // 261-278
    if (s > page_index_.size()) throw std::runtime_error("start_page_id out of range");
    if (e > page_index_.size()) throw std::runtime_error("end_page_id out of range");
    if (s > e) throw std::runtime_error("start_page_id must be <= end_page_id");
    return PageIterator(*this, s, e);
}

std::vector<size_t> ParquetReader::regex_pages(const std::string& name, const std::string& pattern, bool neg) {
    int c = find_column(name);
    if (c < 0) throw std::runtime_error("Column not found: " + name);
    std::vector<pq_chunk_desc> descs;
    for (int rg = 0; rg < static_cast<int>(num_row_groups()); rg++) {
        pq_chunk_desc d{};
        if (int rc = pq_file_chunk(file_, rg, c, &d)) raise(rc, "ColumnChunk has no metadata");
        descs.push_back(d);
    }
    pq_ctx* ctx = dev_.ctx();
    pq_chunk* ch = nullptr;
    if (int rc = pq_chunk_upload(ctx, data_.data(), data_.size(), descs.data(), static_cast<int>(descs.size()), &ch))
        raise(rc, pq_last_error(ctx));
    std::vector<uint8_t> flags(static_cast<size_t>(std::max<int64_t>(pq_chunk_num_pages(ch), 1)));
    int rc = pq_regex_pages(ctx, ch, pattern.c_str(), neg ? 1 : 0, flags.data());
    std::string msg = rc ? pq_last_error(ctx) : "";
    int64_t nw = 0;
    pq_chunk_pages(ch, nullptr, 0, &nw);
    std::vector<pq_page_desc> walked(static_cast<size_t>(nw));
    pq_chunk_pages(ch, walked.data(), nw, &nw);
    pq_chunk_free(ctx, ch);
    if (rc) raise(rc, msg);
    std::vector<int64_t> offs;
    for (const auto& p : walked)
        if (p.page_type == PQ_DATA_PAGE) offs.push_back(p.payload_offset);
    return flagged_page_ids(c, offs, flags);
}

std::vector<size_t> ParquetReader::regex_pages(const std::string& name, const std::string& pattern, bool neg,
                                               const std::vector<Device*>& devices) {
    int c = find_column(name);
    if (c < 0) throw std::runtime_error("Column not found: " + name);
    if (devices.size() <= 1 || num_row_groups() == 0) return regex_pages(name, pattern, neg);
    std::vector<size_t> ids;
    bool walk_failed = false;
    sharded_scan(c, pattern, neg, devices, false, &ids, &walk_failed);
    if (walk_failed) return regex_pages(name, pattern, neg);
    return ids;
}

HostColumn ParquetReader::read_column_regex(const std::string& name, const std::string& pattern, bool neg,
                                            const std::vector<Device*>& devices, std::vector<size_t>* page_ids) {
    int c = find_column(name);
    if (c < 0) throw std::runtime_error("Column not found: " + name);
    if (columns_[static_cast<size_t>(c)].type != ParquetType::BYTE_ARRAY)
        throw std::runtime_error("regex page filter needs a BYTE_ARRAY column");
    std::vector<size_t> ids;
    HostColumn out;
    bool walk_failed = devices.empty() || num_row_groups() == 0;
    if (!walk_failed) out = sharded_scan(c, pattern, neg, devices, true, &ids, &walk_failed);
    if (walk_failed) {  // the one-device calls report the walk's error the reference's way
        out = read_column_columnar(name);
        ids = regex_pages(name, pattern, neg);
    }
    if (page_ids) *page_ids = std::move(ids);
    return out;
}

std::vector<size_t> ParquetReader::flagged_page_ids(int col_idx, const std::vector<int64_t>& data_offsets,
                                                    const std::vector<uint8_t>& flags) const {
    // device data page k <-> the k-th DATA_PAGE of the walks <-> its global id
    std::vector<size_t> out;
    size_t k = 0, gid = 0;
    const int chunk_col = columns_[static_cast<size_t>(col_idx)].column_index;
    std::vector<size_t> ids;
    for (size_t i = 0; i < page_index_.size(); i++)
        if (static_cast<int>(page_index_[i].column_idx) == chunk_col) ids.push_back(i);
    for (const int64_t off : data_offsets) {
        while (gid < ids.size() && page_index_[ids[gid]].data_offset != static_cast<size_t>(off)) gid++;
        if (gid < ids.size() && k < flags.size() && flags[k]) out.push_back(ids[gid]);
        k++;
        gid++;
    }
    return out;
}

HostColumn ParquetReader::sharded_scan(int c, const std::string& pattern, bool neg, const std::vector<Device*>& devices,
                                       bool want_col, std::vector<size_t>* page_ids, bool* walk_failed) {
    *walk_failed = false;
    const int nrg = static_cast<int>(num_row_groups());
    const int D = static_cast<int>(devices.size());
    std::vector<pq_chunk_desc> descs(static_cast<size_t>(nrg));
    std::vector<std::vector<pq_page_desc>> tables(static_cast<size_t>(nrg));
    std::vector<std::vector<int64_t>> plans(static_cast<size_t>(nrg), std::vector<int64_t>(2 * static_cast<size_t>(D)));
    for (int rg = 0; rg < nrg; rg++) {
        pq_chunk_desc& d = descs[static_cast<size_t>(rg)];
        int rc = pq_file_chunk(file_, rg, c, &d);
        if (rc) raise(rc, "ColumnChunk has no metadata");
        std::vector<pq_page_desc>& t = tables[static_cast<size_t>(rg)];
        int64_t n = 0;
        t.resize(1024);
        for (;;) {
            rc = pq_build_page_table(data_.data(), data_.size(), &d, t.data(), static_cast<int64_t>(t.size()), &n,
                                     nullptr, 0);
            if (n <= static_cast<int64_t>(t.size())) break;
            t.resize(static_cast<size_t>(n));
        }
        t.resize(static_cast<size_t>(n));
        if (rc) {  // a walk error: the caller takes the one-device path (the reference's error)
            *walk_failed = true;
            return HostColumn{};
        }
        pq_plan_page_ranges(t.data(), n, D, plans[static_cast<size_t>(rg)].data());
    }
    std::vector<std::vector<HostColumn>> parts(static_cast<size_t>(D), std::vector<HostColumn>(static_cast<size_t>(nrg)));
    std::vector<std::vector<std::vector<uint8_t>>> fl(static_cast<size_t>(D),
                                                      std::vector<std::vector<uint8_t>>(static_cast<size_t>(nrg)));
    std::vector<std::exception_ptr> errs(static_cast<size_t>(D) * static_cast<size_t>(nrg));
    std::vector<std::thread> th;
    for (int k = 0; k < D; k++) {
        th.emplace_back([&, k]() {
            for (int rg = 0; rg < nrg; rg++) {
                const auto& pl = plans[static_cast<size_t>(rg)];
                try {
                    scan_range(*devices[static_cast<size_t>(k)], data_.data(), data_.size(), descs[static_cast<size_t>(rg)],
                               tables[static_cast<size_t>(rg)], pl[2 * static_cast<size_t>(k)],
                               pl[2 * static_cast<size_t>(k) + 1], &pattern, neg,
                               want_col ? &parts[static_cast<size_t>(k)][static_cast<size_t>(rg)] : nullptr,
                               &fl[static_cast<size_t>(k)][static_cast<size_t>(rg)]);
                } catch (...) {
                    errs[static_cast<size_t>(rg) * D + k] = std::current_exception();
                    return;  // (later row groups of this device are never reached by the reference)
                }
            }
        });
    }
    for (auto& x : th) x.join();
    for (auto& e : errs)  // the first error in page order (row group, then shard)
        if (e) std::rethrow_exception(e);
    std::vector<uint8_t> flags;
    for (int rg = 0; rg < nrg; rg++)
        for (int k = 0; k < D; k++) {
            const auto& f = fl[static_cast<size_t>(k)][static_cast<size_t>(rg)];
            flags.insert(flags.end(), f.begin(), f.end());
        }
    std::vector<int64_t> offs;
    for (const auto& t : tables)
        for (const auto& p : t)
            if (p.page_type == PQ_DATA_PAGE) offs.push_back(p.payload_offset);
    *page_ids = flagged_page_ids(c, offs, flags);
    HostColumn out;
    out.type = columns_[static_cast<size_t>(c)].type;
    if (!want_col) return out;
    for (int rg = 0; rg < nrg; rg++)
        for (int k = 0; k < D; k++) append_column(out, parts[static_cast<size_t>(k)][static_cast<size_t>(rg)]);
    if (out.type == ParquetType::BYTE_ARRAY && out.offsets.empty()) out.offsets.push_back(0);
    out.validity.resize(static_cast<size_t>((out.num_rows + 31) / 32) + 1, 0);
    return out;
}

}  // namespace pqgpu
