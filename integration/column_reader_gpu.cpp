// src/reader/column_reader.cpp (reference side) — GPU-backed read_all / read_pages.
// The reference's ColumnReader keeps its constructor and members; the bodies
// of read_all and read_pages become the MI355X path through the C ABI
// (pq_gpu.h), and the std::vector<Value> results are built on host threads.
#include "reader/column_reader.hpp"

#include <algorithm>
#include <cstring>
#include <iterator>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "pq_gpu.h"

static pq_ctx* gpu() {
    static pq_ctx* c = pq_ctx_create(0);
    if (!c) throw std::runtime_error("no HIP device");  // no CPU fallback
    return c;
}

namespace {

// One chunk decoded on the GPU, copied out as host arrays.
struct GpuColumn {
    ParquetType type;
    int64_t n = 0;
    std::vector<uint32_t> valid;
    std::vector<int64_t> offs;
    std::vector<uint8_t> data;

    Value at(int64_t i) const {  // read_plain_value's conversions (column_reader.cpp:227-268)
        if (!((valid[static_cast<size_t>(i >> 5)] >> (i & 31)) & 1u)) return Value::null();
        const uint8_t* p = data.data();
        switch (type) {
            case ParquetType::BYTE_ARRAY:
                return Value::from_string(std::string(reinterpret_cast<const char*>(p) + offs[i],
                                                      static_cast<size_t>(offs[i + 1] - offs[i])));
            case ParquetType::BOOLEAN: return Value::from_bool(p[i] != 0);
            case ParquetType::INT32: { int32_t x; std::memcpy(&x, p + 4 * i, 4); return Value::from_i32(x); }
            case ParquetType::INT64: { int64_t x; std::memcpy(&x, p + 8 * i, 8); return Value::from_i64(x); }
            case ParquetType::FLOAT: { float x; std::memcpy(&x, p + 4 * i, 4); return Value::from_float(x); }
            case ParquetType::DOUBLE: { double x; std::memcpy(&x, p + 8 * i, 8); return Value::from_double(x); }
            case ParquetType::INT96: {  // raw 12 bytes -> the reference's "INT96(hi:lo)" string
                int64_t lo;
                int32_t hi;
                std::memcpy(&lo, p + 12 * i, 8);
                std::memcpy(&hi, p + 12 * i + 8, 4);
                return Value::from_string("INT96(" + std::to_string(hi) + ":" + std::to_string(lo) + ")");
            }
            default: throw std::runtime_error("Unsupported type: " + std::to_string(static_cast<int>(type)));
        }
    }

    // Rows [a, b) as Values: contiguous row ranges on up to 16 host threads
    // (the std::string of a BYTE_ARRAY value is a heap allocation per row).
    std::vector<Value> values(int64_t a, int64_t b) const {
        const int64_t m = std::max<int64_t>(std::min(b, n) - a, 0);
        std::vector<Value> out(static_cast<size_t>(m));
        const int64_t t = std::min<int64_t>(std::max(1u, std::min(16u, std::thread::hardware_concurrency())),
                                            std::max<int64_t>(1, m / 65536));
        auto part = [&](int64_t k) {
            for (int64_t r = m * k / t; r < m * (k + 1) / t; r++) out[static_cast<size_t>(r)] = at(a + r);
        };
        std::vector<std::thread> th;
        for (int64_t k = 1; k < t; k++) th.emplace_back(part, k);
        part(0);
        for (auto& x : th) x.join();
        return out;
    }
};

// The chunk's bytes as one range (start = min(dict_off, data_off),
// column_reader.cpp:22-25, plus a header window) and its descriptor.
void chunk_range(const ColumnMetaData* meta, ParquetType type, int16_t max_def, int16_t max_rep, int64_t* start,
                 size_t* len, pq_chunk_desc* d) {
    *start = meta->dictionary_page_offset ? std::min(*meta->dictionary_page_offset, meta->data_page_offset)
                                          : meta->data_page_offset;
    *len = static_cast<size_t>(meta->total_compressed_size) + 256;
    *d = pq_chunk_desc{};
    d->num_values = meta->num_values;
    d->data_page_offset = meta->data_page_offset - *start;  // offsets into the range
    d->has_dictionary_page_offset = meta->dictionary_page_offset.has_value() ? 1 : 0;
    d->dictionary_page_offset = d->has_dictionary_page_offset ? *meta->dictionary_page_offset - *start : 0;
    d->codec = static_cast<int32_t>(meta->codec);
    d->type = static_cast<int32_t>(type);
    d->max_def_level = max_def;
    d->max_rep_level = max_rep;
    d->total_compressed_size = meta->total_compressed_size;
}

// pq_chunk_upload walks the page headers exactly like the reference
// (256-byte window, zero padding past the range); errors carry its text.
GpuColumn decode(const std::vector<uint8_t>& bytes, const pq_chunk_desc& d, ParquetType type) {
    pq_chunk* ch = nullptr;
    if (pq_chunk_upload(gpu(), bytes.data(), bytes.size(), &d, 1, &ch) != 0)
        throw std::runtime_error(pq_last_error(gpu()));  // same text as the CPU path
    pq_column col{};
    if (pq_decode(gpu(), ch, &col) != 0) {
        std::string msg = pq_last_error(gpu());
        pq_column_free(gpu(), &col);
        pq_chunk_free(gpu(), ch);
        throw std::runtime_error(msg);
    }
    // device -> host arrays (columnar consumers keep col.d_validity /
    // d_offsets / d_values in HBM instead)
    GpuColumn c;
    c.type = type;
    c.n = col.num_rows;
    c.valid.resize(static_cast<size_t>((c.n + 31) / 32 + 1));
    c.offs.resize(type == ParquetType::BYTE_ARRAY ? static_cast<size_t>(c.n + 1) : 0);
    c.data.resize(static_cast<size_t>(col.num_bytes) + 16);
    const int rc = pq_column_copy_out(gpu(), &col, c.valid.data(), c.data.data(), c.offs.empty() ? nullptr : c.offs.data());
    pq_column_free(gpu(), &col);
    pq_chunk_free(gpu(), ch);
    if (rc != 0) throw std::runtime_error(pq_last_error(gpu()));
    return c;
}

}  // namespace

std::vector<Value> ColumnReader::read_all() {
    int64_t start;
    size_t len;
    pq_chunk_desc d;
    chunk_range(meta_, type_, max_def_level_, max_rep_level_, &start, &len, &d);
    const GpuColumn c = decode(read_range_(static_cast<size_t>(start), len), d, type_);
    return c.values(0, c.n);
}

std::vector<PageResult> ColumnReader::read_pages() {
    int64_t start;
    size_t len;
    pq_chunk_desc d;
    chunk_range(meta_, type_, max_def_level_, max_rep_level_, &start, &len, &d);
    const std::vector<uint8_t> bytes = read_range_(static_cast<size_t>(start), len);
    const GpuColumn c = decode(bytes, d, type_);
    // the page records of the same walk: page_num, type and num_values as
    // read_pages reports them (column_reader.cpp:73-126); pages of other
    // types only advance page_num
    int64_t np = 0;
    char err[512] = {0};
    (void)pq_build_page_table(bytes.data(), bytes.size(), &d, nullptr, 0, &np, err, sizeof err);
    std::vector<pq_page_desc> pl(static_cast<size_t>(np));
    if (np && pq_build_page_table(bytes.data(), bytes.size(), &d, pl.data(), np, &np, err, sizeof err) != 0)
        throw std::runtime_error(err);
    std::vector<Value> all = c.values(0, c.n);  // every row at once, then moved out per page
    std::vector<PageResult> pages;
    for (const pq_page_desc& p : pl) {
        if (p.page_type == static_cast<int32_t>(PageType::DICTIONARY_PAGE)) {
            pages.push_back({p.page_num, PageType::DICTIONARY_PAGE, p.num_values, {}});
        } else if (p.page_type == static_cast<int32_t>(PageType::DATA_PAGE)) {
            const int64_t a = std::min(p.first_row, c.n), b = std::min(p.first_row + std::max(p.num_values, 0), c.n);
            pages.push_back({p.page_num, PageType::DATA_PAGE, p.num_values,
                             std::vector<Value>(std::make_move_iterator(all.begin() + a),
                                                std::make_move_iterator(all.begin() + b))});
        }
    }
    return pages;
}
