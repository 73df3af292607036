// src/reader/column_reader.cpp (reference side) — GPU-backed read_all.
// The reference's ColumnReader keeps its constructor, members and read_pages;
// read_all's body becomes the MI355X path through the C ABI (pq_gpu.h).
#include "reader/column_reader.hpp"

#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "pq_gpu.h"

static pq_ctx* gpu() {
    static pq_ctx* c = pq_ctx_create(0);
    if (!c) throw std::runtime_error("no HIP device");  // no CPU fallback
    return c;
}

std::vector<Value> ColumnReader::read_all() {
    // 1. the bytes the reference pulls through read_range_: one range over the
    //    chunk (start = min(dict_off, data_off), column_reader.cpp:22-25) plus a
    //    header window; pq_chunk_upload walks the page headers exactly like the
    //    reference (256-byte window, zero padding past the range).
    const int64_t start = meta_->dictionary_page_offset
                              ? std::min(*meta_->dictionary_page_offset, meta_->data_page_offset)
                              : meta_->data_page_offset;
    const size_t len = static_cast<size_t>(meta_->total_compressed_size) + 256;
    std::vector<uint8_t> bytes = read_range_(static_cast<size_t>(start), len);

    pq_chunk_desc d{};
    d.num_values = meta_->num_values;
    d.data_page_offset = meta_->data_page_offset - start;  // offsets into `bytes`
    d.has_dictionary_page_offset = meta_->dictionary_page_offset.has_value() ? 1 : 0;
    d.dictionary_page_offset = d.has_dictionary_page_offset ? *meta_->dictionary_page_offset - start : 0;
    d.codec = static_cast<int32_t>(meta_->codec);
    d.type = static_cast<int32_t>(type_);
    d.max_def_level = max_def_level_;
    d.max_rep_level = max_rep_level_;
    d.total_compressed_size = meta_->total_compressed_size;

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

    // 2. device -> host arrays, then the reference's Value objects (columnar
    //    consumers keep col.d_validity / d_offsets / d_values in HBM instead)
    const int64_t n = col.num_rows;
    std::vector<uint32_t> valid(static_cast<size_t>((n + 31) / 32 + 1));
    std::vector<int64_t> offs(type_ == ParquetType::BYTE_ARRAY ? static_cast<size_t>(n + 1) : 0);
    std::vector<uint8_t> data(static_cast<size_t>(col.num_bytes) + 16);
    const int rc = pq_column_copy_out(gpu(), &col, valid.data(), data.data(), offs.empty() ? nullptr : offs.data());
    pq_column_free(gpu(), &col);
    pq_chunk_free(gpu(), ch);
    if (rc != 0) throw std::runtime_error(pq_last_error(gpu()));

    std::vector<Value> out(static_cast<size_t>(n));
    const uint8_t* p = data.data();
    for (int64_t i = 0; i < n; i++) {
        if (!((valid[static_cast<size_t>(i >> 5)] >> (i & 31)) & 1u)) {
            out[static_cast<size_t>(i)] = Value::null();
            continue;
        }
        Value& v = out[static_cast<size_t>(i)];
        switch (type_) {  // read_plain_value's conversions (column_reader.cpp:227-268)
            case ParquetType::BYTE_ARRAY:
                v = Value::from_string(std::string(reinterpret_cast<const char*>(p) + offs[i],
                                                   static_cast<size_t>(offs[i + 1] - offs[i])));
                break;
            case ParquetType::BOOLEAN: v = Value::from_bool(p[i] != 0); break;
            case ParquetType::INT32: { int32_t x; std::memcpy(&x, p + 4 * i, 4); v = Value::from_i32(x); break; }
            case ParquetType::INT64: { int64_t x; std::memcpy(&x, p + 8 * i, 8); v = Value::from_i64(x); break; }
            case ParquetType::FLOAT: { float x; std::memcpy(&x, p + 4 * i, 4); v = Value::from_float(x); break; }
            case ParquetType::DOUBLE: { double x; std::memcpy(&x, p + 8 * i, 8); v = Value::from_double(x); break; }
            case ParquetType::INT96: {  // raw 12 bytes -> the reference's "INT96(hi:lo)" string
                int64_t lo;
                int32_t hi;
                std::memcpy(&lo, p + 12 * i, 8);
                std::memcpy(&hi, p + 12 * i + 8, 4);
                v = Value::from_string("INT96(" + std::to_string(hi) + ":" + std::to_string(lo) + ")");
                break;
            }
            default: throw std::runtime_error("Unsupported type: " + std::to_string(static_cast<int>(type_)));
        }
    }
    return out;
}
