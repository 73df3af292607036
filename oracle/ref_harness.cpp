// ref_harness.cpp — TEST INFRASTRUCTURE ONLY.
//
// A thin extern "C" harness over the *unmodified* reference sources
// (compiled where they lie under $(REF), see oracle/Makefile; nothing from the
// reference is copied into this repository).  It exposes:
//   * ColumnReader::read_all / read_pages driven by an in-memory ReadRangeFunc
//     that zero-pads past EOF -> canonical dump;
//   * ParquetReader::open metadata + build_page_index ids (R-PAGEIDX);
//   * ParquetReader::read_column (R-CALLER, ifstream-backed);
//   * ParquetWriter (used to prove the generator's "ref-layout" matches the
//     reference writer byte for byte).
// Output goes only to oracle/_ref/.  Used by tests/ and bench.py's
// cpu_baseline leg; never by the product library.
#include "reader/column_reader.hpp"
#include "reader/parquet_reader.hpp"
#include "writer/parquet_writer.hpp"

#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <thread>
#include <vector>

namespace {

void put_err(char* err, size_t errlen, const std::string& s) {
    if (err && errlen) {
        std::strncpy(err, s.c_str(), errlen - 1);
        err[errlen - 1] = 0;
    }
}

void dump_value(const Value& v, std::vector<uint8_t>& out) {
    out.push_back(v.is_null ? 1 : 0);
    if (v.is_null) return;
    std::visit(
        [&](auto&& a) {
            using T = std::decay_t<decltype(a)>;
            if constexpr (std::is_same_v<T, std::string>) {
                uint32_t n = static_cast<uint32_t>(a.size());
                const uint8_t* p = reinterpret_cast<const uint8_t*>(&n);
                out.insert(out.end(), p, p + 4);
                out.insert(out.end(), a.begin(), a.end());
            } else if constexpr (std::is_same_v<T, bool>) {
                out.push_back(a ? 1 : 0);
            } else {
                const uint8_t* p = reinterpret_cast<const uint8_t*>(&a);
                out.insert(out.end(), p, p + sizeof(T));
            }
        },
        v.data);
}

uint8_t* to_malloc(const std::vector<uint8_t>& v, size_t* len) {
    uint8_t* p = static_cast<uint8_t*>(std::malloc(v.empty() ? 1 : v.size()));
    if (!v.empty()) std::memcpy(p, v.data(), v.size());
    *len = v.size();
    return p;
}

ColumnChunk make_chunk(int64_t num_values, int64_t data_off, int64_t dict_off, int has_dict,
                       int32_t codec, int32_t type, size_t flen) {
    ColumnChunk cc;
    ColumnMetaData md;
    md.type = static_cast<ParquetType>(type);
    md.codec = static_cast<CompressionCodec>(codec);
    md.num_values = num_values;
    md.data_page_offset = data_off;
    if (has_dict) md.dictionary_page_offset = dict_off;
    // (the CPU reader never reads it; a reader that fetches the chunk as one
    // range, INTEGRATION.md path B, gets the bytes up to EOF)
    const int64_t start = has_dict ? std::min(dict_off, data_off) : data_off;
    md.total_compressed_size = std::max<int64_t>(static_cast<int64_t>(flen) - start, 0);
    cc.meta_data = md;
    return cc;
}

ReadRangeFunc memory_range(const uint8_t* file, size_t flen) {
    return [file, flen](size_t off, size_t len) {
        std::vector<uint8_t> b(len, 0);
        if (off < flen) std::memcpy(b.data(), file + off, std::min(len, flen - off));
        return b;
    };
}

}  // namespace

extern "C" {

// ColumnReader::read_all over an in-memory file.  Returns 0, or -1 with the
// exception text in err.  *dump is malloc'd canonical dump.
int pqref_read_all(const uint8_t* file, size_t flen, int64_t num_values, int64_t data_off,
                   int64_t dict_off, int has_dict, int32_t codec, int32_t type, int16_t max_def,
                   int16_t max_rep, uint8_t** dump, size_t* dump_len, char* err, size_t errlen) {
    try {
        ColumnChunk cc = make_chunk(num_values, data_off, dict_off, has_dict, codec, type, flen);
        ColumnReader r(memory_range(file, flen), cc, static_cast<ParquetType>(type), max_def,
                       max_rep);
        std::vector<Value> vals = r.read_all();
        std::vector<uint8_t> out;
        for (const auto& v : vals) dump_value(v, out);
        *dump = to_malloc(out, dump_len);
        return 0;
    } catch (const std::bad_optional_access& e) {
        put_err(err, errlen, std::string("bad optional access: ") + e.what());
        return -3;
    } catch (const std::exception& e) {
        put_err(err, errlen, e.what());
        return -1;
    }
}

// ColumnReader::read_pages: dump of all values, plus per PageResult
// (page_num, type, num_values, nvalues) quadruples in `pages` (cap entries).
int pqref_read_pages(const uint8_t* file, size_t flen, int64_t num_values, int64_t data_off,
                     int64_t dict_off, int has_dict, int32_t codec, int32_t type, int16_t max_def,
                     int16_t max_rep, uint8_t** dump, size_t* dump_len, int64_t* pages, int cap,
                     int* npages, char* err, size_t errlen) {
    try {
        ColumnChunk cc = make_chunk(num_values, data_off, dict_off, has_dict, codec, type, flen);
        ColumnReader r(memory_range(file, flen), cc, static_cast<ParquetType>(type), max_def,
                       max_rep);
        std::vector<PageResult> prs = r.read_pages();
        std::vector<uint8_t> out;
        int n = 0;
        for (const auto& pr : prs) {
            if (n < cap) {
                pages[4 * n + 0] = pr.page_num;
                pages[4 * n + 1] = static_cast<int64_t>(pr.type);
                pages[4 * n + 2] = pr.num_values;
                pages[4 * n + 3] = static_cast<int64_t>(pr.values.size());
            }
            n++;
            for (const auto& v : pr.values) dump_value(v, out);
        }
        *npages = n;
        *dump = to_malloc(out, dump_len);
        return 0;
    } catch (const std::bad_optional_access& e) {
        put_err(err, errlen, std::string("bad optional access: ") + e.what());
        return -3;
    } catch (const std::exception& e) {
        put_err(err, errlen, e.what());
        return -1;
    }
}

// Footer + schema + page index of a file, via ParquetReader::open.
// meta[] receives, per (row group, leaf column) in rg-major order:
//   num_values, data_page_offset, dictionary_page_offset (or -1), codec, type,
//   max_def, max_rep, num_rows_of_rg   (8 int64 each).
// pidx[] receives, per global data page id: data_offset, data_size, rg, col.
int pqref_open(const char* path, int64_t* nrg, int64_t* ncol, int64_t* meta, int meta_cap,
               int64_t* pidx, int64_t pidx_cap, int64_t* npages, char* err, size_t errlen) {
    try {
        ParquetReader pr;
        if (!pr.open(path)) {
            put_err(err, errlen, "open failed");
            return -1;
        }
        *nrg = static_cast<int64_t>(pr.num_row_groups());
        *ncol = static_cast<int64_t>(pr.num_columns());
        int k = 0;
        for (size_t rg = 0; rg < pr.num_row_groups(); rg++) {
            for (size_t c = 0; c < pr.num_columns(); c++) {
                if (k >= meta_cap) break;
                const auto& ci = pr.column(c);
                const auto& md = pr.metadata().row_groups[rg].columns[ci.column_index].meta_data.value();
                int64_t* m = meta + 8 * k++;
                m[0] = md.num_values;
                m[1] = md.data_page_offset;
                m[2] = md.dictionary_page_offset.has_value() ? *md.dictionary_page_offset : -1;
                m[3] = static_cast<int64_t>(md.codec);
                m[4] = static_cast<int64_t>(ci.type);
                m[5] = ci.max_def_level;
                m[6] = ci.max_rep_level;
                m[7] = pr.metadata().row_groups[rg].num_rows;
            }
        }
        *npages = static_cast<int64_t>(pr.num_pages());
        for (size_t i = 0; i < pr.num_pages() && static_cast<int64_t>(i) < pidx_cap; i++) {
            const auto& e = pr.page_index_entry(i);
            pidx[4 * i + 0] = static_cast<int64_t>(e.data_offset);
            pidx[4 * i + 1] = static_cast<int64_t>(e.data_size);
            pidx[4 * i + 2] = static_cast<int64_t>(e.row_group_idx);
            pidx[4 * i + 3] = static_cast<int64_t>(e.column_idx);
        }
        return 0;
    } catch (const std::exception& e) {
        put_err(err, errlen, e.what());
        return -1;
    }
}

// ParquetReader::read_column(name) — the R-CALLER path, ifstream-backed.
int pqref_read_column(const char* path, const char* name, uint8_t** dump, size_t* dump_len,
                      char* err, size_t errlen) {
    try {
        ParquetReader pr;
        if (!pr.open(path)) {
            put_err(err, errlen, "open failed");
            return -1;
        }
        std::vector<Value> vals = pr.read_column(name);
        std::vector<uint8_t> out;
        for (const auto& v : vals) dump_value(v, out);
        *dump = to_malloc(out, dump_len);
        return 0;
    } catch (const std::bad_optional_access& e) {
        put_err(err, errlen, std::string("bad optional access: ") + e.what());
        return -3;
    } catch (const std::exception& e) {
        put_err(err, errlen, e.what());
        return -1;
    }
}

// Write one row group with the reference ParquetWriter.  Columns are given
// in the canonical dump format (one dump per column, nrows rows each).
int pqref_write(const char* path, int ncols, const char** names, const int32_t* types,
                const int32_t* repetition, const int32_t* converted, const uint8_t** dumps,
                int64_t nrows, char* err, size_t errlen) {
    try {
        std::vector<ColumnSpec> specs;
        std::vector<std::vector<Value>> cols(ncols);
        for (int c = 0; c < ncols; c++) {
            ColumnSpec s;
            s.name = names[c];
            s.type = static_cast<ParquetType>(types[c]);
            s.repetition = static_cast<FieldRepetitionType>(repetition[c]);
            if (converted[c] >= 0) s.converted_type = static_cast<ConvertedType>(converted[c]);
            specs.push_back(s);
            const uint8_t* p = dumps[c];
            cols[c].reserve(nrows);
            for (int64_t i = 0; i < nrows; i++) {
                uint8_t is_null = *p++;
                if (is_null) { cols[c].push_back(Value::null()); continue; }
                switch (s.type) {
                    case ParquetType::BOOLEAN: cols[c].push_back(Value::from_bool(*p++ != 0)); break;
                    case ParquetType::INT32: { int32_t v; std::memcpy(&v, p, 4); p += 4; cols[c].push_back(Value::from_i32(v)); break; }
                    case ParquetType::INT64: { int64_t v; std::memcpy(&v, p, 8); p += 8; cols[c].push_back(Value::from_i64(v)); break; }
                    case ParquetType::FLOAT: { float v; std::memcpy(&v, p, 4); p += 4; cols[c].push_back(Value::from_float(v)); break; }
                    case ParquetType::DOUBLE: { double v; std::memcpy(&v, p, 8); p += 8; cols[c].push_back(Value::from_double(v)); break; }
                    default: {
                        uint32_t n; std::memcpy(&n, p, 4); p += 4;
                        cols[c].push_back(Value::from_string(std::string(reinterpret_cast<const char*>(p), n)));
                        p += n;
                    }
                }
            }
        }
        ParquetWriter w(path, specs);
        w.write_row_group(cols);
        w.close();
        return 0;
    } catch (const std::exception& e) {
        put_err(err, errlen, e.what());
        return -1;
    }
}

// CPU baseline: ColumnReader::read_all over an in-memory file, repeated
// `reps` times on `threads` concurrent readers (one private ReadRangeFunc
// each, the reference API's natural parallelism).  Returns wall seconds.
double pqref_time_read_all(const uint8_t* file, size_t flen, int64_t num_values, int64_t data_off,
                           int64_t dict_off, int has_dict, int32_t type, int16_t max_def,
                           int16_t max_rep, int reps, int threads, int64_t* values_out) {
    ColumnChunk cc = make_chunk(num_values, data_off, dict_off, has_dict, 0, type, flen);
    std::vector<int64_t> counts(threads, 0);
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> ts;
    for (int t = 0; t < threads; t++) {
        ts.emplace_back([&, t] {
            for (int r = 0; r < reps; r++) {
                ColumnReader rd(memory_range(file, flen), cc, static_cast<ParquetType>(type),
                                max_def, max_rep);
                counts[t] += static_cast<int64_t>(rd.read_all().size());
            }
        });
    }
    for (auto& th : ts) th.join();
    double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    int64_t tot = 0;
    for (auto c : counts) tot += c;
    if (values_out) *values_out = tot;
    return s;
}

// Page-parallel baseline: `n` independent sub-chunks (each a shard's pages
// extracted as a standalone chunk, pqgpu/shard.py extract_range), read by
// `threads` ColumnReaders that take shards from a shared counter, `reps`
// rounds.  Same reference ColumnReader::read_all per shard.
double pqref_time_read_all_multi(int n, const uint8_t* const* files, const size_t* flens,
                                 const int64_t* num_values, const int64_t* data_off,
                                 const int64_t* dict_off, const int32_t* has_dict, int32_t type,
                                 int16_t max_def, int16_t max_rep, int reps, int threads,
                                 int64_t* values_out) {
    std::vector<ColumnChunk> ccs;
    for (int i = 0; i < n; i++)
        ccs.push_back(make_chunk(num_values[i], data_off[i], dict_off[i], has_dict[i], 0, type, flens[i]));
    std::vector<int64_t> counts(threads, 0);
    std::atomic<int64_t> next{0};
    const int64_t total = static_cast<int64_t>(n) * reps;
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> ts;
    for (int t = 0; t < threads; t++) {
        ts.emplace_back([&, t] {
            for (int64_t k = next.fetch_add(1); k < total; k = next.fetch_add(1)) {
                const int i = static_cast<int>(k % n);
                ColumnReader rd(memory_range(files[i], flens[i]), ccs[i], static_cast<ParquetType>(type),
                                max_def, max_rep);
                counts[t] += static_cast<int64_t>(rd.read_all().size());
            }
        });
    }
    for (auto& th : ts) th.join();
    double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    int64_t tot = 0;
    for (auto c : counts) tot += c;
    if (values_out) *values_out = tot;
    return s;
}

// Regex CPU baseline: the page-parallel read above, then
// every page's non-null values tested with `match` (the build's host DFA,
// pq_regex_host_match, passed in as a function pointer) until one satisfies
// the predicate (match != neg); flags[page] = 1 if none does (the page is
// REPORTED, README.md:54-64).  page_first[i] .. page_first[i + 1] index
// shard i's data-page row counts in `counts`.  `reps` rounds; wall seconds.
double pqref_time_regex_pages_multi(int n, const uint8_t* const* files, const size_t* flens,
                                    const int64_t* num_values, const int64_t* data_off,
                                    const int64_t* dict_off, const int32_t* has_dict, int32_t type,
                                    int16_t max_def, int16_t max_rep, const int64_t* page_first,
                                    const int32_t* counts, int (*match)(const void*, const uint8_t*, size_t),
                                    const void* mstate, int neg, int reps, int threads, uint8_t* flags) {
    std::vector<ColumnChunk> ccs;
    for (int i = 0; i < n; i++)
        ccs.push_back(make_chunk(num_values[i], data_off[i], dict_off[i], has_dict[i], 0, type, flens[i]));
    std::atomic<int64_t> next{0};
    const int64_t total = static_cast<int64_t>(n) * reps;
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> ts;
    for (int t = 0; t < threads; t++) {
        ts.emplace_back([&] {
            for (int64_t k = next.fetch_add(1); k < total; k = next.fetch_add(1)) {
                const int i = static_cast<int>(k % n);
                ColumnReader rd(memory_range(files[i], flens[i]), ccs[i], static_cast<ParquetType>(type),
                                max_def, max_rep);
                std::vector<Value> vals = rd.read_all();
                size_t row = 0;
                for (int64_t pg = page_first[i]; pg < page_first[i + 1]; pg++) {
                    uint8_t rep = 1;
                    const size_t end = row + static_cast<size_t>(counts[pg]);
                    for (size_t r = row; r < end && r < vals.size(); r++) {
                        if (vals[r].is_null) continue;
                        const std::string& s = std::get<std::string>(vals[r].data);
                        if ((match(mstate, reinterpret_cast<const uint8_t*>(s.data()), s.size()) != 0) != (neg != 0)) {
                            rep = 0;
                            break;
                        }
                    }
                    flags[pg] = rep;
                    row = end;
                }
            }
        });
    }
    for (auto& th : ts) th.join();
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

void pqref_free(void* p) { std::free(p); }

}  // extern "C"
