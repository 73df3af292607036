// api_check — drives the C++ reader API (include/pqgpu/reader.hpp) exactly
// as a user of the reference would, and writes canonical dumps (SURVEY §8:
// u8 is_null + value bytes, strings as u32 length + bytes) for the tests.
//
//   api_check <file> read_column <name>            ParquetReader::read_column
//   api_check <file> column_reader <rg> <col>      ColumnReader(read_range,...).read_all
//   api_check <file> read_pages <rg> <col>         ColumnReader::read_pages (page records on stderr)
//   api_check <file> iterator <name>               StringColumnIterator (pos, len, bytes)
//   api_check <file> sharded <name> <k>            read_column over k Devices (device i % count),
//                                                  one host thread each
//   api_check <file> regex_sharded <name> <k> <pattern> <neg>
//                                                  regex_pages over k Devices: page ids, one per line
//   api_check <file> decode_regex_sharded <name> <k> <pattern> <neg>
//                                                  read_column_regex over k Devices: the column's
//                                                  dump on stdout, the page ids on stderr
//   api_check <file> time_read_all <rg> <col> <reps> <dump path>
//                                                  times ColumnReader::read_all (host bytes ->
//                                                  std::vector<Value>), read_columnar and the
//                                                  Value build alone (median ms, JSON on stdout);
//                                                  the last read_all's dump goes to the path
#include <execinfo.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <csignal>
#include <cstdio>
#include <cstring>
#include <iostream>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "pq_gpu.h"
#include "pqgpu/reader.hpp"

static void dump(const pqgpu::Value& v, std::vector<uint8_t>& out) {
    out.push_back(v.is_null ? 1 : 0);
    if (v.is_null) return;
    std::visit([&](auto&& a) {
        using T = std::decay_t<decltype(a)>;
        if constexpr (std::is_same_v<T, std::string>) {
            uint32_t n = static_cast<uint32_t>(a.size());
            out.insert(out.end(), reinterpret_cast<uint8_t*>(&n), reinterpret_cast<uint8_t*>(&n) + 4);
            out.insert(out.end(), a.begin(), a.end());
        } else if constexpr (std::is_same_v<T, bool>) {
            out.push_back(a ? 1 : 0);
        } else {
            const uint8_t* p = reinterpret_cast<const uint8_t*>(&a);
            out.insert(out.end(), p, p + sizeof(T));
        }
    }, v.data);
}

// a crash prints its native stack to stderr (test diagnostics)
static void on_crash(int sig) {
    void* fr[64];
    const int n = backtrace(fr, 64);
    const char msg[] = "api_check: fatal signal; stack:\n";
    (void)!write(2, msg, sizeof msg - 1);
    backtrace_symbols_fd(fr, n, 2);
    std::signal(sig, SIG_DFL);
    std::raise(sig);
}

int main(int argc, char** argv) {
    if (argc < 4) return 2;
    std::signal(SIGSEGV, on_crash);
    std::signal(SIGABRT, on_crash);
    try {
        pqgpu::ParquetReader r;
        if (!r.open(argv[1])) return 1;
        std::string mode = argv[2];
        std::vector<uint8_t> out;
        if (mode == "read_column") {
            for (const auto& v : r.read_column(argv[3])) dump(v, out);
        } else if (mode == "sharded" || mode == "regex_sharded" || mode == "decode_regex_sharded") {
            int k = argc > 4 ? std::atoi(argv[4]) : 2;
            int nd = pqgpu::Device::count();
            if (nd < 1) throw std::runtime_error("no HIP device");
            std::vector<std::unique_ptr<pqgpu::Device>> own;
            std::vector<pqgpu::Device*> devs;
            for (int i = 0; i < k; i++) {
                own.emplace_back(new pqgpu::Device(i % nd));
                devs.push_back(own.back().get());
            }
            if (mode == "sharded") {
                for (const auto& v : r.read_column(argv[3], devs)) dump(v, out);
            } else {
                if (argc < 7) return 2;
                const std::string pat = argv[5];
                const bool neg = std::atoi(argv[6]) != 0;
                std::vector<size_t> ids;
                if (mode == "regex_sharded") {
                    ids = r.regex_pages(argv[3], pat, neg, devs);
                    for (size_t id : ids) {
                        const std::string ln = std::to_string(id) + "\n";
                        out.insert(out.end(), ln.begin(), ln.end());
                    }
                } else {
                    pqgpu::HostColumn h = r.read_column_regex(argv[3], pat, neg, devs, &ids);
                    for (int64_t i = 0; i < h.num_rows; i++) dump(h.value(i), out);
                    for (size_t id : ids) std::fprintf(stderr, "%zu\n", id);
                }
            }
        } else if (mode == "iterator") {
            auto it = r.column_iterator(argv[3]);
            while (it.has_next()) {
                auto [pos, len, ptr] = it.next();
                uint64_t p = pos;
                uint32_t l = static_cast<uint32_t>(len);
                out.insert(out.end(), reinterpret_cast<uint8_t*>(&p), reinterpret_cast<uint8_t*>(&p) + 8);
                out.insert(out.end(), reinterpret_cast<uint8_t*>(&l), reinterpret_cast<uint8_t*>(&l) + 4);
                out.insert(out.end(), ptr, ptr + len);
            }
        } else {
            int rg = std::atoi(argv[3]), col = std::atoi(argv[4]);
            const auto& ci = r.column(static_cast<size_t>(col));
            pqgpu::ColumnChunk cc;
            // metadata through the public file helpers of the C ABI is what
            // ParquetReader uses; rebuild a ColumnChunk the way a caller would
            pqgpu::ColumnMetaData md;
            std::vector<uint8_t> all = r.read_range(0, r.file_size());
            pq_file* f = nullptr;
            pq_file_open(all.data(), all.size(), &f, nullptr, 0);
            pq_chunk_desc d{};
            pq_file_chunk(f, rg, col, &d);
            pq_file_close(f);
            md.type = static_cast<pqgpu::ParquetType>(d.type);
            md.num_values = d.num_values;
            md.data_page_offset = d.data_page_offset;
            md.total_compressed_size = d.total_compressed_size;
            if (d.has_dictionary_page_offset) md.dictionary_page_offset = d.dictionary_page_offset;
            cc.meta_data = md;
            pqgpu::ColumnReader cr([&](size_t off, size_t len) { return r.read_range(off, len); }, cc,
                                   ci.type, ci.max_def_level, ci.max_rep_level);
            if (mode == "column_reader") {
                for (const auto& v : cr.read_all()) dump(v, out);
            } else if (mode == "time_read_all") {
                if (argc < 7) return 2;
                const int reps = std::max(1, std::atoi(argv[5]));
                auto now = [] { return std::chrono::steady_clock::now(); };
                auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
                auto med = [](std::vector<double> v) {
                    std::sort(v.begin(), v.end());
                    return v[v.size() / 2];
                };
                std::vector<double> ta, tc, tv, td, tr, tf, tz, tl, tdh;
                std::vector<pqgpu::Value> vals = cr.read_all();  // warm-up (device buffers, first-touch pages)
                for (int i = 0; i < reps; i++) {
                    const auto tq = now();
                    vals.clear();  // the previous result's destruction (10M strings freed)
                    vals.shrink_to_fit();
                    const auto t0 = now();
                    vals = cr.read_all();
                    const auto t1 = now();
                    const pqgpu::ToValuesPhases P = pqgpu::last_to_values_phases();
                    pqgpu::HostColumn h = cr.read_columnar();
                    const auto t2 = now();
                    std::vector<pqgpu::Value> v2 = pqgpu::to_values(h);
                    const auto t3 = now();
                    { std::vector<pqgpu::Value> drop(std::move(v2)); }
                    const auto t4 = now();
                    td.push_back(ms(tq, t0));
                    ta.push_back(ms(t0, t1));
                    tc.push_back(ms(t1, t2));
                    tv.push_back(ms(t2, t3));
                    tdh.push_back(ms(t3, t4));
                    tr.push_back(P.reserve_ms);
                    tf.push_back(P.fault_ms);
                    tz.push_back(P.resize_ms);
                    tl.push_back(P.fill_ms);
                }
                for (const auto& v : vals) dump(v, out);
                FILE* fh = std::fopen(argv[6], "wb");
                if (!fh) throw std::runtime_error("cannot write the dump");
                std::fwrite(out.data(), 1, out.size(), fh);
                std::fclose(fh);
                auto list = [](const std::vector<double>& v) {
                    std::string r = "[";
                    for (size_t i = 0; i < v.size(); i++) r += (i ? ", " : "") + std::to_string(v[i]);
                    return r + "]";
                };
                // read_all's phases: columnar read (read_all_ms - the to_values
                // phases), then to_values' reserve / fault / resize / fill; the
                // destruction of a result before the next read is timed apart
                std::printf("{\"values\": %zu, \"read_all_ms\": %.4f, \"read_columnar_ms\": %.4f, "
                            "\"to_values_ms\": %.4f, \"threads\": %u, \"read_all_samples\": %s, "
                            "\"to_values_samples\": %s, \"phases_ms\": {\"reserve\": %.4f, \"fault\": %.4f, "
                            "\"resize\": %.4f, \"fill\": %.4f, \"destroy_before\": %.4f, \"destroy_v2\": %.4f}}\n",
                            vals.size(), med(ta), med(tc), med(tv),
                            std::max(1u, std::min(16u, std::thread::hardware_concurrency())), list(ta).c_str(),
                            list(tv).c_str(), med(tr), med(tf), med(tz), med(tl), med(td), med(tdh));
                return 0;
            } else {
                for (const auto& pr : cr.read_pages()) {
                    std::fprintf(stderr, "%d %d %d %zu\n", pr.page_num, static_cast<int>(pr.type),
                                 pr.num_values, pr.values.size());
                    for (const auto& v : pr.values) dump(v, out);
                }
            }
        }
        std::fwrite(out.data(), 1, out.size(), stdout);
        return 0;
    } catch (const std::bad_optional_access& e) {
        std::cerr << "bad optional access\n";
        return 3;
    } catch (const std::exception& e) {
        std::cerr << e.what() << "\n";
        return 1;
    }
}
