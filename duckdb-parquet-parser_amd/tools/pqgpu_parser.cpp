// pqgpu_parser — the README CLI of the reference (README.md:44-64), on the GPU.
//
//   pqgpu_parser <parquet_file>
//       schema, row groups and data-page sizes of every column
//   pqgpu_parser <parquet_file> --regex-column <column> --regex <pattern> [--neg-regex]
//       global data-page ids of <column> with no value matching <pattern>
//       (with --neg-regex: no value failing to match, i.e. NOT LIKE)
#include <cstdio>
#include <cstring>
#include <iostream>
#include <string>

#include "pqgpu/reader.hpp"

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s <parquet_file> [--regex-column C --regex P [--neg-regex]]\n", argv[0]);
        return 2;
    }
    std::string col, pat;
    bool neg = false;
    for (int i = 2; i < argc; i++) {
        if (!std::strcmp(argv[i], "--regex-column") && i + 1 < argc) col = argv[++i];
        else if (!std::strcmp(argv[i], "--regex") && i + 1 < argc) pat = argv[++i];
        else if (!std::strcmp(argv[i], "--neg-regex")) neg = true;
        else { std::fprintf(stderr, "unknown argument %s\n", argv[i]); return 2; }
    }
    try {
        pqgpu::ParquetReader r;
        if (!r.open(argv[1])) return 1;
        if (col.empty()) {
            std::cout << r.schema_string();
            for (size_t p = 0; p < r.num_pages(); p++) {
                const auto& e = r.page_index_entry(p);
                std::cout << "page " << p << " rg=" << e.row_group_idx << " col=" << e.column_idx
                          << " offset=" << e.data_offset << " size=" << e.data_size << "\n";
            }
            return 0;
        }
        auto pages = r.regex_pages(col, pat, neg);
        std::cout << "column " << col << (neg ? " NOT LIKE /" : " LIKE /") << pat << "/: "
                  << pages.size() << " page(s) with no qualifying value\n";
        for (size_t id : pages) std::cout << id << "\n";
        return 0;
    } catch (const std::exception& e) {
        std::cerr << "error: " << e.what() << "\n";
        return 1;
    }
}
