// fuzz_host.cpp — seeded mutation fuzzing of the host code that parses
// untrusted bytes (test infrastructure; built by `make sanitize` with
// AddressSanitizer + UndefinedBehaviorSanitizer, and with ThreadSanitizer).
//
//   walk   <seed> <iters> <file>...
//       Mutates page-header bytes (and, now and then, any byte of the chunk
//       or of the footer) of each input file and runs, on every mutant:
//         pqfmt::parse_footer / leaf_columns / page_index  (ParquetReader::open,
//             parquet_reader.cpp:14-61, 495-605);
//         pqfmt::walk_chunk serially and speculatively on 16 threads (the
//             chunk's extent declared as 64 MiB, so even small inputs walk
//             through the speculative segments and linked_walk);
//       and requires the speculative result (page table, status, message)
//       to equal the serial walk's, which is ColumnReader::read_all's loop
//       (column_reader.cpp:18-71) bounded as ByteBuffer::check bounds it
//       (common.hpp:162-168; PageHeader::deserialize, metadata.cpp:121-155).
//   regex  <seed> <iters>
//       Random patterns over the supported syntax and random bytes: compile,
//       then for each pattern the DFA image (build_dfa) run on the host must
//       agree with the NFA (match_host) on random strings.
//   zstd   <seed> <iters> <file>...
//       Each file: [u32 decompressed size][one or more zstd frames].  The
//       codec pass's zstd decoder (csrc/kernels/zstd.hpp through
//       tools/zstd_check.cpp's host harness) must decode the clean frame to
//       exactly that size, then every mutant (1-4 flipped bytes, a cut tail,
//       a short output buffer) must end in a status, never a fault.
//   lz     <seed> <iters> <file>...
//       Each file: [u32 codec][u32 decompressed size][payload], codec 1
//       SNAPPY, 5 LZ4 (Hadoop framing) or 7 LZ4_RAW: the codec pass's parsers
//       (csrc/kernels/lz.hpp through tools/lz_check.cpp, with k_codec's queue
//       checks), the same clean-then-mutants rule as zstd.
//   gzip   <seed> <iters> <file>...
//       Each file: [u32 decompressed size][GZIP members or a zlib stream]:
//       the codec pass's DEFLATE decoder (csrc/kernels/deflate.hpp through
//       tools/gzip_check.cpp), the same rule as zstd.
//   threads <seed> <iters> <file>...
//       Speculative walks of several files from several host threads at
//       once (the process-wide walk pool and its busy fallback; ThreadSanitizer
//       build).
// Exit status 0 when every check held; a sanitizer report aborts.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "host/format.hpp"
#include "regex/regex.hpp"

namespace {

std::vector<uint8_t> load(const char* path) {
    std::ifstream f(path, std::ios::binary);
    return std::vector<uint8_t>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

bool same_walk(const pqfmt::WalkResult& a, const pqfmt::WalkResult& b) {
    if (a.error != b.error || a.message != b.message || a.pages.size() != b.pages.size()) return false;
    return a.pages.empty() || std::memcmp(a.pages.data(), b.pages.data(), a.pages.size() * sizeof(pq_page_desc)) == 0;
}

struct Chunk {
    pq_chunk_desc d;
    size_t lo, hi;  // byte extent of the chunk in the file
};

// The chunks of a parsed file, as pq_file_chunk describes them.
std::vector<Chunk> chunks_of(const std::vector<uint8_t>& f) {
    std::vector<Chunk> out;
    try {
        const pqfmt::FileMeta fm = pqfmt::parse_footer(f.data(), f.size());
        const auto cols = pqfmt::leaf_columns(fm);
        for (const auto& rg : fm.row_groups)
            for (const auto& lc : cols) {
                if (lc.column_index >= static_cast<int>(rg.columns.size()) || !rg.columns[lc.column_index].meta) continue;
                const auto& m = *rg.columns[lc.column_index].meta;
                Chunk c{};
                c.d.num_values = m.num_values;
                c.d.data_page_offset = m.data_page_offset;
                c.d.has_dictionary_page_offset = m.dictionary_page_offset.has_value();
                c.d.dictionary_page_offset = m.dictionary_page_offset.value_or(0);
                c.d.codec = m.codec;
                c.d.type = lc.type;
                c.d.max_def_level = lc.max_def;
                c.d.max_rep_level = lc.max_rep;
                c.d.total_compressed_size = m.total_compressed;
                const int64_t off = c.d.has_dictionary_page_offset ? std::min(c.d.dictionary_page_offset, c.d.data_page_offset)
                                                                 : c.d.data_page_offset;
                c.lo = static_cast<size_t>(std::max<int64_t>(off, 0));
                c.hi = std::min(f.size(), c.lo + static_cast<size_t>(std::max<int64_t>(m.total_compressed, 0)));
                out.push_back(c);
            }
    } catch (const std::exception&) {
    }
    return out;
}

pqfmt::WalkResult walk(const std::vector<uint8_t>& f, pq_chunk_desc d, bool spec) {
    d.total_compressed_size = spec ? (int64_t{64} << 20) : 0;
    d.ext_flags = PQ_EXT_CODECS | PQ_EXT_PAGE_V2;
    return pqfmt::walk_chunk(f.data(), f.size(), d, spec ? 16 : 1);
}

int fuzz_walk(uint64_t seed, int iters, int nfiles, char** files) {
    std::mt19937_64 rng(seed);
    long checks = 0, errors = 0;
    for (int fi = 0; fi < nfiles; fi++) {
        const std::vector<uint8_t> orig = load(files[fi]);
        if (orig.size() < 12) continue;
        const std::vector<Chunk> chunks = chunks_of(orig);
        // header positions of the clean file: the mutations' main target
        std::vector<std::pair<size_t, size_t>> hdrs;
        for (const auto& c : chunks) {
            const auto w = walk(orig, c.d, false);
            for (const auto& p : w.pages)
                hdrs.emplace_back(static_cast<size_t>(p.header_offset),
                                  static_cast<size_t>(p.payload_offset - p.header_offset));
        }
        const size_t flen = orig.size();
        for (int it = 0; it < iters; it++) {
            std::vector<uint8_t> f = orig;
            const int nmut = 1 + static_cast<int>(rng() % 4);
            for (int k = 0; k < nmut; k++) {
                const uint32_t r = static_cast<uint32_t>(rng() % 100);
                size_t pos;
                if (r < 70 && !hdrs.empty()) {  // a page header byte
                    const auto& h = hdrs[rng() % hdrs.size()];
                    pos = h.first + rng() % std::max<size_t>(h.second, 1);
                } else if (r < 90) {  // anywhere before the footer
                    pos = rng() % flen;
                } else {  // the footer (its length word and magic excluded)
                    const uint32_t flen_word = f[flen - 8] | (f[flen - 7] << 8) | (f[flen - 6] << 16) | (uint32_t(f[flen - 5]) << 24);
                    const size_t fstart = flen_word + 8 <= flen ? flen - 8 - flen_word : 0;
                    pos = fstart + rng() % std::max<size_t>(flen - 8 - fstart, 1);
                }
                if (pos >= flen) continue;
                switch (rng() % 4) {
                    case 0: f[pos] ^= static_cast<uint8_t>(1u << (rng() % 8)); break;
                    case 1: f[pos] = static_cast<uint8_t>(rng()); break;
                    case 2: f[pos] = static_cast<uint8_t>(f[pos] + 1); break;
                    default: f[pos] = (rng() & 1) ? 0xFF : 0x00; break;
                }
            }
            if (rng() % 16 == 0) f.resize(rng() % flen);  // truncated file
            // ParquetReader::open on the mutant: must throw or succeed, nothing else
            std::vector<Chunk> mc = chunks_of(f);
            try {
                const pqfmt::FileMeta fm = pqfmt::parse_footer(f.data(), f.size());
                (void)pqfmt::page_index(f.data(), f.size(), fm);
            } catch (const std::exception&) {
            }
            // the clean file's chunk descriptors on the mutated bytes, and the
            // mutant's own (a mutated footer describes other chunks)
            std::vector<pq_chunk_desc> descs;
            for (const auto& c : chunks) descs.push_back(c.d);
            for (const auto& c : mc) descs.push_back(c.d);
            for (const auto& d : descs) {
                if (d.num_values > (int64_t{1} << 26)) continue;  // (a walk of 2^26+ pages: memory, not parsing)
                const auto a = walk(f, d, false);
                const auto b = walk(f, d, true);
                checks++;
                if (a.error) errors++;
                if (!same_walk(a, b)) {
                    std::fprintf(stderr, "walk mismatch: file %s iter %d chunk@%lld: serial %zu pages rc %d '%s', "
                                         "speculative %zu pages rc %d '%s'\n",
                                 files[fi], it, static_cast<long long>(d.data_page_offset), a.pages.size(), a.error,
                                 a.message.c_str(), b.pages.size(), b.error, b.message.c_str());
                    return 1;
                }
            }
        }
    }
    std::printf("walk: %ld chunk walks, %ld with errors, speculative == serial on all\n", checks, errors);
    return 0;
}

// The DFA image (regex.hpp DevDfa + u16 rows) run on the host, as the
// kernels read it.
bool dfa_match(const std::vector<uint8_t>& img, const uint8_t* s, size_t n) {
    const auto* D = reinterpret_cast<const pqre::DevDfa*>(img.data());
    if (n == 0) return D->empty_string != 0;
    if (D->nonempty_trivial) return true;
    const uint16_t* T = reinterpret_cast<const uint16_t*>(img.data() + sizeof(pqre::DevDfa));
    uint32_t st = pqre::DFA_START;
    bool acc_end = false;
    for (size_t i = 0; i < n; i++) {
        uint32_t e;
        if (D->full) {
            e = T[st * (pqre::kDfaRowBytes / 2) + s[i]];
            const uint32_t nxt = e / pqre::kDfaRowBytes;
            acc_end = T[nxt * (pqre::kDfaRowBytes / 2) + 256] != 0;
            st = nxt;
        } else {
            e = T[st * D->nclasses + D->cls_of[s[i]]];
            st = e & 0x7FFFu;
            acc_end = (e & 0x8000u) != 0;
        }
        if (st == pqre::DFA_ACCEPT) return true;
        if (st == pqre::DFA_DEAD) return false;
    }
    return acc_end;
}

int fuzz_regex(uint64_t seed, int iters) {
    std::mt19937_64 rng(seed);
    static const char* atoms[] = {"a", "b", "c", "e", "x", ".", "[a-c]", "[^ab]", "\\d", "\\w", "\\s", "\\D", "\\W",
                                  "\\S", " ", "ab", "[0-9]", "[a-z ]", "q", "\\.", "(", ")", "|", "*", "+", "?",
                                  "{2}", "{1,3}", "{0,2}", "^", "$", "*?", "(?:", "[", "]", "\\", "{", "\\A", "\\Z"};
    const int natoms = static_cast<int>(sizeof(atoms) / sizeof(atoms[0]));
    long compiled = 0, rejected = 0, dfas = 0, strings = 0;
    for (int it = 0; it < iters; it++) {
        std::string pat;
        const int len = 1 + static_cast<int>(rng() % 10);
        for (int k = 0; k < len; k++) pat += atoms[rng() % natoms];
        if (rng() % 8 == 0) pat[rng() % pat.size()] = static_cast<char>(rng());  // any byte
        pqre::Program prog;
        std::string msg;
        if (pqre::compile(pat, &prog, &msg) != 0) {
            rejected++;
            continue;
        }
        compiled++;
        std::vector<uint8_t> img;
        if (!pqre::build_dfa(prog, &img)) continue;
        dfas++;
        static const uint8_t alpha[] = {'a', 'b', 'c', 'e', 'x', 'q', ' ', '1', '.', 'Z', 0x00, 0xC3, 0xA9, '\n', '_'};
        for (int k = 0; k < 40; k++) {
            uint8_t s[24];
            const size_t n = rng() % sizeof(s);
            for (size_t j = 0; j < n; j++) s[j] = (rng() % 4) ? alpha[rng() % sizeof(alpha)] : static_cast<uint8_t>(rng());
            strings++;
            if (pqre::match_host(prog, s, n) != dfa_match(img, s, n)) {
                std::fprintf(stderr, "regex mismatch: pattern '%s' on %zu bytes: nfa %d dfa %d\n", pat.c_str(), n,
                             static_cast<int>(pqre::match_host(prog, s, n)), static_cast<int>(dfa_match(img, s, n)));
                return 1;
            }
        }
    }
    std::printf("regex: %ld patterns compiled, %ld rejected, %ld DFAs, %ld strings: DFA == NFA on all\n", compiled,
                rejected, dfas, strings);
    return 0;
}

int fuzz_threads(uint64_t seed, int iters, int nfiles, char** files) {
    std::vector<std::vector<uint8_t>> data;
    for (int i = 0; i < nfiles; i++) data.push_back(load(files[i]));
    std::atomic<int> bad{0};
    std::vector<std::thread> th;
    for (int t = 0; t < 4; t++)
        th.emplace_back([&, t] {
            std::mt19937_64 rng(seed + t);
            for (int it = 0; it < iters; it++) {
                const auto& f = data[rng() % data.size()];
                for (const auto& c : chunks_of(f))
                    if (!same_walk(walk(f, c.d, false), walk(f, c.d, true))) bad++;
            }
        });
    for (auto& x : th) x.join();
    std::printf("threads: 4 host threads x %d walks each, %d mismatches\n", iters, bad.load());
    return bad.load() ? 1 : 0;
}

}  // namespace

extern "C" int zs_decompress(const uint8_t* src, uint32_t len, uint8_t* dst, uint32_t cap, uint32_t* out_len);
extern "C" int gz_decompress(const uint8_t* src, uint32_t len, uint8_t* dst, uint32_t cap, uint32_t* out_len);
extern "C" int lz_decompress(int codec, const uint8_t* src, uint32_t len, uint8_t* dst, uint32_t cap, uint32_t ring,
                             uint32_t* out_len);

// The clean payload of each file must decode to exactly its size, then every
// mutant (1-4 flipped bytes, a cut tail, a short output buffer) must end in a
// status with no more bytes written than the output holds.  `hdr`: the file's
// u32 header words ([size] for zstd, [codec][size] for lz); dec(hdr, src, len,
// dst, cap, out_len) decodes one payload.
template <class Dec>
int fuzz_payloads(const char* name, uint64_t seed, int iters, int nfiles, char** files, int hdr, Dec&& dec) {
    std::mt19937_64 rng(seed);
    long mutants = 0, rejected = 0;
    for (int fi = 0; fi < nfiles; fi++) {
        std::ifstream in(files[fi], std::ios::binary);
        std::vector<uint8_t> f((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
        if (f.size() < static_cast<size_t>(4 * hdr)) return 3;
        uint32_t h[2] = {0, 0};
        std::memcpy(h, f.data(), 4 * static_cast<size_t>(hdr));
        const uint32_t want = h[hdr - 1];
        const std::vector<uint8_t> clean(f.begin() + 4 * hdr, f.end());
        std::vector<uint8_t> out(static_cast<size_t>(want) + 16);
        uint32_t ol = 0;
        // (exact-size heap buffers, so ASan sees any read or write past them)
        {
            std::vector<uint8_t> src(clean);
            const int rc = dec(h, src.data(), static_cast<uint32_t>(src.size()), out.data(), want, &ol);
            if (rc != 0 || ol != want) {
                std::printf("clean payload %s: rc %d, %u of %u bytes\n", files[fi], rc, ol, want);
                return 1;
            }
        }
        for (int it = 0; it < iters; it++) {
            std::vector<uint8_t> m(clean);
            const int kind = static_cast<int>(rng() % 8);
            if (kind == 0 && m.size() > 1) {
                m.resize(1 + rng() % (m.size() - 1));  // a cut tail
            } else if (!m.empty()) {
                const int flips = 1 + static_cast<int>(rng() % 4);
                for (int k = 0; k < flips; k++) m[rng() % m.size()] = static_cast<uint8_t>(rng());
            }
            const uint32_t cap = kind == 1 ? static_cast<uint32_t>(rng() % (want + 1)) : want;
            std::vector<uint8_t> dst(static_cast<size_t>(cap) + 1);
            ol = 0;
            const int rc = dec(h, m.data(), static_cast<uint32_t>(m.size()), dst.data(), cap, &ol);
            if (ol > cap) {
                std::printf("mutant wrote %u bytes into %u\n", ol, cap);
                return 1;
            }
            mutants++;
            rejected += rc != 0;
        }
    }
    std::printf("%s: %ld mutants, %ld rejected, no fault\n", name, mutants, rejected);
    return 0;
}

int fuzz_zstd(uint64_t seed, int iters, int nfiles, char** files) {
    return fuzz_payloads("zstd", seed, iters, nfiles, files, 1,
                         [](const uint32_t*, const uint8_t* s, uint32_t n, uint8_t* d, uint32_t cap, uint32_t* ol) {
                             return zs_decompress(s, n, d, cap, ol);
                         });
}

int fuzz_gzip(uint64_t seed, int iters, int nfiles, char** files) {
    return fuzz_payloads("gzip", seed, iters, nfiles, files, 1,
                         [](const uint32_t*, const uint8_t* s, uint32_t n, uint8_t* d, uint32_t cap, uint32_t* ol) {
                             return gz_decompress(s, n, d, cap, ol);
                         });
}

// both of k_codec's history sizes: the 64 KiB ring and the small-page 8 KiB one
int fuzz_lz(uint64_t seed, int iters, int nfiles, char** files) {
    return fuzz_payloads("lz", seed, iters, nfiles, files, 2,
                         [](const uint32_t* h, const uint8_t* s, uint32_t n, uint8_t* d, uint32_t cap, uint32_t* ol) {
                             const uint32_t ring = cap < 8192 ? 8192u : 65536u;
                             return lz_decompress(static_cast<int>(h[0]), s, n, d, cap, ring, ol);
                         });
}

int main(int argc, char** argv) {
    if (argc < 4) {
        std::fprintf(stderr, "usage: %s walk|regex|threads|zstd|lz|gzip <seed> <iters> [file...]\n", argv[0]);
        return 2;
    }
    const std::string mode = argv[1];
    const uint64_t seed = std::strtoull(argv[2], nullptr, 10);
    const int iters = std::atoi(argv[3]);
    if (mode == "walk") return fuzz_walk(seed, iters, argc - 4, argv + 4);
    if (mode == "regex") return fuzz_regex(seed, iters);
    if (mode == "threads") return fuzz_threads(seed, iters, argc - 4, argv + 4);
    if (mode == "zstd") return fuzz_zstd(seed, iters, argc - 4, argv + 4);
    if (mode == "lz") return fuzz_lz(seed, iters, argc - 4, argv + 4);
    if (mode == "gzip") return fuzz_gzip(seed, iters, argc - 4, argv + 4);
    return 2;
}
