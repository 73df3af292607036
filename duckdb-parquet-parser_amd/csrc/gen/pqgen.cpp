// pqgen.cpp — deterministic synthetic Parquet generator (see pqgen.h).
//
// Encoders restate the reference writer's *format* so that "ref-layout" files
// decode through exactly the page shapes the reference produces:
//   page split        parquet_writer.cpp:56-98
//   level encoding    parquet_writer.cpp:103-135 (RLE runs only)
//   index encoding    rle_bp_encoder.hpp:11-61 (RLE >= 4 repeats, else one
//                     8-value bit-packed group per run, zero-padded tail)
//   dictionary rule   parquet_writer.cpp:254-280 (first-appearance order,
//                     PLAIN when distinct > non-null / 5)
//   page headers      parquet_writer.cpp:230-242, 291-301, 353-365
//   footer            parquet_writer.cpp:463-581
// The arrow layout keeps the same header/footer but fixed rows per page and
// long bit-packed runs (up to 63 groups), RLE only for runs >= 8.
#include "pqgpu/pqgen.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

namespace {

enum { T_BOOLEAN = 0, T_INT32, T_INT64, T_INT96, T_FLOAT, T_DOUBLE, T_BYTE_ARRAY };
constexpr size_t kRefPageTarget = 1024;  // parquet_writer.hpp:35

inline uint64_t splitmix64(uint64_t& s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
inline uint64_t uniform(uint64_t& s, uint64_t n) {  // [0, n), n > 0
    return static_cast<uint64_t>((static_cast<unsigned __int128>(splitmix64(s)) * n) >> 64);
}

// ── values of one column of one row group ───────────────────────────────────
struct ColValues {
    int width = 0;                 // fixed width bytes; 0 for BYTE_ARRAY
    std::vector<uint8_t> valid;    // 1 = non-null
    std::vector<uint8_t> fixed;    // nrows * width (null rows zero)
    std::vector<uint64_t> offsets; // BYTE_ARRAY: nrows + 1
    std::vector<uint8_t> chars;
    size_t nrows() const { return valid.size(); }
    size_t len(size_t i) const { return width ? width : offsets[i + 1] - offsets[i]; }
    const uint8_t* ptr(size_t i) const {
        return width ? fixed.data() + i * width : chars.data() + offsets[i];
    }
};

int type_width(int t) {
    switch (t) {
        case T_BOOLEAN: return 1;
        case T_INT32: case T_FLOAT: return 4;
        case T_INT64: case T_DOUBLE: return 8;
        default: return 0;
    }
}

const char* kVocab[36] = {
    "furiously", "carefully", "quickly", "blithely", "slyly", "special", "requests",
    "deposits", "packages", "accounts", "ironic", "final", "regular", "express",
    "pending", "bold", "even", "silent", "unusual", "foxes", "ideas", "theodolites",
    "pinto", "beans", "instructions", "dependencies", "excuses", "platelets",
    "asymptotes", "courts", "dolphins", "across", "about", "above", "after", "against"};

uint64_t col_seed(uint64_t seed, int col, int rg) {
    uint64_t s = seed * 0x100000001B3ull + static_cast<uint64_t>(col) * 0x9E3779B97F4A7C15ull +
                 static_cast<uint64_t>(rg) * 0xD1B54A32D192ED03ull + 0x632BE59BD9B4E019ull;
    splitmix64(s);
    return s;
}

ColValues generate(const pqgen_col& c, int col, int64_t rows, int rg, uint64_t seed) {
    ColValues v;
    uint64_t s = col_seed(seed, col, rg);
    uint64_t ns = s ^ 0xA5A5A5A5DEADBEEFull;  // independent null stream
    v.width = type_width(c.type);
    v.valid.resize(rows);
    uint64_t null_thresh = 0;
    if (c.optional && c.null_frac > 0) {
        double f = c.null_frac >= 1.0 ? 1.0 : c.null_frac;
        null_thresh = f >= 1.0 ? ~0ull : static_cast<uint64_t>(f * 18446744073709551616.0);
    }
    for (int64_t i = 0; i < rows; i++)
        v.valid[i] = (null_thresh && splitmix64(ns) < null_thresh) ? 0 : 1;

    if (c.type == T_BYTE_ARRAY) {
        v.offsets.resize(rows + 1);
        v.offsets[0] = 0;
        if (c.kind == PQGEN_COMMENT) {
            int lmin = c.len_min > 0 ? c.len_min : 10, lmax = c.len_max > lmin ? c.len_max : 44;
            std::string buf;
            for (int64_t i = 0; i < rows; i++) {
                size_t L = lmin + uniform(s, lmax - lmin);
                buf.clear();
                while (buf.size() < L) {
                    if (!buf.empty()) buf.push_back(' ');
                    buf += kVocab[uniform(s, 36)];
                }
                buf.resize(L);
                if (v.valid[i]) v.chars.insert(v.chars.end(), buf.begin(), buf.end());
                v.offsets[i + 1] = v.chars.size();
            }
        } else {  // dictionary strings (also the default for other kinds)
            int dn = c.dict_size > 0 ? c.dict_size : 1000;
            int lmin = c.len_min > 0 ? c.len_min : 8, lmax = c.len_max > lmin ? c.len_max : 40;
            std::vector<std::string> dict;
            std::unordered_map<std::string, int> seen;
            while (static_cast<int>(dict.size()) < dn) {  // distinct entries
                size_t L = lmin + uniform(s, lmax - lmin);
                std::string e(L, 'a');
                for (auto& ch : e) ch = static_cast<char>('a' + uniform(s, 26));
                if (seen.emplace(e, 0).second) dict.push_back(e);
            }
            int max_run = c.max_run > 0 ? c.max_run : 16;
            int64_t i = 0;
            while (i < rows) {
                int64_t run = 1 + static_cast<int64_t>(uniform(s, max_run));
                int idx = static_cast<int>(uniform(s, dn));
                for (int64_t k = 0; k < run && i < rows; k++, i++) {
                    if (v.valid[i]) v.chars.insert(v.chars.end(), dict[idx].begin(), dict[idx].end());
                    v.offsets[i + 1] = v.chars.size();
                }
            }
        }
        return v;
    }

    v.fixed.assign(static_cast<size_t>(rows) * v.width, 0);
    for (int64_t i = 0; i < rows; i++) {
        uint64_t u = splitmix64(s);
        uint8_t* p = v.fixed.data() + i * v.width;
        if (!v.valid[i]) continue;
        if (c.kind == PQGEN_DOUBLE_RANGE && c.type == T_DOUBLE) {
            double d = static_cast<double>(u >> 11) * 0x1p-53 * 2000.0 - 1000.0;
            std::memcpy(p, &d, 8);
        } else if (c.kind == PQGEN_DOUBLE_RANGE && c.type == T_FLOAT) {
            float f = static_cast<float>(u >> 40) * 0x1p-24f * 2000.0f - 1000.0f;
            std::memcpy(p, &f, 4);
        } else if (c.kind == PQGEN_SMALL_INT) {
            uint64_t x = (static_cast<unsigned __int128>(u) * static_cast<uint64_t>(c.dict_size > 0 ? c.dict_size : 16)) >> 64;
            std::memcpy(p, &x, v.width);
        } else if (c.type == T_BOOLEAN) {
            p[0] = static_cast<uint8_t>(u & 1);
        } else {
            std::memcpy(p, &u, v.width);
        }
    }
    return v;
}

// ── thrift compact writer (own; same byte choices as thrift_writer.cpp) ────
struct TW {
    std::vector<uint8_t> b;
    int16_t last = 0;
    std::vector<int16_t> stack;
    void varint(uint64_t v) {
        while (v >= 0x80) { b.push_back(static_cast<uint8_t>(v | 0x80)); v >>= 7; }
        b.push_back(static_cast<uint8_t>(v));
    }
    void zz(int64_t v) { varint(static_cast<uint64_t>((v << 1) ^ (v >> 63))); }
    void field(int16_t id, uint8_t t) {
        int16_t d = id - last;
        if (d > 0 && d <= 15) b.push_back(static_cast<uint8_t>((d << 4) | t));
        else { b.push_back(t); zz(id); }
        last = id;
    }
    void i32(int16_t id, int32_t v) { field(id, 5); zz(v); }
    void i64(int16_t id, int64_t v) { field(id, 6); zz(v); }
    void str(int16_t id, const std::string& s) {
        field(id, 8);
        varint(s.size());
        b.insert(b.end(), s.begin(), s.end());
    }
    void list(int16_t id, uint8_t et, int32_t n) {
        field(id, 9);
        if (n < 15) b.push_back(static_cast<uint8_t>((n << 4) | et));
        else { b.push_back(static_cast<uint8_t>(0xF0 | et)); varint(n); }
    }
    void sbegin(int16_t id) { field(id, 12); stack.push_back(last); last = 0; }
    void send() { b.push_back(0); last = stack.back(); stack.pop_back(); }
    void push() { stack.push_back(last); last = 0; }
    void pop() { last = stack.back(); stack.pop_back(); }
    void stop() { b.push_back(0); }
};

void put_u32(std::vector<uint8_t>& o, uint32_t v) {
    const uint8_t* p = reinterpret_cast<const uint8_t*>(&v);
    o.insert(o.end(), p, p + 4);
}
void put_varint(std::vector<uint8_t>& o, uint32_t v) {
    while (v >= 0x80) { o.push_back(static_cast<uint8_t>(v | 0x80)); v >>= 7; }
    o.push_back(static_cast<uint8_t>(v));
}
void put_value_bytes(std::vector<uint8_t>& o, uint64_t v, int nbytes) {
    for (int i = 0; i < nbytes; i++) { o.push_back(static_cast<uint8_t>(v & 0xFF)); v >>= 8; }
}
void pack_bits(std::vector<uint8_t>& o, const uint32_t* vals, size_t n, int bw) {
    size_t start = o.size();
    o.resize(start + (n * bw + 7) / 8, 0);
    size_t bit = 0;
    for (size_t i = 0; i < n; i++)
        for (int b = 0; b < bw; b++, bit++)
            if ((vals[i] >> b) & 1) o[start + bit / 8] |= static_cast<uint8_t>(1u << (bit % 8));
}

// rle_bp_encoder.hpp:11-61 semantics.
struct RefRleBp {
    int bw, byte_w;
    uint32_t rle_count = 0, rle_value = 0, bp[8] = {}, bp_count = 0;
    std::vector<uint8_t> out;
    explicit RefRleBp(int w) : bw(w), byte_w((w + 7) / 8) {}
    void flush_rle() { put_varint(out, rle_count << 1); put_value_bytes(out, rle_value, byte_w); rle_count = 0; }
    void flush_bp() { put_varint(out, 3); pack_bits(out, bp, 8, bw); bp_count = 0; }
    void put(uint32_t v) {
        if (bp_count) { bp[bp_count++] = v; if (bp_count == 8) flush_bp(); return; }
        if (rle_count == 0) { rle_value = v; rle_count = 1; return; }
        if (rle_value == v) { rle_count++; return; }
        if (rle_count >= 4) { flush_rle(); rle_value = v; rle_count = 1; return; }
        for (uint32_t i = 0; i < rle_count; i++) bp[bp_count++] = rle_value;
        bp[bp_count++] = v;
        rle_count = 0;
        if (bp_count == 8) flush_bp();
    }
    void finish() {
        if (rle_count > 0) flush_rle();
        else if (bp_count > 0) { for (uint32_t i = bp_count; i < 8; i++) bp[i] = 0; flush_bp(); }
    }
};

// parquet_writer.cpp:103-135: one RLE run per maximal run of equal levels.
std::vector<uint8_t> ref_levels(const uint8_t* valid, size_t n, int bw) {
    std::vector<uint8_t> o;
    if (n == 0 || bw == 0) return o;
    int nb = (bw + 7) / 8;
    size_t i = 0;
    while (i < n) {
        size_t r = 1;
        while (i + r < n && valid[i + r] == valid[i]) r++;
        put_varint(o, static_cast<uint32_t>(r) << 1);
        put_value_bytes(o, valid[i] ? 1 : 0, nb);
        i += r;
    }
    return o;
}

// Arrow-style hybrid encoder: RLE for runs >= 8 at a group boundary, long
// bit-packed runs (<= 63 groups) otherwise, zero-padded final group.
std::vector<uint8_t> arrow_hybrid(const uint32_t* v, size_t n, int bw) {
    std::vector<uint8_t> o;
    std::vector<uint32_t> bp;
    int nb = (bw + 7) / 8;
    auto flush_bp = [&](bool final_flush) {
        size_t full = final_flush ? (bp.size() + 7) / 8 * 8 : bp.size() / 8 * 8;
        bp.resize(std::max(full, bp.size()), 0);
        size_t pos = 0;
        while (pos < full) {
            size_t groups = std::min<size_t>((full - pos) / 8, 63);
            put_varint(o, static_cast<uint32_t>(groups << 1 | 1));
            pack_bits(o, bp.data() + pos, groups * 8, bw);
            pos += groups * 8;
        }
        bp.erase(bp.begin(), bp.begin() + full);
    };
    size_t i = 0;
    while (i < n) {
        size_t r = 1;
        while (i + r < n && v[i + r] == v[i]) r++;
        if (r >= 8 && bp.size() % 8 == 0) {
            flush_bp(false);
            put_varint(o, static_cast<uint32_t>(r) << 1);
            put_value_bytes(o, v[i], nb);
            i += r;
        } else if (r >= 8) {
            size_t k = 8 - bp.size() % 8;
            for (size_t j = 0; j < k; j++) bp.push_back(v[i]);
            i += k;
        } else {
            for (size_t j = 0; j < r; j++) bp.push_back(v[i]);
            i += r;
        }
    }
    flush_bp(true);
    return o;
}

int dict_bit_width(uint32_t max_value) {  // parquet_writer.cpp:30-35
    if (max_value == 0) return 1;
    int bw = 0;
    while (max_value) { bw++; max_value >>= 1; }
    return bw;
}

struct Dict {
    bool use = false;
    std::vector<size_t> entry_row;  // representative row of each entry
    std::vector<uint32_t> index;    // per non-null row: dictionary index
};

// parquet_writer.cpp:254-280 (first-appearance order, PLAIN above n/5).
Dict analyze(const ColValues& v, bool allow) {
    Dict d;
    if (!allow) return d;
    size_t nn = 0;
    for (auto x : v.valid) nn += x;
    std::unordered_map<std::string, uint32_t> map;
    map.reserve(1024);
    d.index.reserve(nn);
    for (size_t i = 0; i < v.nrows(); i++) {
        if (!v.valid[i]) continue;
        std::string key(reinterpret_cast<const char*>(v.ptr(i)), v.len(i));
        if (v.width == 1 && v.fixed.size()) key.assign(1, static_cast<char>(v.ptr(i)[0] != 0));
        auto it = map.find(key);
        if (it == map.end()) {
            if (d.entry_row.size() + 1 > nn / 5) return Dict{};  // early PLAIN decision
            it = map.emplace(key, static_cast<uint32_t>(d.entry_row.size())).first;
            d.entry_row.push_back(i);
        }
        d.index.push_back(it->second);
    }
    if (d.entry_row.empty() || d.entry_row.size() > nn / 5) return Dict{};
    d.use = true;
    return d;
}

void plain_value(std::vector<uint8_t>& o, const ColValues& v, size_t i, int type) {
    if (type == T_BYTE_ARRAY) put_u32(o, static_cast<uint32_t>(v.len(i)));
    if (type == T_BOOLEAN) { o.push_back(v.ptr(i)[0] ? 1 : 0); return; }
    o.insert(o.end(), v.ptr(i), v.ptr(i) + v.len(i));
}

std::vector<uint8_t> page_header(int type, int32_t size, int32_t nvals, int32_t enc) {
    TW t;
    t.i32(1, type);
    t.i32(2, size);
    t.i32(3, size);
    if (type == 2) {
        t.sbegin(7);
        t.i32(1, nvals);
        t.i32(2, enc);
        t.send();
    } else {
        t.sbegin(5);
        t.i32(1, nvals);
        t.i32(2, enc);
        t.i32(3, 3);
        t.i32(4, 3);
        t.send();
    }
    t.stop();
    return t.b;
}

struct ChunkMeta {
    int64_t data_off, size, num_values, dict_off = -1;
};

void emit_page(std::vector<uint8_t>& f, int type, const std::vector<uint8_t>& payload, int32_t nv, int32_t enc) {
    auto h = page_header(type, static_cast<int32_t>(payload.size()), nv, enc);
    f.insert(f.end(), h.begin(), h.end());
    f.insert(f.end(), payload.begin(), payload.end());
}

ChunkMeta write_chunk(std::vector<uint8_t>& f, const pqgen_col& c, const ColValues& v, const pqgen_opts& o) {
    ChunkMeta m;
    int64_t start = static_cast<int64_t>(f.size());
    m.num_values = static_cast<int64_t>(v.nrows());
    const int max_def = c.optional ? 1 : 0;
    const bool arrow = o.layout == PQGEN_ARROW_LAYOUT;
    const size_t rpp = o.rows_per_page > 0 ? static_cast<size_t>(o.rows_per_page) : 20000;
    Dict d = analyze(v, arrow ? (!c.force_plain && (c.kind == PQGEN_DICT_STRINGS || c.kind == PQGEN_SMALL_INT)) : true);

    auto levels = [&](std::vector<uint8_t>& payload, size_t a, size_t n) {
        if (!max_def) return;
        std::vector<uint8_t> lv;
        if (arrow) {
            std::vector<uint32_t> tmp(v.valid.begin() + a, v.valid.begin() + a + n);
            lv = arrow_hybrid(tmp.data(), n, 1);
        } else {
            lv = ref_levels(v.valid.data() + a, n, 1);
        }
        put_u32(payload, static_cast<uint32_t>(lv.size()));
        payload.insert(payload.end(), lv.begin(), lv.end());
    };

    // page boundaries
    std::vector<std::pair<size_t, size_t>> pages;
    const size_t n = v.nrows();
    int bw = d.use ? dict_bit_width(static_cast<uint32_t>(d.entry_row.size() - 1)) : 0;
    if (arrow) {
        for (size_t a = 0; a < n; a += rpp) pages.push_back({a, std::min(rpp, n - a)});
    } else if (d.use) {  // parquet_writer.cpp:83-98
        size_t bpv = std::max<size_t>(1, (bw + 7) / 8), vpp = std::max<size_t>(1, kRefPageTarget / bpv);
        for (size_t a = 0; a < n; a += vpp) pages.push_back({a, std::min(vpp, n - a)});
    } else {  // parquet_writer.cpp:56-80
        size_t a = 0, est = 0;
        for (size_t i = 0; i < n; i++) {
            if (v.valid[i]) est += (c.type == T_BYTE_ARRAY ? 4 : 0) + (c.type == T_BOOLEAN ? 1 : v.len(i));
            if (est >= kRefPageTarget) { pages.push_back({a, i - a + 1}); a = i + 1; est = 0; }
        }
        if (a < n) pages.push_back({a, n - a});
    }

    if (d.use) {
        m.dict_off = start;
        std::vector<uint8_t> payload;
        for (size_t r : d.entry_row) plain_value(payload, v, r, c.type);
        emit_page(f, 2, payload, static_cast<int32_t>(d.entry_row.size()), 2);
        m.data_off = static_cast<int64_t>(f.size());
        size_t k = 0;  // running non-null index
        for (auto [a, cnt] : pages) {
            std::vector<uint8_t> payload2;
            levels(payload2, a, cnt);
            payload2.push_back(static_cast<uint8_t>(bw));
            std::vector<uint32_t> idx;
            for (size_t i = a; i < a + cnt; i++)
                if (v.valid[i]) idx.push_back(d.index[k++]);
            if (arrow) {
                auto enc = arrow_hybrid(idx.data(), idx.size(), bw);
                payload2.insert(payload2.end(), enc.begin(), enc.end());
            } else {
                RefRleBp enc(bw);
                for (auto x : idx) enc.put(x);
                enc.finish();
                payload2.insert(payload2.end(), enc.out.begin(), enc.out.end());
            }
            emit_page(f, 0, payload2, static_cast<int32_t>(cnt), 8);
        }
    } else {
        m.data_off = start;
        for (auto [a, cnt] : pages) {
            std::vector<uint8_t> payload;
            levels(payload, a, cnt);
            if (c.type == T_BOOLEAN && arrow) {  // bit-packed BOOLEAN (column_reader.cpp:197-212)
                std::vector<uint32_t> bits;
                for (size_t i = a; i < a + cnt; i++)
                    if (v.valid[i]) bits.push_back(v.ptr(i)[0] ? 1 : 0);
                pack_bits(payload, bits.data(), bits.size(), 1);
            } else {
                for (size_t i = a; i < a + cnt; i++)
                    if (v.valid[i]) plain_value(payload, v, i, c.type);
            }
            emit_page(f, 0, payload, static_cast<int32_t>(cnt), 0);
        }
    }
    m.size = static_cast<int64_t>(f.size()) - start;
    return m;
}

}  // namespace

extern "C" {

int pqgen_build(const pqgen_col* cols, int ncols, int64_t rows_per_rg, int nrg, uint64_t seed,
                const pqgen_opts* opts, uint8_t** out, size_t* out_len) {
    if (!cols || ncols <= 0 || rows_per_rg < 0 || nrg < 0 || !out || !out_len) return -1;
    pqgen_opts o{};
    if (opts) o = *opts;
    std::vector<uint8_t> f = {'P', 'A', 'R', '1'};
    std::vector<std::vector<ChunkMeta>> metas(nrg);
    for (int rg = 0; rg < nrg; rg++)
        for (int c = 0; c < ncols; c++) {
            ColValues v = generate(cols[c], c, rows_per_rg, o.first_rg + rg, seed);
            metas[rg].push_back(write_chunk(f, cols[c], v, o));
        }
    // footer (parquet_writer.cpp:463-581)
    int64_t footer_start = static_cast<int64_t>(f.size());
    TW t;
    t.i32(1, 2);
    t.list(2, 12, 1 + ncols);
    t.push();
    t.str(4, "schema");
    t.i32(5, ncols);
    t.stop();
    t.pop();
    for (int c = 0; c < ncols; c++) {
        t.push();
        t.i32(1, cols[c].type);
        t.i32(3, cols[c].optional ? 1 : 0);
        t.str(4, cols[c].name ? cols[c].name : ("c" + std::to_string(c)));
        if (cols[c].type == T_BYTE_ARRAY) t.i32(6, 0);  // UTF8
        t.stop();
        t.pop();
    }
    t.i64(3, rows_per_rg * nrg);
    t.list(4, 12, nrg);
    for (int rg = 0; rg < nrg; rg++) {
        t.push();
        t.list(1, 12, ncols);
        int64_t total = 0;
        for (int c = 0; c < ncols; c++) {
            const ChunkMeta& m = metas[rg][c];
            total += m.size;
            t.push();
            t.i64(2, m.dict_off >= 0 ? m.dict_off : m.data_off);
            t.sbegin(3);
            t.i32(1, cols[c].type);
            if (m.dict_off >= 0) { t.list(2, 5, 2); t.zz(0); t.zz(8); }
            else { t.list(2, 5, 1); t.zz(0); }
            std::string name = cols[c].name ? cols[c].name : ("c" + std::to_string(c));
            t.list(3, 8, 1);
            t.varint(name.size());
            t.b.insert(t.b.end(), name.begin(), name.end());
            t.i32(4, 0);
            t.i64(5, m.num_values);
            t.i64(6, m.size);
            t.i64(7, m.size);
            t.i64(9, m.data_off);
            if (m.dict_off >= 0) t.i64(11, m.dict_off);
            t.send();
            t.stop();
            t.pop();
        }
        t.i64(2, total);
        t.i64(3, rows_per_rg);
        t.stop();
        t.pop();
    }
    if (o.footer_pad) t.str(6, std::string("pqgen synthetic parquet; deterministic splitmix64 generator; ") +
                                   std::string(240, '.'));
    t.stop();
    f.insert(f.end(), t.b.begin(), t.b.end());
    put_u32(f, static_cast<uint32_t>(static_cast<int64_t>(f.size()) - footer_start));
    f.insert(f.end(), {'P', 'A', 'R', '1'});
    *out = static_cast<uint8_t*>(std::malloc(f.size()));
    if (!*out) return -2;
    std::memcpy(*out, f.data(), f.size());
    *out_len = f.size();
    return 0;
}

int pqgen_values_dump(const pqgen_col* col, int col_idx, int64_t rows, int rg, uint64_t seed,
                      uint8_t** out, size_t* out_len) {
    ColValues v = generate(*col, col_idx, rows, rg, seed);
    std::vector<uint8_t> d;
    for (size_t i = 0; i < v.nrows(); i++) {
        d.push_back(v.valid[i] ? 0 : 1);
        if (!v.valid[i]) continue;
        if (col->type == T_BYTE_ARRAY) put_u32(d, static_cast<uint32_t>(v.len(i)));
        if (col->type == T_BOOLEAN) d.push_back(v.ptr(i)[0] ? 1 : 0);
        else d.insert(d.end(), v.ptr(i), v.ptr(i) + v.len(i));
    }
    *out = static_cast<uint8_t*>(std::malloc(d.empty() ? 1 : d.size()));
    if (!d.empty()) std::memcpy(*out, d.data(), d.size());
    *out_len = d.size();
    return 0;
}

void pqgen_free(void* p) { std::free(p); }

}  // extern "C"
