// format.cpp — see format.hpp for the reference behaviour each part follows.
#include "format.hpp"

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <thread>

#include <unistd.h>

namespace pqfmt {

// common.hpp:136-147 semantics: 7-bit groups, "varint too long" past 63 bits.
uint64_t Cursor::varint() {
    uint64_t r = 0;
    int shift = 0;
    for (;;) {
        uint8_t b = byte();
        r |= static_cast<uint64_t>(b & 0x7F) << shift;
        if ((b & 0x80) == 0) break;
        shift += 7;
        if (shift > 63) throw Error(PQ_ERR_THRIFT, "varint too long");
    }
    return r;
}

bool Thrift::field(int16_t& id, uint8_t& type) {  // thrift.cpp:6-21
    uint8_t b = c_.byte();
    if (b == 0) { id = 0; type = 0; return false; }
    type = b & 0x0F;
    int16_t delta = (b >> 4) & 0x0F;
    id = delta ? static_cast<int16_t>(last_ + delta) : static_cast<int16_t>(c_.zigzag());
    last_ = id;
    // a nonzero byte whose type nibble is 0 (so delta != 0) is a STOP too: every
    // struct loop of the reference breaks on fh.type == CT_STOP (metadata.cpp:8 ff.,
    // thrift.cpp:110), not on the byte
    return type != 0;
}

std::string Thrift::str() {  // thrift.cpp:35-39
    uint32_t n = static_cast<uint32_t>(c_.varint());
    const uint8_t* p = c_.bytes(n);
    return std::string(reinterpret_cast<const char*>(p), n);
}

void Thrift::list(uint8_t& et, int32_t& n) {  // thrift.cpp:44-55
    uint8_t b = c_.byte();
    et = b & 0x0F;
    n = ((b >> 4) & 0x0F) == 0x0F ? static_cast<int32_t>(c_.varint()) : (b >> 4) & 0x0F;
}

void Thrift::skip(uint8_t type) {  // thrift.cpp:67-119
    switch (type) {
        case 1: case 2: return;
        case 3: c_.byte(); return;
        case 4: case 5: case 6: c_.varint(); return;
        case 7: c_.bytes(8); return;
        case 8: str(); return;
        case 9: case 10: {
            uint8_t et; int32_t n;
            list(et, n);
            for (int32_t i = 0; i < n; i++) skip(et);
            return;
        }
        case 11: {
            int32_t n = static_cast<int32_t>(c_.varint());
            if (n > 0) {
                uint8_t kv = c_.byte();
                for (int32_t i = 0; i < n; i++) { skip((kv >> 4) & 0x0F); skip(kv & 0x0F); }
            }
            return;
        }
        case 12: {
            push();
            int16_t id; uint8_t t;
            while (field(id, t)) skip(t);
            pop();
            return;
        }
        default:
            throw Error(PQ_ERR_THRIFT, "ThriftReader::skip: unknown type " + std::to_string(type));
    }
}

namespace {

SchemaElement read_schema(Thrift& t) {  // metadata.cpp:5-22
    SchemaElement s;
    int16_t id; uint8_t ty;
    while (t.field(id, ty)) {
        switch (id) {
            case 1: s.type = t.i32(); break;
            case 2: s.type_length = t.i32(); break;
            case 3: s.repetition = t.i32(); break;
            case 4: s.name = t.str(); break;
            case 5: s.num_children = t.i32(); break;
            case 6: s.converted_type = t.i32(); break;
            case 7: s.scale = t.i32(); break;
            case 8: s.precision = t.i32(); break;
            case 9: s.field_id = t.i32(); break;
            default: t.skip(ty);
        }
    }
    return s;
}

ColumnMeta read_column_meta(Thrift& t) {  // metadata.cpp:36-64
    ColumnMeta m;
    int16_t id; uint8_t ty;
    while (t.field(id, ty)) {
        switch (id) {
            case 1: m.type = t.i32(); break;
            case 2: { uint8_t et; int32_t n; t.list(et, n); for (int32_t i = 0; i < n; i++) m.encodings.push_back(t.i32()); break; }
            case 3: { uint8_t et; int32_t n; t.list(et, n); for (int32_t i = 0; i < n; i++) m.path.push_back(t.str()); break; }
            case 4: m.codec = t.i32(); break;
            case 5: m.num_values = t.i64(); break;
            case 6: m.total_uncompressed = t.i64(); break;
            case 7: m.total_compressed = t.i64(); break;
            case 9: m.data_page_offset = t.i64(); break;
            case 10: m.index_page_offset = t.i64(); break;
            case 11: m.dictionary_page_offset = t.i64(); break;
            default: t.skip(ty);
        }
    }
    return m;
}

ColumnChunkMeta read_chunk(Thrift& t) {  // metadata.cpp:68-86
    ColumnChunkMeta c;
    int16_t id; uint8_t ty;
    while (t.field(id, ty)) {
        switch (id) {
            case 1: c.file_path = t.str(); break;
            case 2: c.file_offset = t.i64(); break;
            case 3: t.push(); c.meta = read_column_meta(t); t.pop(); break;
            default: t.skip(ty);
        }
    }
    return c;
}

RowGroupMeta read_row_group(Thrift& t) {  // metadata.cpp:159-180
    RowGroupMeta r;
    int16_t id; uint8_t ty;
    while (t.field(id, ty)) {
        switch (id) {
            case 1: {
                uint8_t et; int32_t n;
                t.list(et, n);
                for (int32_t i = 0; i < n; i++) { t.push(); r.columns.push_back(read_chunk(t)); t.pop(); }
                break;
            }
            case 2: r.total_byte_size = t.i64(); break;
            case 3: r.num_rows = t.i64(); break;
            default: t.skip(ty);
        }
    }
    return r;
}

void skip_key_value(Thrift& t) {  // metadata.cpp:184-194
    int16_t id; uint8_t ty;
    while (t.field(id, ty)) {
        if (id == 1 || id == 2) t.str();
        else t.skip(ty);
    }
}

// The schema is a pre-order list whose groups give their child counts.  The
// reference walks it without bounds (skip_schema_subtree reads past the list
// when a count overstates the elements left: undefined behaviour); here a
// count that runs past the list, or nesting deeper than kMaxSchemaDepth, is
// an error (fuzz_host found the unbounded read).
constexpr int kMaxSchemaDepth = 1000;
[[noreturn]] void schema_error() {
    throw Error(PQ_ERR_UNSUPPORTED, "schema: a group's num_children runs past the schema list");
}

int skip_subtree(const FileMeta& fm, int idx, int depth) {  // parquet_reader.cpp:545-557
    const int n = static_cast<int>(fm.schema.size());
    if (idx >= n || depth > kMaxSchemaDepth) schema_error();
    int children = fm.schema[idx].num_children.value_or(0);
    idx++;
    for (int i = 0; i < children; i++) {
        if (idx >= n) schema_error();
        if (fm.schema[idx].num_children.value_or(0) > 0) idx = skip_subtree(fm, idx, depth + 1);
        else idx++;
    }
    return idx;
}

void build_leaves(const FileMeta& fm, int idx, int end, int16_t def, int16_t rep, int& col,
                  std::vector<LeafColumn>& out, int depth = 0) {  // parquet_reader.cpp:495-543
    if (depth > kMaxSchemaDepth) schema_error();
    while (idx < end) {
        const SchemaElement& e = fm.schema[idx];
        int16_t d = def, r = rep;
        if (e.repetition) {
            if (*e.repetition == 1) d++;
            else if (*e.repetition == 2) { d++; r++; }
        }
        if (e.num_children.value_or(0) > 0) {
            int children = *e.num_children;
            idx++;
            int i = idx, remaining = children;
            while (remaining > 0 && i < end) {
                remaining--;
                if (fm.schema[i].num_children.value_or(0) > 0) i = skip_subtree(fm, i, depth + 1);
                else i++;
            }
            build_leaves(fm, idx, i, d, r, col, out, depth + 1);
            idx = i;
        } else {
            LeafColumn lc;
            lc.name = e.name;
            lc.type = e.type.value_or(PQ_BYTE_ARRAY);
            lc.column_index = col++;
            lc.max_def = d;
            lc.max_rep = r;
            lc.repetition = e.repetition;
            lc.converted_type = e.converted_type;
            out.push_back(lc);
            idx++;
        }
    }
}

}  // namespace

FileMeta parse_footer(const uint8_t* file, size_t len) {  // parquet_reader.cpp:14-61
    if (len < 12) throw Error(PQ_ERR_ARG, "file too small to be a Parquet file");
    if (std::memcmp(file, "PAR1", 4) != 0) throw Error(PQ_ERR_ARG, "missing PAR1 magic at start");
    if (std::memcmp(file + len - 4, "PAR1", 4) != 0) throw Error(PQ_ERR_ARG, "missing PAR1 magic at end");
    uint32_t flen;
    std::memcpy(&flen, file + len - 8, 4);
    if (static_cast<uint64_t>(flen) + 8 > len) throw Error(PQ_ERR_ARG, "invalid footer length");
    Thrift t(file + len - 8 - flen, flen);
    FileMeta fm;
    int16_t id; uint8_t ty;
    while (t.field(id, ty)) {  // metadata.cpp:198-242
        switch (id) {
            case 1: fm.version = t.i32(); break;
            case 2: { uint8_t et; int32_t n; t.list(et, n); for (int32_t i = 0; i < n; i++) { t.push(); fm.schema.push_back(read_schema(t)); t.pop(); } break; }
            case 3: fm.num_rows = t.i64(); break;
            case 4: { uint8_t et; int32_t n; t.list(et, n); for (int32_t i = 0; i < n; i++) { t.push(); fm.row_groups.push_back(read_row_group(t)); t.pop(); } break; }
            case 5: { uint8_t et; int32_t n; t.list(et, n); for (int32_t i = 0; i < n; i++) { t.push(); skip_key_value(t); t.pop(); } break; }
            case 6: fm.created_by = t.str(); break;
            default: t.skip(ty);
        }
    }
    return fm;
}

std::vector<LeafColumn> leaf_columns(const FileMeta& fm) {
    std::vector<LeafColumn> out;
    if (fm.schema.empty()) return out;
    int col = 0;
    build_leaves(fm, 1, static_cast<int>(fm.schema.size()), 0, 0, col, out);
    return out;
}

PageHeader read_page_header(const uint8_t* file, size_t len, size_t off) {  // metadata.cpp:121-155
    uint8_t win[256] = {0};  // column_reader.cpp:34-38: fixed window, zeros past EOF
    if (off < len) std::memcpy(win, file + off, std::min<size_t>(256, len - off));
    Thrift t(win, sizeof win);
    PageHeader h;
    int16_t id; uint8_t ty;
    while (t.field(id, ty)) {
        switch (id) {
            case 1: h.type = t.i32(); break;
            case 2: h.uncompressed = t.i32(); break;
            case 3: h.compressed = t.i32(); break;
            case 4: t.i32(); break;
            case 5: {  // DataPageHeader, metadata.cpp:90-102
                t.push();
                h.has_data = true;
                h.data_num_values = 0;
                h.data_encoding = 0;
                int16_t i2; uint8_t t2;
                while (t.field(i2, t2)) {
                    if (i2 == 1) h.data_num_values = t.i32();
                    else if (i2 == 2) h.data_encoding = t.i32();
                    else if (i2 == 3 || i2 == 4) t.i32();
                    else t.skip(t2);
                }
                t.pop();
                break;
            }
            case 8: {  // DataPageHeaderV2 (parquet.thrift; skipped by the reference)
                if (ty != 12) {  // not a struct: skipped by its wire type, as the reference does
                    t.skip(ty);
                    break;
                }
                t.push();
                h.has_v2 = true;
                int16_t i2; uint8_t t2;
                while (t.field(i2, t2)) {
                    if (t2 == 5 && i2 == 1) h.v2_num_values = t.i32();
                    else if (t2 == 5 && i2 == 4) h.v2_encoding = t.i32();
                    else if (t2 == 5 && i2 == 5) h.v2_def_len = t.i32();
                    else if (t2 == 5 && i2 == 6) h.v2_rep_len = t.i32();
                    else if ((t2 == 1 || t2 == 2) && i2 == 7) h.v2_compressed = t2 == 1;
                    else t.skip(t2);
                }
                t.pop();
                break;
            }
            case 7: {  // DictionaryPageHeader, metadata.cpp:106-117
                t.push();
                h.has_dict = true;
                h.dict_num_values = 0;
                int16_t i2; uint8_t t2;
                while (t.field(i2, t2)) {
                    if (i2 == 1) h.dict_num_values = t.i32();
                    else if (i2 == 2) t.i32();
                    else if (i2 == 3) { /* read_bool: no bytes */ }
                    else t.skip(t2);
                }
                t.pop();
                break;
            }
            default: t.skip(ty);
        }
    }
    h.header_size = t.pos();
    return h;
}

namespace {

// Non-throwing page-header parse over the same 256-byte window (zeros past
// EOF).  For every header read_page_header accepts it yields the identical
// PageHeader; on any condition where read_page_header would throw it returns
// false (the walk then re-parses with read_page_header for the exact error).
// No allocation: the walk calls it once per page, the speculative walk at
// candidate positions.
class FastHdr {
public:
    FastHdr(const uint8_t* file, size_t len, size_t off) {
        if (off < len && len - off >= 256) {
            p_ = file + off;
        } else {
            std::memset(win_, 0, sizeof win_);
            if (off < len) std::memcpy(win_, file + off, len - off);
            p_ = win_;
        }
        b_ = p_;
        e_ = p_ + 256;
    }
    bool parse(PageHeader& h) {
        int16_t last = 0;
        for (;;) {
            int16_t id;
            uint8_t ty;
            if (!field(last, id, ty)) return false;
            if (ty == 0 && id == 0) break;
            switch (id) {
                case 1: if (!i32(h.type)) return false; break;
                case 2: if (!i32(h.uncompressed)) return false; break;
                case 3: if (!i32(h.compressed)) return false; break;
                case 4: { int32_t x; if (!i32(x)) return false; break; }
                case 5: {
                    h.has_data = true;
                    h.data_num_values = 0;
                    h.data_encoding = 0;
                    int16_t l2 = 0;
                    for (;;) {
                        int16_t i2; uint8_t t2;
                        if (!field(l2, i2, t2)) return false;
                        if (t2 == 0 && i2 == 0) break;
                        int32_t x;
                        if (i2 == 1) { if (!i32(h.data_num_values)) return false; }
                        else if (i2 == 2) { if (!i32(h.data_encoding)) return false; }
                        else if (i2 == 3 || i2 == 4) { if (!i32(x)) return false; }
                        else if (!skip(t2, 0)) return false;
                    }
                    break;
                }
                case 8: {  // DataPageHeaderV2
                    if (ty != 12) {  // not a struct: skipped by its wire type (metadata.cpp:149-151)
                        if (!skip(ty, 0)) return false;
                        break;
                    }
                    h.has_v2 = true;
                    int16_t l2 = 0;
                    for (;;) {
                        int16_t i2; uint8_t t2;
                        if (!field(l2, i2, t2)) return false;
                        if (t2 == 0 && i2 == 0) break;
                        if (t2 == 5 && i2 == 1) { if (!i32(h.v2_num_values)) return false; }
                        else if (t2 == 5 && i2 == 4) { if (!i32(h.v2_encoding)) return false; }
                        else if (t2 == 5 && i2 == 5) { if (!i32(h.v2_def_len)) return false; }
                        else if (t2 == 5 && i2 == 6) { if (!i32(h.v2_rep_len)) return false; }
                        else if ((t2 == 1 || t2 == 2) && i2 == 7) h.v2_compressed = t2 == 1;
                        else if (!skip(t2, 0)) return false;
                    }
                    break;
                }
                case 7: {
                    h.has_dict = true;
                    h.dict_num_values = 0;
                    int16_t l2 = 0;
                    for (;;) {
                        int16_t i2; uint8_t t2;
                        if (!field(l2, i2, t2)) return false;
                        if (t2 == 0 && i2 == 0) break;
                        int32_t x;
                        if (i2 == 1) { if (!i32(h.dict_num_values)) return false; }
                        else if (i2 == 2) { if (!i32(x)) return false; }
                        else if (i2 == 3) { /* read_bool: no bytes */ }
                        else if (!skip(t2, 0)) return false;
                    }
                    break;
                }
                default: if (!skip(ty, 0)) return false;
            }
        }
        h.header_size = static_cast<size_t>(p_ - b_);
        return true;
    }

private:
    bool byte(uint8_t& v) { if (p_ >= e_) return false; v = *p_++; return true; }
    bool varint(uint64_t& r) {
        r = 0;
        for (int shift = 0;; shift += 7) {
            if (shift > 63) return false;
            uint8_t b;
            if (!byte(b)) return false;
            r |= static_cast<uint64_t>(b & 0x7F) << shift;
            if ((b & 0x80) == 0) return true;
        }
    }
    bool zigzag(int64_t& v) {
        uint64_t u;
        if (!varint(u)) return false;
        v = static_cast<int64_t>((u >> 1) ^ (~(u & 1) + 1));
        return true;
    }
    bool i32(int32_t& v) { int64_t x; if (!zigzag(x)) return false; v = static_cast<int32_t>(x); return true; }
    // id = 0, type = 0 at STOP
    bool field(int16_t& last, int16_t& id, uint8_t& type) {
        uint8_t b;
        if (!byte(b)) return false;
        if (b == 0) { id = 0; type = 0; return true; }
        type = b & 0x0F;
        const int16_t delta = (b >> 4) & 0x0F;
        if (delta) {
            id = static_cast<int16_t>(last + delta);
        } else {
            int64_t z;
            if (!zigzag(z)) return false;
            id = static_cast<int16_t>(z);
        }
        last = id;
        if (type == 0) id = 0;  // type nibble 0 ends the struct like the STOP byte (Thrift::field)
        return true;
    }
    bool bytes(uint64_t n) { if (n > static_cast<uint64_t>(e_ - p_)) return false; p_ += n; return true; }
    bool skip(uint8_t type, int depth) {
        if (depth > 256) return false;
        uint64_t u;
        switch (type) {
            case 1: case 2: return true;
            case 3: { uint8_t b; return byte(b); }
            case 4: case 5: case 6: return varint(u);
            case 7: return bytes(8);
            case 8: return varint(u) && bytes(static_cast<uint32_t>(u));
            case 9: case 10: {
                uint8_t b;
                if (!byte(b)) return false;
                const uint8_t et = b & 0x0F;
                int32_t n = (b >> 4) & 0x0F;
                if (n == 0x0F) { if (!varint(u)) return false; n = static_cast<int32_t>(u); }
                if (et == 1 || et == 2) return true;  // bool elements take no bytes (n may be ~2^31)
                for (int32_t i = 0; i < n; i++) if (!skip(et, depth + 1)) return false;
                return true;
            }
            case 11: {
                if (!varint(u)) return false;
                const int32_t n = static_cast<int32_t>(u);
                if (n > 0) {
                    uint8_t kv;
                    if (!byte(kv)) return false;
                    const uint8_t kt = (kv >> 4) & 0x0F, vt = kv & 0x0F;
                    if ((kt == 1 || kt == 2) && (vt == 1 || vt == 2)) return true;  // entries take no bytes
                    for (int32_t i = 0; i < n; i++)
                        if (!skip((kv >> 4) & 0x0F, depth + 1) || !skip(kv & 0x0F, depth + 1)) return false;
                }
                return true;
            }
            case 12: {
                int16_t last = 0;
                for (;;) {
                    int16_t id; uint8_t t;
                    if (!field(last, id, t)) return false;
                    if (t == 0 && id == 0) return true;
                    if (!skip(t, depth + 1)) return false;
                }
            }
            default: return false;
        }
    }
    uint8_t win_[256];
    const uint8_t *p_, *b_, *e_;
};

// Exact header at `cur`: the fast parse, or read_page_header's exception.
inline PageHeader header_at(const uint8_t* file, size_t len, size_t cur) {
    PageHeader h;
    if (FastHdr(file, len, cur).parse(h)) return h;
    return read_page_header(file, len, cur);  // throws the reference's error
}

}  // namespace

namespace {

// A header the fast parse accepts and that a real page chain could hold.
inline bool plausible(const PageHeader& h, size_t pos, size_t end) {
    if (h.type < 0 || h.type > 3 || h.compressed < 0 || h.uncompressed < 0 || h.header_size < 2) return false;
    if (h.type == PQ_DATA_PAGE && !h.has_data) return false;
    if (h.type == PQ_DICTIONARY_PAGE && !h.has_dict) return false;
    return pos + h.header_size + static_cast<size_t>(h.compressed) <= end;
}

// Speculative page-chain segments of [start, end): the
// range is cut into nseg byte segments; segment 0 walks from the true start,
// segment k > 0 from the first position of its range where a plausible header
// begins a plausible three-page chain.  Each records the headers it meets
// until it leaves its range (or a parse fails).  The exact walk then follows
// the real chain and takes a recorded header only where the positions agree,
// so a false start costs time, never correctness.
struct SpecSeg {
    size_t lo = 0, hi = 0;
    std::vector<std::pair<size_t, PageHeader>> recs;
};

// Each thread interleaves kSpecLanes segments: one hop of every chain in
// turn, the next header's line prefetched as soon as its position is known,
// so a thread keeps several independent DRAM misses in flight (a single
// chain is one dependent miss per page).
constexpr int kSpecLanes = 16;
constexpr size_t kSpecScan = 16384;  // bytes a segment scans for its first header

std::vector<SpecSeg> speculate(const uint8_t* file, size_t len, size_t start, size_t end, int threads) {
    const int nseg = threads * kSpecLanes;
    std::vector<SpecSeg> segs(static_cast<size_t>(nseg));
    const size_t span = end - start;
    for (int k = 0; k < nseg; k++) {
        segs[k].lo = start + span * static_cast<size_t>(k) / static_cast<size_t>(nseg);
        segs[k].hi = start + span * static_cast<size_t>(k + 1) / static_cast<size_t>(nseg);
        segs[k].recs.reserve(64);
    }
    auto find_start = [&](int k) {
        const SpecSeg& sg = segs[static_cast<size_t>(k)];
        size_t pos = sg.lo;
        if (k == 0) return pos;
        // a segment inside one large page finds no start: give up after
        // kSpecScan bytes (the exact walk crosses it in one hop anyway)
        const size_t lim = std::min(sg.hi, sg.lo + kSpecScan);
        for (; pos < lim; pos++) {
            // a header opens with a short-form field header of an i32 or a
            // struct field (type 5 / 12); other bytes are not parsed (a
            // long-form opening only costs the exact walk, never a result)
            const uint8_t b0 = file[pos], ft = b0 & 0x0F;
            if ((b0 >> 4) == 0 || (ft != 5 && ft != 12)) continue;
            PageHeader h;
            if (!FastHdr(file, len, pos).parse(h) || !plausible(h, pos, end)) continue;
            size_t q = pos + h.header_size + static_cast<size_t>(h.compressed);
            bool ok = true;
            for (int hop = 0; hop < 2 && ok && q < end; hop++) {
                PageHeader h2;
                ok = FastHdr(file, len, q).parse(h2) && plausible(h2, q, end);
                if (ok) q += h2.header_size + static_cast<size_t>(h2.compressed);
            }
            if (ok) break;
        }
        return pos < lim ? pos : sg.hi;
    };
    auto work = [&](int t) {
        size_t pos[kSpecLanes];
        int live = 0;
        for (int l = 0; l < kSpecLanes; l++) {
            SpecSeg& sg = segs[static_cast<size_t>(t * kSpecLanes + l)];
            pos[l] = find_start(t * kSpecLanes + l);
            live += pos[l] < sg.hi;
            // room for the segment's records at its first page's size (no
            // regrowth copies when the pages are alike)
            PageHeader h;
            if (pos[l] < sg.hi && FastHdr(file, len, pos[l]).parse(h) && h.compressed >= 0) {
                const size_t est = (sg.hi - pos[l]) / std::max<size_t>(h.header_size + static_cast<size_t>(h.compressed), 16) + 16;
                sg.recs.reserve(est + est / 4);
            }
        }
        while (live > 0) {
            live = 0;
            for (int l = 0; l < kSpecLanes; l++) {
                SpecSeg& sg = segs[static_cast<size_t>(t * kSpecLanes + l)];
                if (pos[l] >= sg.hi) continue;
                PageHeader h;
                if (!FastHdr(file, len, pos[l]).parse(h) || h.compressed < 0) {
                    pos[l] = sg.hi;
                    continue;
                }
                sg.recs.emplace_back(pos[l], h);
                pos[l] += h.header_size + static_cast<size_t>(h.compressed);
                if (pos[l] < sg.hi) {
                    if (pos[l] + 64 < len) { __builtin_prefetch(file + pos[l]); __builtin_prefetch(file + pos[l] + 64); }
                    live++;
                }
            }
        }
    };
    parallel_run(threads, threads, work);
    return segs;
}

// The exact walk over linked speculative segments, on the same threads: when
// every segment the true chain enters starts its records exactly where the
// previous one's chain left, and no segment's chain broke inside its range,
// the segments' records ARE the chain from `start`.  The page table then
// follows from prefix sums (values, rows, the dictionary in force) instead of
// one serial pass.  Anything the serial loop would stop on (a header error
// before the value count, a chain that ends first, num_values <= 0) returns
// false: the caller runs the serial loop, which produces the reference's
// exact pages and error.
bool linked_walk(std::vector<SpecSeg>& segs, size_t start, const pq_chunk_desc& c, bool ext_v2, int32_t cflag,
                 int threads, WalkResult& w) {
    if (c.num_values <= 0) return false;
    std::vector<int> parts;     // segments on the chain, in order
    std::vector<size_t> first;  // the record of each where the true chain enters
    size_t expect = start;
    for (size_t k = 0; k < segs.size(); k++) {
        const SpecSeg& sg = segs[k];
        if (expect >= sg.hi) continue;  // the chain jumps over this segment
        // a segment that started on a false chain usually meets the true one
        // a few pages later: enter at the record where the positions agree
        const auto it = std::lower_bound(sg.recs.begin(), sg.recs.end(), expect,
                                         [](const std::pair<size_t, PageHeader>& r, size_t v) { return r.first < v; });
        if (it == sg.recs.end() || it->first != expect) return false;
        const auto& last = sg.recs.back();
        const size_t exit = last.first + last.second.header_size + static_cast<size_t>(last.second.compressed);
        if (exit < sg.hi) return false;  // the segment's chain broke inside it
        parts.push_back(static_cast<int>(k));
        first.push_back(static_cast<size_t>(it - sg.recs.begin()));
        expect = exit;
    }
    const size_t np = parts.size();
    if (np == 0) return false;
    // per part: data values, rows, records, first error, last dictionary page
    struct Sum { int64_t vals = 0, rows = 0; size_t n = 0, err = SIZE_MAX; int64_t last_dict = -1; };
    std::vector<Sum> sum(np);
    auto kind = [&](const PageHeader& h, int64_t* vals, bool* bad) {  // 0 other, 1 dict, 2 data, 3 v2
        *vals = 0;
        *bad = false;
        if (h.compressed < 0) { *bad = true; return 0; }
        if (h.type == PQ_DICTIONARY_PAGE) {
            *bad = !h.has_dict || h.dict_num_values < 0;
            return 1;
        }
        if (h.type == PQ_DATA_PAGE) {
            *bad = !h.has_data || h.data_num_values < 0;
            *vals = h.data_num_values;
            return 2;
        }
        if (h.type == PQ_DATA_PAGE_V2 && ext_v2) {
            *bad = !h.has_v2 || h.v2_num_values < 0 || h.v2_def_len < 0 || h.v2_rep_len < 0 ||
                   static_cast<int64_t>(h.v2_def_len) + h.v2_rep_len > h.compressed ||
                   static_cast<int64_t>(h.v2_def_len) + h.v2_rep_len > h.uncompressed;
            *vals = h.v2_num_values;
            return 3;
        }
        return 0;
    };
    auto par = [&](auto&& fn) {
        parallel_run(static_cast<int>(np), threads, [&](int i) { fn(static_cast<size_t>(i)); });
    };
    par([&](size_t i) {
        const auto& r = segs[static_cast<size_t>(parts[i])].recs;
        const size_t j0 = first[i];
        Sum& S = sum[i];
        S.n = r.size() - j0;
        for (size_t j = j0; j < r.size(); j++) {
            int64_t v;
            bool bad;
            const int kd = kind(r[j].second, &v, &bad);
            if (bad) { S.err = j - j0; break; }
            S.vals += v;
            S.rows += v;
            if (kd == 1) S.last_dict = static_cast<int64_t>(j - j0);
        }
    });
    // the cut: the page at which the values read reach num_values (serial
    // over parts, then within the one part)
    std::vector<size_t> base(np + 1, 0);
    std::vector<int64_t> vbase(np, 0), dict_in(np, -1);
    int64_t acc = 0, dict = -1;
    size_t cut_part = np, total = 0;
    for (size_t i = 0; i < np; i++) {
        base[i] = total;
        vbase[i] = acc;
        dict_in[i] = dict;
        if (sum[i].err != SIZE_MAX || acc + sum[i].vals >= c.num_values) { cut_part = i; break; }
        acc += sum[i].vals;
        if (sum[i].last_dict >= 0) dict = static_cast<int64_t>(total) + sum[i].last_dict;
        total += sum[i].n;
    }
    if (cut_part == np) return false;  // the chain ends before the value count
    size_t cut = 0;                    // records of cut_part kept
    {
        const auto& r = segs[static_cast<size_t>(parts[cut_part])].recs;
        int64_t a = acc;
        for (size_t j = first[cut_part]; j < r.size(); j++) {
            int64_t v;
            bool bad;
            kind(r[j].second, &v, &bad);
            if (bad) return false;  // an error before the count: the serial loop reports it
            a += v;
            if (a >= c.num_values) { cut = j + 1 - first[cut_part]; break; }
        }
        if (cut == 0) return false;
    }
    const size_t npages = base[cut_part] + cut;
    w.pages.resize(npages);
    par([&](size_t i) {
        if (i > cut_part) return;
        const auto& r = segs[static_cast<size_t>(parts[i])].recs;
        const size_t j0 = first[i];
        const size_t m = i == cut_part ? cut : r.size() - j0;
        int64_t row = vbase[i], d = dict_in[i];
        for (size_t j = 0; j < m; j++) {
            const size_t pos = r[j0 + j].first;
            const PageHeader& h = r[j0 + j].second;
            const size_t idx = base[i] + j;
            int64_t v;
            bool bad;
            const int kd = kind(h, &v, &bad);
            pq_page_desc p{};
            p.header_offset = static_cast<int64_t>(pos);
            p.payload_offset = static_cast<int64_t>(pos + h.header_size);
            p.payload_size = h.compressed;
            p.page_type = h.type;
            p.first_row = row;
            p.page_num = -1;
            p.uncompressed_size = h.uncompressed;
            if (kd == 1) {
                d = static_cast<int64_t>(idx);
                p.num_values = h.dict_num_values;
                p.page_num = static_cast<int32_t>(idx);
                p.flags = cflag;
            } else if (kd == 2) {
                p.num_values = h.data_num_values;
                p.encoding = h.data_encoding;
                p.page_num = static_cast<int32_t>(idx);
                p.flags = cflag;
            } else if (kd == 3) {
                p.page_type = PQ_DATA_PAGE;
                p.num_values = h.v2_num_values;
                p.encoding = h.v2_encoding;
                p.page_num = static_cast<int32_t>(idx);
                p.flags = PQ_PAGE_V2 | (h.v2_compressed ? cflag : 0);
                p.v2_def_len = h.v2_def_len;
                p.v2_rep_len = h.v2_rep_len;
            }
            p.dict_page = static_cast<int32_t>(d);
            row += v;
            w.pages[idx] = p;
        }
    });
    return true;
}

}  // namespace

namespace {
struct HostPool {
    const pid_t pid = getpid();  // the process whose threads these are
    std::mutex busy;  // one job at a time
    std::mutex m;
    std::condition_variable cv, done_cv;
    std::vector<std::thread> workers;
    const std::function<void(int)>* fn = nullptr;
    int n = 0, want = 0, finished = 0;
    uint64_t gen = 0;
    bool stop = false;
    std::atomic<int> next{0};
    void worker(int id) {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(int)>* f;
            {
                std::unique_lock<std::mutex> lk(m);
                cv.wait(lk, [&] { return stop || (gen != seen && id < want); });
                if (stop) return;
                seen = gen;
                f = fn;
            }
            for (int i = next.fetch_add(1); i < n; i = next.fetch_add(1)) (*f)(i);
            std::lock_guard<std::mutex> lk(m);
            if (++finished == want) done_cv.notify_one();
        }
    }
    ~HostPool() {
        {
            std::lock_guard<std::mutex> lk(m);
            stop = true;
        }
        cv.notify_all();
        for (auto& t : workers) t.join();
    }
};
// The pool belongs to the process that started its threads.  A child forked
// after that (bench.py's fork pools) inherits the pool's memory but none of
// its threads, and possibly a mutex some parent thread held at the fork: it
// must not touch that pool.  It builds its own; the inherited one is left
// alone (leaked), and only the owning process joins its threads at exit.
struct PoolHolder {
    std::atomic<HostPool*> pool{nullptr};
    ~PoolHolder() {
        HostPool* p = pool.load();
        if (p && p->pid == getpid()) delete p;
    }
};
PoolHolder g_pools;
HostPool& host_pool() {
    const pid_t me = getpid();
    HostPool* p = g_pools.pool.load(std::memory_order_acquire);
    while (!p || p->pid != me) {  // lock-free: no mutex a fork could have caught held
        HostPool* fresh = new HostPool;
        if (g_pools.pool.compare_exchange_strong(p, fresh, std::memory_order_acq_rel)) return *fresh;
        delete fresh;  // another thread of this process installed one first (p now holds it)
    }
    return *p;
}
}  // namespace

void parallel_run(int n, int threads, const std::function<void(int)>& fn) {
    if (n <= 0) return;
    threads = std::max(1, std::min(threads, n));
    if (threads == 1) {
        for (int i = 0; i < n; i++) fn(i);
        return;
    }
    HostPool& P = host_pool();
    std::unique_lock<std::mutex> job(P.busy, std::try_to_lock);
    if (!job.owns_lock()) {  // another host thread's job holds the pool
        std::atomic<int> next{0};
        std::vector<std::thread> th;
        for (int t = 1; t < threads; t++)
            th.emplace_back([&] { for (int i = next.fetch_add(1); i < n; i = next.fetch_add(1)) fn(i); });
        for (int i = next.fetch_add(1); i < n; i = next.fetch_add(1)) fn(i);
        for (auto& x : th) x.join();
        return;
    }
    {
        std::lock_guard<std::mutex> lk(P.m);
        while (static_cast<int>(P.workers.size()) < threads - 1) {
            const int id = static_cast<int>(P.workers.size());
            P.workers.emplace_back([&P, id] { P.worker(id); });
        }
        P.fn = &fn;
        P.n = n;
        P.want = threads - 1;
        P.finished = 0;
        P.next.store(0);
        P.gen++;
    }
    P.cv.notify_all();
    for (int i = P.next.fetch_add(1); i < n; i = P.next.fetch_add(1)) fn(i);
    std::unique_lock<std::mutex> lk(P.m);
    P.done_cv.wait(lk, [&] { return P.finished == P.want; });
    P.fn = nullptr;
}

WalkResult walk_chunk(const uint8_t* file, size_t len, const pq_chunk_desc& c, int threads) {
    WalkResult w;
    try {
        const bool ext_codecs = (c.ext_flags & PQ_EXT_CODECS) != 0, ext_v2 = (c.ext_flags & PQ_EXT_PAGE_V2) != 0;
        if (c.codec != 0 && !ext_codecs) throw Error(PQ_ERR_CODEC, "Only uncompressed parquet files are supported");
        if (c.codec != 0 && c.codec != 1 && c.codec != 2 && c.codec != 5 && c.codec != 6 && c.codec != 7)
            throw Error(PQ_ERR_CODEC, "Unsupported compression codec " + std::to_string(c.codec) +
                                          " (SNAPPY, GZIP, LZ4, ZSTD and LZ4_RAW are decoded)");
        const int32_t cflag = c.codec != 0 ? (PQ_PAGE_COMPRESSED | (c.codec << 8)) : 0;
        int64_t off = c.data_page_offset;
        if (c.has_dictionary_page_offset) off = std::min(off, c.dictionary_page_offset);
        size_t cur = static_cast<size_t>(off);
        int64_t values_read = 0, row = 0;
        int32_t page_num = 0, dict_page = -1;
        // speculative segments when the chunk's extent is known and large
        std::vector<SpecSeg> segs;
        w.pages.reserve(c.total_compressed_size > 0 ? static_cast<size_t>(std::min<int64_t>(c.total_compressed_size / 256, 1 << 22)) : 16);
        if (threads <= 0) threads = static_cast<int>(std::min(16u, std::max(1u, std::thread::hardware_concurrency())));
        threads = static_cast<int>(std::min<int64_t>(threads, c.total_compressed_size / (1 << 20)));
        // pages of tens of KiB or more: few enough for the exact walk alone
        // (probe the first headers; a segment would mostly scan page bytes)
        bool small_pages = true;
        if (c.total_compressed_size >= kSpecMinBytes && off >= 0 && static_cast<size_t>(off) < len) {
            size_t q = static_cast<size_t>(off);
            int k = 0;
            for (; k < 4 && q < len; k++) {
                PageHeader h;
                if (!FastHdr(file, len, q).parse(h) || h.compressed < 0) break;
                q += h.header_size + static_cast<size_t>(h.compressed);
            }
            small_pages = k == 0 || (q - static_cast<size_t>(off)) / static_cast<size_t>(k) < kSpecScan;
        }
        if (c.total_compressed_size >= kSpecMinBytes && threads > 1 && off >= 0 && small_pages &&
            static_cast<size_t>(off) < len) {
            const size_t end = std::min(len, static_cast<size_t>(off) + static_cast<size_t>(c.total_compressed_size));
            if (end > cur) segs = speculate(file, len, cur, end, threads);
            if (!segs.empty() && linked_walk(segs, cur, c, ext_v2, cflag, threads, w)) return w;
        }
        size_t sk = 0, si = 0;
        auto spec_at = [&](size_t pos, PageHeader& h) {
            while (sk < segs.size() && segs[sk].hi <= pos) { sk++; si = 0; }
            if (sk >= segs.size()) return false;
            auto& r = segs[sk].recs;
            while (si < r.size() && r[si].first < pos) si++;
            if (si < r.size() && r[si].first == pos) { h = r[si++].second; return true; }
            return false;
        };
        while (values_read < c.num_values) {  // column_reader.cpp:31-68
            PageHeader h;
            if (!spec_at(cur, h)) h = header_at(file, len, cur);
            pq_page_desc p{};
            p.header_offset = static_cast<int64_t>(cur);
            cur += h.header_size;
            p.payload_offset = static_cast<int64_t>(cur);
            p.payload_size = h.compressed;
            p.page_type = h.type;
            p.dict_page = dict_page;
            p.first_row = row;
            p.page_num = -1;
            p.uncompressed_size = h.uncompressed;
            if (h.compressed < 0)
                throw Error(PQ_ERR_ALLOC, "cannot create std::vector larger than max_size()");
            if (h.type == PQ_DICTIONARY_PAGE) {
                if (!h.has_dict) throw Error(PQ_ERR_OPTIONAL, "bad optional access");
                if (h.dict_num_values < 0) throw Error(PQ_ERR_ALLOC, "vector::reserve");
                p.num_values = h.dict_num_values;
                p.page_num = page_num++;
                p.flags = cflag;
                dict_page = static_cast<int32_t>(w.pages.size());
                p.dict_page = dict_page;
            } else if (h.type == PQ_DATA_PAGE) {
                if (!h.has_data) throw Error(PQ_ERR_OPTIONAL, "bad optional access");
                if (h.data_num_values < 0)
                    throw Error(PQ_ERR_ALLOC, "cannot create std::vector larger than max_size()");
                p.num_values = h.data_num_values;
                p.encoding = h.data_encoding;
                p.page_num = page_num++;
                p.flags = cflag;
                values_read += h.data_num_values;
                if (h.data_num_values > 0) row += h.data_num_values;
            } else if (h.type == PQ_DATA_PAGE_V2 && ext_v2) {
                // listed as a data page: the device rebuilds it in the V1 layout
                if (!h.has_v2) throw Error(PQ_ERR_OPTIONAL, "bad optional access");
                if (h.v2_num_values < 0 || h.v2_def_len < 0 || h.v2_rep_len < 0 ||
                    static_cast<int64_t>(h.v2_def_len) + h.v2_rep_len > h.compressed ||
                    static_cast<int64_t>(h.v2_def_len) + h.v2_rep_len > h.uncompressed)
                    throw Error(PQ_ERR_UNSUPPORTED, "DATA_PAGE_V2 header: level sections outside the page");
                p.page_type = PQ_DATA_PAGE;
                p.num_values = h.v2_num_values;
                p.encoding = h.v2_encoding;
                p.page_num = page_num++;
                p.flags = PQ_PAGE_V2 | (h.v2_compressed ? cflag : 0);
                p.v2_def_len = h.v2_def_len;
                p.v2_rep_len = h.v2_rep_len;
                values_read += h.v2_num_values;
                row += h.v2_num_values;
            } else {
                page_num++;  // read_pages counts skipped pages (column_reader.cpp:122)
            }
            w.pages.push_back(p);
            cur += static_cast<size_t>(h.compressed);
        }
    } catch (const Error& e) {
        w.error = e.code;
        w.message = e.what();
    }
    return w;
}

std::vector<std::array<int64_t, 4>> page_index(const uint8_t* file, size_t len, const FileMeta& fm) {
    std::vector<std::array<int64_t, 4>> out;  // parquet_reader.cpp:559-605
    for (size_t rg = 0; rg < fm.row_groups.size(); rg++) {
        const auto& r = fm.row_groups[rg];
        for (size_t col = 0; col < r.columns.size(); col++) {
            if (!r.columns[col].meta) continue;
            const ColumnMeta& m = *r.columns[col].meta;
            int64_t off = m.data_page_offset;
            if (m.dictionary_page_offset) off = std::min(off, *m.dictionary_page_offset);
            size_t cur = static_cast<size_t>(off);
            int64_t values_read = 0;
            while (values_read < m.num_values) {
                if (cur > len + 256)  // corrupt chunk: the reference would loop forever here
                    throw Error(PQ_ERR_UNSUPPORTED, "page walk ran past end of file");
                PageHeader h = header_at(file, len, cur);
                cur += h.header_size;
                // a negative size steps the reference's walk backwards (it never
                // ends); chunks a corrupt footer overlays could list the file's
                // bytes many times over: both are errors here
                if (h.compressed < 0) throw Error(PQ_ERR_UNSUPPORTED, "page walk: negative compressed_page_size");
                if (out.size() > len) throw Error(PQ_ERR_UNSUPPORTED, "page index: more pages than the file has bytes");
                if (h.type == PQ_DATA_PAGE || h.type == PQ_DATA_PAGE_V2) {
                    out.push_back({static_cast<int64_t>(cur), static_cast<int64_t>(static_cast<size_t>(h.compressed)),
                                   static_cast<int64_t>(rg), static_cast<int64_t>(col)});
                    if (h.type == PQ_DATA_PAGE && h.has_data) values_read += h.data_num_values;
                    // V2 values count too (the reference does not count them and walks
                    // past the chunk: outside its parity scope, SURVEY §8a R-WALK)
                    if (h.type == PQ_DATA_PAGE_V2 && h.has_v2) values_read += h.v2_num_values;
                }
                cur += static_cast<size_t>(h.compressed);
            }
        }
    }
    return out;
}

}  // namespace pqfmt
