/*
 * pq_oracle.c — TEST INFRASTRUCTURE ONLY (parity checker, never shipped).
 *
 * A plain-C restatement of the reference decode path of
 * sputnik89/duckdb-parquet-parser.  Each function cites the reference
 * file:line it follows (paths relative to the reference root).  Quirks are
 * reproduced on purpose: the fixed 256-byte header window, the zero-fill of
 * an exhausted hybrid stream, out-of-range dictionary indices -> NULL,
 * BOOLEAN dictionary entries as one byte, INT96 -> "INT96(hi:lo)" string.
 *
 * Cases the reference leaves undefined (SURVEY §8a "out of parity scope") are
 * given one deterministic meaning here and in the HIP path and are reported
 * as PQO_ERR_UNSUPPORTED where the reference would read freed/unowned memory:
 *   - a zero-count run (RLE count 0 or bit-packed group count 0) makes the
 *     reference fall into its literal branch with literal_count_ == 0, which
 *     wraps the counter (rle_decoder.hpp:26-31): every later value of that
 *     batch is read as consecutive bit fields from the literal cursor.  This
 *     is reproduced; it is UNSUPPORTED only when no literal run preceded it
 *     and bit width > 0 (the reference dereferences a NULL literal_pos_);
 *   - bit widths > 64 (rle_decoder.hpp:58-65 shifts past 63);
 *   - def levels above max_def on a dictionary page (column_reader.cpp:
 *     185-196 would index past the `indices` vector);
 *   - literal bits beyond the end of the page buffer read as zero.
 */
#include "pq_oracle.h"

#include <inttypes.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

enum { PT_BOOLEAN = 0, PT_INT32, PT_INT64, PT_INT96, PT_FLOAT, PT_DOUBLE,
       PT_BYTE_ARRAY, PT_FLBA };
enum { PG_DATA = 0, PG_INDEX = 1, PG_DICT = 2, PG_DATA_V2 = 3 };
enum { ENC_PLAIN_DICTIONARY = 2, ENC_RLE_DICTIONARY = 8 };
#define HEADER_READ_SIZE 256 /* column_reader.cpp:34 */

typedef struct {
    int code;
    char* msg;
    size_t msglen;
} err_t;

static int fail(err_t* e, int code, const char* fmt, ...) {
    if (e->code == 0) {
        e->code = code;
        if (e->msg && e->msglen) {
            va_list ap;
            va_start(ap, fmt);
            vsnprintf(e->msg, e->msglen, fmt, ap);
            va_end(ap);
        }
    }
    return code;
}

/* ── ByteBuffer (common.hpp:110-173) ─────────────────────────────────────── */
typedef struct {
    const uint8_t* data;
    size_t size, pos;
} bbuf;

/* common.hpp:162-168 — the exception text is part of the error contract. */
static int bb_check(bbuf* b, size_t n, err_t* e) {
    if (b->pos + n > b->size)
        return fail(e, PQO_ERR_BUFFER,
                    "ByteBuffer: read beyond end (pos=%zu need=%zu size=%zu)",
                    b->pos, n, b->size);
    return 0;
}
static int bb_byte(bbuf* b, uint8_t* v, err_t* e) {
    if (bb_check(b, 1, e)) return e->code;
    *v = b->data[b->pos++];
    return 0;
}
static int bb_bytes(bbuf* b, size_t n, const uint8_t** p, err_t* e) {
    if (bb_check(b, n, e)) return e->code;
    *p = b->data + b->pos;
    b->pos += n;
    return 0;
}
static int bb_u32(bbuf* b, uint32_t* v, err_t* e) {
    const uint8_t* p;
    if (bb_bytes(b, 4, &p, e)) return e->code;
    memcpy(v, p, 4);
    return 0;
}
/* common.hpp:136-147 */
static int bb_varint(bbuf* b, uint64_t* v, err_t* e) {
    uint64_t r = 0;
    int shift = 0;
    for (;;) {
        uint8_t x;
        if (bb_byte(b, &x, e)) return e->code;
        r |= (uint64_t)(x & 0x7F) << shift;
        if ((x & 0x80) == 0) break;
        shift += 7;
        if (shift > 63) return fail(e, PQO_ERR_THRIFT, "varint too long");
    }
    *v = r;
    return 0;
}
/* common.hpp:149-152 */
static int bb_zigzag(bbuf* b, int64_t* v, err_t* e) {
    uint64_t u;
    if (bb_varint(b, &u, e)) return e->code;
    *v = (int64_t)((u >> 1) ^ (~(u & 1) + 1));
    return 0;
}

/* ── Thrift compact reader (thrift.cpp:6-119) ────────────────────────────── */
typedef struct {
    bbuf b;
    int16_t last;
    int16_t stack[512];
    int depth;
} thrift_t;

static int th_push(thrift_t* t, err_t* e) { /* thrift.cpp:57-60 */
    if (t->depth >= 512) return fail(e, PQO_ERR_UNSUPPORTED, "thrift nesting too deep");
    t->stack[t->depth++] = t->last;
    t->last = 0;
    return 0;
}
static void th_pop(thrift_t* t) { t->last = t->stack[--t->depth]; } /* 62-65 */

/* thrift.cpp:6-21 */
static int th_field(thrift_t* t, int16_t* id, uint8_t* type, err_t* e) {
    uint8_t byte;
    if (bb_byte(&t->b, &byte, e)) return e->code;
    if (byte == 0) { *id = 0; *type = 0; return 0; }
    *type = byte & 0x0F;
    int16_t delta = (byte >> 4) & 0x0F;
    if (delta != 0) {
        *id = (int16_t)(t->last + delta);
    } else {
        int64_t z;
        if (bb_zigzag(&t->b, &z, e)) return e->code;
        *id = (int16_t)z;
    }
    t->last = *id;
    return 0;
}
static int th_i32(thrift_t* t, int32_t* v, err_t* e) { /* thrift.cpp:29 */
    int64_t z;
    if (bb_zigzag(&t->b, &z, e)) return e->code;
    *v = (int32_t)z;
    return 0;
}
/* thrift.cpp:44-55 */
static int th_list(thrift_t* t, uint8_t* et, int32_t* count, err_t* e) {
    uint8_t byte;
    if (bb_byte(&t->b, &byte, e)) return e->code;
    *et = byte & 0x0F;
    if (((byte >> 4) & 0x0F) == 0x0F) {
        uint64_t c;
        if (bb_varint(&t->b, &c, e)) return e->code;
        *count = (int32_t)c;
    } else {
        *count = (byte >> 4) & 0x0F;
    }
    return 0;
}
/* thrift.cpp:67-119 */
static int th_skip(thrift_t* t, uint8_t type, err_t* e) {
    uint64_t u;
    const uint8_t* p;
    switch (type) {
    case 1: case 2: return 0;
    case 3: { uint8_t x; return bb_byte(&t->b, &x, e); }
    case 4: case 5: case 6: return bb_varint(&t->b, &u, e);
    case 7: return bb_bytes(&t->b, 8, &p, e);
    case 8:
        if (bb_varint(&t->b, &u, e)) return e->code;
        return bb_bytes(&t->b, (uint32_t)u, &p, e);
    case 9: case 10: {
        uint8_t et; int32_t n;
        if (th_list(t, &et, &n, e)) return e->code;
        for (int32_t i = 0; i < n; i++)
            if (th_skip(t, et, e)) return e->code;
        return 0;
    }
    case 11: {
        if (bb_varint(&t->b, &u, e)) return e->code;
        int32_t n = (int32_t)u;
        if (n > 0) {
            uint8_t kv;
            if (bb_byte(&t->b, &kv, e)) return e->code;
            for (int32_t i = 0; i < n; i++) {
                if (th_skip(t, (kv >> 4) & 0x0F, e)) return e->code;
                if (th_skip(t, kv & 0x0F, e)) return e->code;
            }
        }
        return 0;
    }
    case 12: {
        if (th_push(t, e)) return e->code;
        for (;;) {
            int16_t id; uint8_t ft;
            if (th_field(t, &id, &ft, e)) return e->code;
            if (ft == 0) break;
            if (th_skip(t, ft, e)) return e->code;
        }
        th_pop(t);
        return 0;
    }
    default:
        return fail(e, PQO_ERR_THRIFT, "ThriftReader::skip: unknown type %d", (int)type);
    }
}

/* ── PageHeader (metadata.cpp:90-155) ────────────────────────────────────── */
typedef struct {
    int32_t type, uncompressed, compressed;
    int has_dph, has_dict;
    int32_t dph_num_values, dph_encoding;
    int32_t dict_num_values;
} page_header;

static int parse_dph(thrift_t* t, page_header* h, err_t* e) { /* 90-102 */
    int32_t v;
    h->dph_num_values = 0;
    h->dph_encoding = 0;
    for (;;) {
        int16_t id; uint8_t ft;
        if (th_field(t, &id, &ft, e)) return e->code;
        if (ft == 0) break;
        switch (id) {
        case 1: if (th_i32(t, &h->dph_num_values, e)) return e->code; break;
        case 2: if (th_i32(t, &h->dph_encoding, e)) return e->code; break;
        case 3: case 4: if (th_i32(t, &v, e)) return e->code; break;
        default: if (th_skip(t, ft, e)) return e->code;
        }
    }
    return 0;
}
static int parse_dict_hdr(thrift_t* t, page_header* h, err_t* e) { /* 106-117 */
    int32_t v;
    h->dict_num_values = 0;
    for (;;) {
        int16_t id; uint8_t ft;
        if (th_field(t, &id, &ft, e)) return e->code;
        if (ft == 0) break;
        switch (id) {
        case 1: if (th_i32(t, &h->dict_num_values, e)) return e->code; break;
        case 2: if (th_i32(t, &v, e)) return e->code; break;
        case 3: break; /* read_bool consumes nothing in compact protocol */
        default: if (th_skip(t, ft, e)) return e->code;
        }
    }
    return 0;
}
static int parse_page_header(thrift_t* t, page_header* h, err_t* e) { /* 121-155 */
    int32_t v;
    memset(h, 0, sizeof *h);
    for (;;) {
        int16_t id; uint8_t ft;
        if (th_field(t, &id, &ft, e)) return e->code;
        if (ft == 0) break;
        switch (id) {
        case 1: if (th_i32(t, &h->type, e)) return e->code; break;
        case 2: if (th_i32(t, &h->uncompressed, e)) return e->code; break;
        case 3: if (th_i32(t, &h->compressed, e)) return e->code; break;
        case 4: if (th_i32(t, &v, e)) return e->code; break;
        case 5:
            if (th_push(t, e) || parse_dph(t, h, e)) return e->code;
            th_pop(t);
            h->has_dph = 1;
            break;
        case 7:
            if (th_push(t, e) || parse_dict_hdr(t, h, e)) return e->code;
            th_pop(t);
            h->has_dict = 1;
            break;
        default: if (th_skip(t, ft, e)) return e->code;
        }
    }
    return 0;
}


/* ── RleDecoder (rle_decoder.hpp:6-108), state machine kept verbatim ─────── */
typedef struct {
    const uint8_t* data;
    uint32_t size, pos;   /* size_, pos_                                       */
    size_t phys;          /* bytes addressable from data (rest of page buffer) */
    uint32_t bw;          /* bit_width_                                        */
    uint32_t repeat;      /* repeat_count_                                     */
    uint32_t literal;     /* literal_count_ (wraps like the reference's u32)   */
    uint64_t value;       /* current_value_                                    */
    int lit_valid;        /* literal_pos_ != nullptr                           */
    uint32_t lit_start;   /* literal_pos_ - data_                              */
    uint32_t lit_bit;     /* literal_bit_offset_ (u32 like the reference)      */
} rle_t;

static void rle_init(rle_t* r, const uint8_t* d, uint32_t size, size_t phys, uint32_t bw) {
    memset(r, 0, sizeof *r);
    r->data = d;
    r->size = size;
    r->phys = phys;
    r->bw = bw;
}
static uint32_t rle_varint(rle_t* r) { /* rle_decoder.hpp:76-86 */
    uint32_t v = 0;
    int shift = 0;
    while (r->pos < r->size) {
        uint8_t b = r->data[r->pos++];
        if (shift < 32) v |= (uint32_t)(b & 0x7F) << shift;
        if ((b & 0x80) == 0) break;
        shift += 7;
    }
    return v;
}
static int rle_next(rle_t* r) { /* rle_decoder.hpp:37-53 */
    if (r->pos >= r->size) return 0;
    uint32_t ind = rle_varint(r);
    if (ind & 1) {
        r->literal = (ind >> 1) * 8;
        r->lit_start = r->pos;
        r->lit_valid = 1;
        r->lit_bit = 0;
    } else {
        r->repeat = ind >> 1;
        uint32_t nb = (r->bw + 7) / 8; /* read_fixed_width_value 88-95 */
        uint64_t v = 0;
        for (uint32_t i = 0; i < nb && r->pos < r->size; i++) {
            uint64_t byte = r->data[r->pos++];
            if (i < 8) v |= byte << (i * 8);
        }
        r->value = v;
    }
    return 1;
}
static uint64_t rle_literal(rle_t* r) { /* rle_decoder.hpp:55-74 */
    if (r->bw == 0) return 0;
    uint64_t v = 0;
    for (uint32_t i = 0; i < r->bw; i++) {
        uint32_t bit = r->lit_bit++;
        size_t at = (size_t)r->lit_start + (bit >> 3);
        uint8_t byte = at < r->phys ? r->data[at] : 0;
        if (byte & (1u << (bit & 7))) v |= (uint64_t)1 << i;
    }
    if (r->literal == 1) r->pos = r->lit_start + (r->lit_bit + 7) / 8;
    return v;
}
/* get_batch (rle_decoder.hpp:17-34).  Values stay u64; callers truncate
 * exactly like static_cast<int16_t>/<int32_t>. */
static int rle_batch(rle_t* r, uint64_t* out, uint32_t count, err_t* e) {
    for (uint32_t i = 0; i < count; i++) {
        if (r->repeat == 0 && r->literal == 0) {
            if (!rle_next(r)) {
                for (; i < count; i++) out[i] = 0;
                return 0;
            }
        }
        if (r->bw > 64) return fail(e, PQO_ERR_UNSUPPORTED, "bit width %u > 64", r->bw);
        if (r->repeat > 0) {
            out[i] = r->value;
            r->repeat--;
        } else {
            if (r->bw > 0 && !r->lit_valid)
                return fail(e, PQO_ERR_UNSUPPORTED, "zero-count run before any literal run");
            out[i] = rle_literal(r);
            r->literal--;
        }
    }
    return 0;
}

int pqo_rle_decode(const uint8_t* data, uint32_t size, uint32_t bit_width,
                   int32_t* out, uint32_t count) {
    char msg[128];
    err_t e = {0, msg, sizeof msg};
    rle_t r;
    uint64_t* tmp = (uint64_t*)malloc((count ? count : 1) * sizeof(uint64_t));
    if (!tmp) return PQO_ERR_ALLOC;
    rle_init(&r, data, size, size, bit_width);
    int rc = rle_batch(&r, tmp, count, &e);
    for (uint32_t i = 0; rc == 0 && i < count; i++) out[i] = (int32_t)(uint32_t)tmp[i];
    free(tmp);
    return rc;
}

/* ── growable output ─────────────────────────────────────────────────────── */
typedef struct {
    uint8_t* p;
    size_t n, cap;
} vbytes;
typedef struct {
    int64_t* p;
    size_t n, cap;
} vi64;

static int vb_reserve(vbytes* v, size_t add) {
    if (v->n + add <= v->cap) return 0;
    size_t c = v->cap ? v->cap : 256;
    while (c < v->n + add) c *= 2;
    uint8_t* q = (uint8_t*)realloc(v->p, c);
    if (!q) return -1;
    v->p = q;
    v->cap = c;
    return 0;
}
static int vb_put(vbytes* v, const void* src, size_t n) {
    if (vb_reserve(v, n)) return -1;
    if (n) memcpy(v->p + v->n, src, n);
    v->n += n;
    return 0;
}
static int vi_put(vi64* v, int64_t x) {
    if (v->n + 1 > v->cap) {
        size_t c = v->cap ? v->cap * 2 : 256;
        int64_t* q = (int64_t*)realloc(v->p, c * sizeof(int64_t));
        if (!q) return -1;
        v->p = q;
        v->cap = c;
    }
    v->p[v->n++] = x;
    return 0;
}

/* Columnar builder: one row = (valid, bytes). */
typedef struct {
    vbytes valid, data;
    vi64 offsets; /* start offset of each row; the final end is data.n */
} colbuf;

static int col_null(colbuf* c, err_t* e) {
    uint8_t z = 0;
    if (vb_put(&c->valid, &z, 1) || vi_put(&c->offsets, (int64_t)c->data.n))
        return fail(e, PQO_ERR_ALLOC, "out of memory");
    return 0;
}
static int col_value(colbuf* c, const void* p, size_t n, err_t* e) {
    uint8_t one = 1;
    if (vb_put(&c->valid, &one, 1) || vi_put(&c->offsets, (int64_t)c->data.n) ||
        vb_put(&c->data, p, n))
        return fail(e, PQO_ERR_ALLOC, "out of memory");
    return 0;
}
static void col_release(colbuf* c) {
    free(c->valid.p);
    free(c->data.p);
    free(c->offsets.p);
    memset(c, 0, sizeof *c);
}

/* ── read_plain_value (column_reader.cpp:227-268) ────────────────────────── */
static int read_plain_value(int32_t type, bbuf* b, colbuf* out, err_t* e) {
    const uint8_t* p;
    switch (type) {
    case PT_BOOLEAN: { /* 229-232: a dictionary BOOLEAN entry is one byte */
        uint8_t x;
        if (bb_byte(b, &x, e)) return e->code;
        uint8_t v = x != 0;
        return col_value(out, &v, 1, e);
    }
    case PT_INT32: case PT_FLOAT: /* 233-236, 241-244 */
        if (bb_bytes(b, 4, &p, e)) return e->code;
        return col_value(out, p, 4, e);
    case PT_INT64: case PT_DOUBLE: /* 237-240, 245-248 */
        if (bb_bytes(b, 8, &p, e)) return e->code;
        return col_value(out, p, 8, e);
    case PT_BYTE_ARRAY: { /* 249-253: u32 length prefix + bytes */
        uint32_t len;
        if (bb_u32(b, &len, e) || bb_bytes(b, len, &p, e)) return e->code;
        return col_value(out, p, len, e);
    }
    case PT_FLBA: /* 254-256 */
        return fail(e, PQO_ERR_FLBA, "FIXED_LEN_BYTE_ARRAY not supported without type_length");
    case PT_INT96: { /* 257-264: "INT96(" + to_string(high) + ":" + to_string(low) + ")" */
        int64_t lo;
        int32_t hi;
        char s[64];
        if (bb_bytes(b, 12, &p, e)) return e->code;
        memcpy(&lo, p, 8);
        memcpy(&hi, p + 8, 4);
        int n = snprintf(s, sizeof s, "INT96(%" PRId32 ":%" PRId64 ")", hi, lo);
        return col_value(out, s, (size_t)n, e);
    }
    default: /* 265-266 */
        return fail(e, PQO_ERR_TYPE, "Unsupported type: %d", (int)type);
    }
}

/* ColumnReader::bit_width (column_reader.cpp:270-276) */
static uint32_t level_bit_width(int16_t max_level) {
    uint32_t bw = 0;
    int32_t v = max_level;
    if (v <= 0) return 0;
    while (v > 0) { bw++; v >>= 1; }
    return bw;
}

/* ── read_data_page (column_reader.cpp:140-225) ──────────────────────────── */
static int read_data_page(const pqo_chunk* c, const uint8_t* data, size_t size,
                          int32_t num_values, int32_t encoding,
                          const colbuf* dict, int64_t dict_n, colbuf* out, err_t* e) {
    bbuf buf = {data, size, 0};
    int rc = 0;
    if (num_values < 0) /* std::vector<int16_t>(num_values) with a negative count */
        return fail(e, PQO_ERR_ALLOC, "cannot create std::vector larger than max_size()");
    int16_t* def = (int16_t*)malloc(((size_t)num_values + 1) * sizeof(int16_t));
    uint64_t* tmp = (uint64_t*)malloc(((size_t)num_values + 1) * sizeof(uint64_t));
    if (!def || !tmp) { rc = fail(e, PQO_ERR_ALLOC, "out of memory"); goto done; }
    for (int32_t i = 0; i < num_values; i++) def[i] = c->max_def_level;

    if (c->max_def_level > 0) { /* 146-154 */
        uint32_t def_len;
        rle_t r;
        if (bb_u32(&buf, &def_len, e)) { rc = e->code; goto done; }
        if (bb_check(&buf, def_len, e)) { rc = e->code; goto done; } /* read_bytes(def_len) */
        rle_init(&r, data + buf.pos, def_len, size - buf.pos, level_bit_width(c->max_def_level));
        if (rle_batch(&r, tmp, (uint32_t)num_values, e)) { rc = e->code; goto done; }
        for (int32_t i = 0; i < num_values; i++) def[i] = (int16_t)(uint16_t)tmp[i];
        buf.pos += def_len;
    }
    if (c->max_rep_level > 0) { /* 156-164: decoded then unused for flat output */
        uint32_t rep_len;
        if (bb_u32(&buf, &rep_len, e) || bb_check(&buf, rep_len, e)) { rc = e->code; goto done; }
        buf.pos += rep_len;
    }
    int32_t num_non_null = 0; /* 166-170 */
    int any_above = 0;
    for (int32_t i = 0; i < num_values; i++) {
        if (def[i] == c->max_def_level) num_non_null++;
        if (def[i] > c->max_def_level) any_above = 1;
    }

    int use_dict = encoding == ENC_PLAIN_DICTIONARY || encoding == ENC_RLE_DICTIONARY;
    if (use_dict && dict) { /* 174-196 */
        uint8_t bw;
        rle_t r;
        if (bb_byte(&buf, &bw, e)) { rc = e->code; goto done; }
        if (any_above) {
            rc = fail(e, PQO_ERR_UNSUPPORTED, "definition level above max on a dictionary page");
            goto done;
        }
        rle_init(&r, data + buf.pos, (uint32_t)(size - buf.pos), size - buf.pos, bw);
        if (rle_batch(&r, tmp, (uint32_t)num_non_null, e)) { rc = e->code; goto done; }
        int32_t k = 0;
        for (int32_t i = 0; i < num_values; i++) {
            if (def[i] < c->max_def_level) {
                if (col_null(out, e)) { rc = e->code; goto done; }
            } else {
                int32_t idx = (int32_t)(uint32_t)tmp[k++];
                if (idx >= 0 && idx < dict_n) {
                    int64_t s = dict->offsets.p[idx];
                    int64_t t = idx + 1 < dict_n ? dict->offsets.p[idx + 1] : (int64_t)dict->data.n;
                    if (col_value(out, dict->data.p + s, (size_t)(t - s), e)) { rc = e->code; goto done; }
                } else if (col_null(out, e)) { rc = e->code; goto done; }
            }
        }
    } else if (c->type == PT_BOOLEAN) { /* 197-212 */
        int32_t bit = 0;
        uint8_t cur = 0;
        for (int32_t i = 0; i < num_values; i++) {
            if (def[i] < c->max_def_level) {
                if (col_null(out, e)) { rc = e->code; goto done; }
            } else {
                if (bit % 8 == 0 && bb_byte(&buf, &cur, e)) { rc = e->code; goto done; }
                uint8_t v = (cur >> (bit % 8)) & 1;
                if (col_value(out, &v, 1, e)) { rc = e->code; goto done; }
                bit++;
            }
        }
    } else { /* 213-222 */
        for (int32_t i = 0; i < num_values; i++) {
            if (def[i] < c->max_def_level) {
                if (col_null(out, e)) { rc = e->code; goto done; }
            } else if (read_plain_value(c->type, &buf, out, e)) { rc = e->code; goto done; }
        }
    }
done:
    free(def);
    free(tmp);
    return rc;
}

/* In-memory ReadRangeFunc that zero-pads past EOF. */
static uint8_t* read_range(const uint8_t* file, size_t flen, size_t off, size_t n) {
    uint8_t* b = (uint8_t*)calloc(n ? n : 1, 1);
    if (!b) return NULL;
    if (off < flen) memcpy(b, file + off, (flen - off) < n ? (flen - off) : n);
    return b;
}

/* ── ColumnReader::read_all / read_pages (column_reader.cpp:3-126) ───────── */
int pqo_read_all(const uint8_t* file, size_t flen, const pqo_chunk* c,
                 pqo_column* out, char* msg, size_t msglen) {
    err_t e = {0, msg, msglen};
    if (msg && msglen) msg[0] = 0;
    memset(out, 0, sizeof *out);
    out->type = c->type;
    if (c->codec != 0) /* 13-15 */
        return fail(&e, PQO_ERR_CODEC, "Only uncompressed parquet files are supported");

    colbuf col, dict;
    memset(&col, 0, sizeof col);
    memset(&dict, 0, sizeof dict);
    int has_dict = 0;
    int64_t dict_n = 0;
    pqo_page* pages = NULL;
    int32_t npages = 0, pcap = 0, page_num = 0;

    int64_t offset = c->data_page_offset; /* 21-25 */
    if (c->has_dictionary_page_offset && c->dictionary_page_offset < offset)
        offset = c->dictionary_page_offset;
    size_t cur = (size_t)offset;
    int64_t values_read = 0;

    while (values_read < c->num_values) { /* 31 */
        uint8_t* hb = read_range(file, flen, cur, HEADER_READ_SIZE); /* 34-38 */
        thrift_t t;
        page_header h;
        if (!hb) { fail(&e, PQO_ERR_ALLOC, "out of memory"); break; }
        memset(&t, 0, sizeof t);
        t.b.data = hb;
        t.b.size = HEADER_READ_SIZE;
        int prc = parse_page_header(&t, &h, &e);
        free(hb);
        if (prc) break;
        cur += t.b.pos;
        int32_t psize = h.compressed;
        if (psize < 0) {
            fail(&e, PQO_ERR_ALLOC, "cannot create std::vector larger than max_size()");
            break;
        }
        if (h.type == PG_DICT || h.type == PG_DATA) {
            if ((h.type == PG_DICT && !h.has_dict) || (h.type == PG_DATA && !h.has_dph)) {
                fail(&e, PQO_ERR_OPTIONAL, "bad optional access");
                break;
            }
            uint8_t* pb = read_range(file, flen, cur, (size_t)psize);
            if (!pb) { fail(&e, PQO_ERR_ALLOC, "out of memory"); break; }
            int rc = 0;
            int64_t first_row = (int64_t)col.valid.n;
            if (h.type == PG_DICT) { /* 128-138 */
                if (h.dict_num_values < 0) {
                    rc = fail(&e, PQO_ERR_ALLOC, "vector::reserve");
                } else {
                    bbuf b = {pb, (size_t)psize, 0};
                    col_release(&dict);
                    dict_n = 0;
                    for (int32_t i = 0; i < h.dict_num_values && rc == 0; i++) {
                        rc = read_plain_value(c->type, &b, &dict, &e);
                        if (rc == 0) dict_n++;
                    }
                    has_dict = 1;
                }
            } else {
                rc = read_data_page(c, pb, (size_t)psize, h.dph_num_values, h.dph_encoding,
                                    has_dict ? &dict : NULL, dict_n, &col, &e);
            }
            free(pb);
            if (rc) break;
            if (npages == pcap) {
                pcap = pcap ? pcap * 2 : 64;
                pqo_page* q = (pqo_page*)realloc(pages, (size_t)pcap * sizeof *pages);
                if (!q) { fail(&e, PQO_ERR_ALLOC, "out of memory"); break; }
                pages = q;
            }
            pqo_page* pg = &pages[npages++];
            pg->page_num = page_num++;
            pg->page_type = h.type;
            if (h.type == PG_DICT) {
                pg->num_values = h.dict_num_values;
                pg->first_row = first_row;
                pg->nrows = 0;
            } else {
                pg->num_values = h.dph_num_values;
                pg->first_row = first_row;
                pg->nrows = (int64_t)col.valid.n - first_row;
                values_read += h.dph_num_values;
            }
            cur += (size_t)psize;
            continue;
        }
        cur += (size_t)psize; /* unknown page types are skipped (64-67) */
        page_num++;
    }
    col_release(&dict);
    if (e.code) {
        col_release(&col);
        free(pages);
        return e.code;
    }
    out->nrows = (int64_t)col.valid.n;
    out->valid = col.valid.p ? col.valid.p : (uint8_t*)calloc(1, 1);
    out->data = col.data.p ? col.data.p : (uint8_t*)calloc(1, 1);
    out->data_len = (int64_t)col.data.n;
    if (vi_put(&col.offsets, (int64_t)col.data.n)) return fail(&e, PQO_ERR_ALLOC, "out of memory");
    out->offsets = col.offsets.p;
    out->pages = pages;
    out->npages = npages;
    return 0;
}

void pqo_free(pqo_column* col) {
    if (!col) return;
    free(col->valid);
    free(col->offsets);
    free(col->data);
    free(col->pages);
    memset(col, 0, sizeof *col);
}

int pqo_dump(const pqo_column* col, uint8_t** out, size_t* out_len) {
    int var = col->type == PT_BYTE_ARRAY || col->type == PT_INT96;
    size_t n = (size_t)col->nrows + (size_t)col->data_len + (var ? 4 * (size_t)col->nrows : 0);
    uint8_t* d = (uint8_t*)malloc(n ? n : 1);
    if (!d) return PQO_ERR_ALLOC;
    size_t w = 0;
    for (int64_t i = 0; i < col->nrows; i++) {
        d[w++] = col->valid[i] ? 0 : 1;
        if (!col->valid[i]) continue;
        uint32_t len = (uint32_t)(col->offsets[i + 1] - col->offsets[i]);
        if (var) { memcpy(d + w, &len, 4); w += 4; }
        memcpy(d + w, col->data + col->offsets[i], len);
        w += len;
    }
    *out = d;
    *out_len = w;
    return 0;
}

void pqo_free_buf(void* p) { free(p); }

/* src/main.cpp:17-32: `if (chunk.size() >= chunk_size) { clear; chunk_id++; }`
 * before each non-NULL string, then `chunk += to_string(len) + string` and
 * tuple_to_chunk[pos] = chunk_id.  Only the chunk's size matters here. */
void pqo_chunk_assign(const uint8_t* valid, const int64_t* offsets, int64_t nrows,
                      int64_t chunk_size, int64_t* out, int64_t* num_chunks) {
    int64_t size = 0, chunk_id = 0;
    for (int64_t r = 0; r < nrows; r++) {
        out[r] = 0;  /* std::vector<size_t> tuple_to_chunk(num_rows) */
        if (!valid[r]) continue;
        if (size >= chunk_size) {
            size = 0;
            chunk_id++;
        }
        uint64_t len = (uint64_t)(offsets[r + 1] - offsets[r]), d = 1;
        for (uint64_t v = len; v >= 10; v /= 10) d++;
        size += (int64_t)(d + len);
        out[r] = chunk_id;
    }
    *num_chunks = chunk_id + 1;
}
