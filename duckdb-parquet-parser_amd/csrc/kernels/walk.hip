// walk.hip — the chunk's page walk on the GPU over bytes already in HBM
// (the device page table; the host form is
// csrc/host/format.cpp walk_chunk, whose page list this reproduces).
//
// The reference walks a column chunk's page chain serially: read the Thrift
// PageHeader at the cursor, step over header and payload, until the data
// pages' values reach ColumnMetaData.num_values
// (src/reader/column_reader.cpp:18-71, src/reader/metadata.cpp:121-155).
// Here the extent is cut into segments of `seg` bytes, one wave each:
//   k_walk_seg    segment 0 starts at the chunk's first page; segment k > 0
//                 at the first position of its range where a plausible header
//                 begins a plausible three-page chain (format.cpp speculate's
//                 rule); each lane records the headers its chain meets until
//                 it leaves the segment (a 256-byte window per hop in LDS,
//                 parsed with the host parser's exact acceptance rules);
//   k_walk_link   segment k is entered where segment k - 1's chain left: the
//                 record at that position (a false start converges or the
//                 walk is refused), its chain records, data values and last
//                 dictionary page;
//   k_walk_scan   one workgroup: page and value prefixes over the segments,
//                 the dictionary in force, the page where the values reach
//                 num_values (the cut), every segment up to it linked;
//   k_walk_emit   the pq_page_desc of every page up to the cut.
// Anything the speculative chain cannot settle exactly (a page longer than a
// segment, a header the parse refuses, an invalid header before the cut, a
// chain that ends first, a segment over its record capacity) returns
// "refused": the caller walks on the host, which also reports the
// reference's errors.  Uncompressed V1 scope only (no PQ_EXT_* flags).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels/kernels.hpp"

namespace pqk {
namespace {

constexpr uint32_t kWin = 256;          // header window (read_page_header's fixed window)
constexpr uint32_t kWinStride = 65;     // dwords per window: 256 bytes from any byte of the first dword
constexpr uint32_t kScanLimit = 16384;  // bytes a segment scans for its first header (format.cpp kSpecScan)
constexpr int kSkipDepth = 8;

// LDS pointers typed as such: a generic pointer compiles to flat loads, which
// wait on both counters and take the longer path
using lds8c = const __attribute__((address_space(3))) uint8_t;
using lds32 = __attribute__((address_space(3))) uint32_t;

struct DHdr {
    int32_t type, uncomp, comp, dnv, denc, dictnv;
    uint32_t hs;
    uint32_t flags;  // 1 has_data, 2 has_dict, 4 has_v2
};

// One lane's 256-byte window: bytes [0, avail) valid (zeros past the buffer).
struct Win {
    lds8c* w;
    uint32_t p, e;
    __device__ __forceinline__ bool byte(uint32_t& v) {
        if (p >= e) return false;
        v = w[p++];
        return true;
    }
    __device__ __forceinline__ bool varint(uint64_t& r) {
        r = 0;
        for (int shift = 0;; shift += 7) {
            if (shift > 63) return false;
            uint32_t b;
            if (!byte(b)) return false;
            r |= static_cast<uint64_t>(b & 0x7Fu) << shift;
            if ((b & 0x80u) == 0) return true;
        }
    }
    __device__ __forceinline__ bool i32(int32_t& v) {
        uint64_t u;
        if (!varint(u)) return false;
        v = static_cast<int32_t>(static_cast<int64_t>((u >> 1) ^ (~(u & 1) + 1)));
        return true;
    }
    // id = 0, type = 0 at STOP (a type nibble 0 ends the struct too: format.cpp FastHdr::field).
    // Results by value: out-parameters of the callers' loop locals were kept
    // in scratch (a global store and load per field, ~8 us per header hop)
    struct Fld {
        int32_t id, last;
        uint32_t type;
        bool ok;
    };
    __device__ __forceinline__ Fld field(int32_t last) {
        Fld f{0, last, 0u, false};
        uint32_t b;
        if (!byte(b)) return f;
        f.ok = true;
        if (b == 0) return f;
        f.type = b & 0x0Fu;
        const int32_t delta = static_cast<int32_t>((b >> 4) & 0x0Fu);
        if (delta) {
            f.id = static_cast<int16_t>(last + delta);
        } else {
            uint64_t u;
            if (!varint(u)) { f.ok = false; return f; }
            f.id = static_cast<int16_t>(static_cast<int64_t>((u >> 1) ^ (~(u & 1) + 1)));
        }
        f.last = f.id;
        if (f.type == 0) f.id = 0;
        return f;
    }
    __device__ bool bytes(uint64_t n) {
        if (n > static_cast<uint64_t>(e - p)) return false;
        p += static_cast<uint32_t>(n);
        return true;
    }
    // Thrift skip of a value of `type` (skip_value below: out of line, by value,
    // so this cursor stays in registers on the paths that never skip)
    __device__ __forceinline__ bool skip(uint32_t type);
    // iterative (format.cpp FastHdr::skip; nesting past kSkipDepth refuses,
    // which the walk treats as a parse failure); its frame arrays live in scratch
    __device__ __forceinline__ bool skip_impl(uint32_t type) {
        // frame: kind 0 struct (last id), 1 list (remaining, elem type), 2 map (remaining pairs, kt, vt, half)
        uint32_t kind[kSkipDepth], et[kSkipDepth], et2[kSkipDepth];
        int64_t rem[kSkipDepth];
        int32_t lastid[kSkipDepth];
        int sp = 0;
        uint32_t t = type;
        for (;;) {
            // a scalar or a container header for type t
            bool pushed = false;
            uint64_t u;
            switch (t) {
                case 1: case 2: break;
                case 3: { uint32_t b; if (!byte(b)) return false; break; }
                case 4: case 5: case 6: if (!varint(u)) return false; break;
                case 7: if (!bytes(8)) return false; break;
                case 8: if (!varint(u) || !bytes(static_cast<uint32_t>(u))) return false; break;
                case 9: case 10: {
                    uint32_t b;
                    if (!byte(b)) return false;
                    const uint32_t e1 = b & 0x0Fu;
                    int64_t n = static_cast<int64_t>((b >> 4) & 0x0Fu);
                    if (n == 0x0F) { if (!varint(u)) return false; n = static_cast<int32_t>(u); }
                    if (e1 == 1 || e1 == 2 || n <= 0) break;  // bool elements take no bytes
                    if (sp == kSkipDepth) return false;
                    kind[sp] = 1; et[sp] = e1; rem[sp] = n; sp++;
                    pushed = true;
                    break;
                }
                case 11: {
                    if (!varint(u)) return false;
                    const int32_t n = static_cast<int32_t>(u);
                    if (n <= 0) break;
                    uint32_t kv;
                    if (!byte(kv)) return false;
                    const uint32_t kt = (kv >> 4) & 0x0Fu, vt = kv & 0x0Fu;
                    if ((kt == 1 || kt == 2) && (vt == 1 || vt == 2)) break;
                    if (sp == kSkipDepth) return false;
                    kind[sp] = 2; et[sp] = kt; et2[sp] = vt; rem[sp] = 2 * static_cast<int64_t>(n); sp++;
                    pushed = true;
                    break;
                }
                case 12:
                    if (sp == kSkipDepth) return false;
                    kind[sp] = 0; lastid[sp] = 0; sp++;
                    pushed = true;
                    break;
                default: return false;
            }
            (void)pushed;
            // the next value to skip: from the innermost open container
            for (;;) {
                if (sp == 0) return true;
                const int f = sp - 1;
                if (kind[f] == 0) {
                    const Fld fd = field(lastid[f]);
                    if (!fd.ok) return false;
                    lastid[f] = fd.last;
                    if (fd.type == 0 && fd.id == 0) { sp--; continue; }
                    t = fd.type;
                    break;
                }
                if (rem[f] == 0) { sp--; continue; }
                rem[f]--;
                t = kind[f] == 1 ? et[f] : ((rem[f] & 1) ? et[f] : et2[f]);  // map: key then value
                break;
            }
        }
    }
};

__device__ __noinline__ uint32_t skip_value(lds8c* w, uint32_t p, uint32_t e, uint32_t type) {
    Win c{w, p, e};
    return c.skip_impl(type) ? c.p : 0xFFFFFFFFu;
}
__device__ __forceinline__ bool Win::skip(uint32_t type) {
    const uint32_t np = skip_value(w, p, e, type);
    if (np == 0xFFFFFFFFu) return false;
    p = np;
    return true;
}

// format.cpp FastHdr::parse: true for every header read_page_header accepts
// (identical fields), false where it would throw.
__device__ __forceinline__ bool dev_parse(lds8c* w, uint32_t avail, DHdr& h) {
    Win c{w, 0, avail};
    h = DHdr{0, 0, 0, 0, 0, 0, 0, 0};
    int32_t last = 0;
    for (;;) {
        const Win::Fld fd = c.field(last);
        if (!fd.ok) return false;
        last = fd.last;
        const int32_t id = fd.id;
        const uint32_t ty = fd.type;
        if (ty == 0 && id == 0) break;
        switch (id) {
            case 1: if (!c.i32(h.type)) return false; break;
            case 2: if (!c.i32(h.uncomp)) return false; break;
            case 3: if (!c.i32(h.comp)) return false; break;
            case 4: { int32_t x; if (!c.i32(x)) return false; break; }
            case 5: {
                h.flags |= 1u;
                h.dnv = 0;
                h.denc = 0;
                int32_t l2 = 0;
                for (;;) {
                    const Win::Fld f2 = c.field(l2);
                    if (!f2.ok) return false;
                    l2 = f2.last;
                    const int32_t i2 = f2.id;
                    const uint32_t t2 = f2.type;
                    if (t2 == 0 && i2 == 0) break;
                    int32_t x;
                    if (i2 == 1) { if (!c.i32(h.dnv)) return false; }
                    else if (i2 == 2) { if (!c.i32(h.denc)) return false; }
                    else if (i2 == 3 || i2 == 4) { if (!c.i32(x)) return false; }
                    else if (!c.skip(t2)) return false;
                }
                break;
            }
            case 8: {  // DataPageHeaderV2 (skipped by the reference: only its bytes)
                if (ty != 12) {
                    if (!c.skip(ty)) return false;
                    break;
                }
                h.flags |= 4u;
                int32_t l2 = 0;
                for (;;) {
                    const Win::Fld f2 = c.field(l2);
                    if (!f2.ok) return false;
                    l2 = f2.last;
                    const int32_t i2 = f2.id;
                    const uint32_t t2 = f2.type;
                    if (t2 == 0 && i2 == 0) break;
                    int32_t x;
                    if (t2 == 5 && (i2 == 1 || i2 == 4 || i2 == 5 || i2 == 6)) { if (!c.i32(x)) return false; }
                    else if ((t2 == 1 || t2 == 2) && i2 == 7) { /* bool: no bytes */ }
                    else if (!c.skip(t2)) return false;
                }
                break;
            }
            case 7: {
                h.flags |= 2u;
                h.dictnv = 0;
                int32_t l2 = 0;
                for (;;) {
                    const Win::Fld f2 = c.field(l2);
                    if (!f2.ok) return false;
                    l2 = f2.last;
                    const int32_t i2 = f2.id;
                    const uint32_t t2 = f2.type;
                    if (t2 == 0 && i2 == 0) break;
                    int32_t x;
                    if (i2 == 1) { if (!c.i32(h.dictnv)) return false; }
                    else if (i2 == 2) { if (!c.i32(x)) return false; }
                    else if (i2 == 3) { /* read_bool: no bytes */ }
                    else if (!c.skip(t2)) return false;
                }
                break;
            }
            default: if (!c.skip(ty)) return false;
        }
    }
    h.hs = c.p;
    return true;
}

// format.cpp plausible()
__device__ __forceinline__ bool dev_plausible(const DHdr& h, uint64_t pos, uint64_t end) {
    if (h.type < 0 || h.type > 3 || h.comp < 0 || h.uncomp < 0 || h.hs < 2) return false;
    if (h.type == PQ_DATA_PAGE && !(h.flags & 1u)) return false;
    if (h.type == PQ_DICTIONARY_PAGE && !(h.flags & 2u)) return false;
    return pos + h.hs + static_cast<uint64_t>(h.comp) <= end;
}

// The window at file offset pos, loaded by the whole wave (one dword per lane,
// lane 0 also the 65th): 260 bytes from the dword-aligned offset at or below
// pos (zeros past the device buffer [base, base + len)); returns pos's offset
// in it (0 .. 3), so 256 bytes from pos are in the window.
__device__ __forceinline__ uint32_t load_win(lds32* win, const uint8_t* __restrict__ d, uint64_t base, uint64_t len,
                                                 uint64_t pos) {
    const uint64_t rel = pos - base, a0 = rel & ~3ull;
    const uint32_t l = __lane_id();
    auto dword = [&](uint32_t i) -> uint32_t {
        const uint64_t q = a0 + 4ull * i;
        if (q + 4 <= len) return *reinterpret_cast<const uint32_t*>(d + q);  // (the buffer is 16-byte aligned)
        uint32_t w = 0;
        for (uint32_t b = 0; b < 4; b++) w |= static_cast<uint32_t>(q + b < len ? d[q + b] : 0u) << (8 * b);
        return w;
    };
    const uint32_t v = dword(l);
    const uint32_t v2 = l == 0 ? dword(kWinStride - 1) : 0u;
    __builtin_amdgcn_wave_barrier();  // every lane is done parsing the previous window
    win[l] = v;
    if (l == 0) win[kWinStride - 1] = v2;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    return static_cast<uint32_t>(rel & 3u);
}

struct WalkSeg {
    uint64_t exit;      // where the segment's chain left it (or stopped)
    uint32_t n;         // records
    uint32_t flags;     // 1: overflow, 2: the chain broke inside (parse failure / negative size)
};

// One wave per segment.  Every lane parses the same header from the shared
// window (the parse is serial; identical work keeps the lanes in step), and
// the 64 lanes test 64 positions at once for a header opening while the
// segment looks for its first chain start.
__global__ void __launch_bounds__(kWave) k_walk_seg(const uint8_t* __restrict__ d, uint64_t base, uint64_t len,
                                                    uint64_t start, uint64_t end, uint64_t seg, uint32_t nseg,
                                                    uint32_t cap, WalkRec* __restrict__ recs,
                                                    WalkSeg* __restrict__ segs, uint32_t stage_cap) {
    __shared__ uint32_t win_s[kWinStride + 3];
    extern __shared__ __attribute__((aligned(16))) uint32_t seg_dyn[];
    lds32* win = (lds32*)win_s;
    const uint32_t k = blockIdx.x;
    if (k >= nseg) return;
    const uint32_t l = __lane_id();
    lds8c* wb = (lds8c*)win_s;
    const uint64_t lo = start + seg * k, hi = min(end, lo + seg);
    // The segment and one header window past it, staged in LDS once (16-byte
    // loads, zeros past the buffer): every hop inside it parses from LDS
    // instead of waiting for a 260-byte load from HBM per header (a hop was
    // ~10 us, almost all of it that load).  Positions outside (the start
    // search past the segment, the three-page check) load their window.
    const uint64_t rlo = (lo - base) & ~15ull;
    uint32_t sbytes = 0;
    if (stage_cap) {
        sbytes = static_cast<uint32_t>(min<uint64_t>((hi - base) + kWin + 16 - rlo, stage_cap)) & ~15u;
        lds32* sd = (lds32*)seg_dyn;
        for (uint32_t b = l; b < sbytes / 16; b += kWave) {
            const uint64_t q = rlo + 16ull * b;
            uint4 v = make_uint4(0u, 0u, 0u, 0u);
            if (q + 16 <= len) {
                v = *reinterpret_cast<const uint4*>(d + q);  // (the buffer is 16-byte aligned)
            } else if (q < len) {  // the buffer's last bytes, zeros past them
                uint32_t w0 = 0, w1 = 0, w2 = 0, w3 = 0;
                for (uint32_t j = 0; j < 16 && q + j < len; j++) {
                    const uint32_t x = static_cast<uint32_t>(d[q + j]) << (8 * (j & 3));
                    if (j < 4) w0 |= x;
                    else if (j < 8) w1 |= x;
                    else if (j < 12) w2 |= x;
                    else w3 |= x;
                }
                v = make_uint4(w0, w1, w2, w3);
            }
            sd[4 * b] = v.x;
            sd[4 * b + 1] = v.y;
            sd[4 * b + 2] = v.z;
            sd[4 * b + 3] = v.w;
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    }
    // 256 bytes from pos: in the staged segment, else loaded into the window
    lds8c* segb = (lds8c*)seg_dyn;
    auto at = [&](uint64_t pos) -> lds8c* {
        const uint64_t rel = pos - base;
        if (rel >= rlo && rel + kWin <= rlo + sbytes) return segb + (rel - rlo);
        return wb + load_win(win, d, base, len, pos);
    };
    uint64_t pos = lo;
    DHdr h;
    if (k > 0) {
        // the first plausible three-page chain start (format.cpp speculate):
        // 64 positions per window; candidates in order
        // (a narrower opening than the host's: PageHeader field 1, an i32 in
        // short form, 0x15, as every writer emits it; a start it misses only
        // leaves the segment unlinked, which refuses the walk)
        const uint64_t lim = min(hi, lo + kScanLimit);
        bool found = false;
        for (uint64_t c = lo; c < lim && !found; c += kWave) {
            // a PageHeader opens with field 1 (an i32 in short form, 0x15),
            // the page type's zigzag byte (0, 2, 4 or 6: types 0..3, as the
            // plausibility rule requires) and field 2 (0x15): the three bytes
            // reject almost every payload position before a parse is tried
            // (a parse from a random 0x15 could run through hundreds of bytes)
            lds8c* cw = at(c);
            uint64_t m = __ballot(c + l < lim && cw[l] == 0x15u && (cw[l + 1] & 0xF9u) == 0u && cw[l + 2] == 0x15u);
            while (m && !found) {
                const uint32_t b = static_cast<uint32_t>(__builtin_ctzll(m));
                m &= m - 1;
                const uint64_t p = c + b;
                bool ok = dev_parse(at(p), kWin, h) && dev_plausible(h, p, end);  // 256 bytes from p
                uint64_t q = p + h.hs + static_cast<uint64_t>(h.comp);
                for (int hop = 0; hop < 2 && ok && q < end; hop++) {
                    DHdr h2;
                    ok = dev_parse(at(q), kWin, h2) && dev_plausible(h2, q, end);
                    if (ok) q += h2.hs + static_cast<uint64_t>(h2.comp);
                }
                if (ok) {
                    found = true;
                    pos = p;
                }
            }
        }
        if (!found) pos = hi;
    }
    WalkRec* r = recs + static_cast<uint64_t>(k) * cap;
    uint32_t n = 0, fl = 0;
    auto emit = [&](uint64_t at_pos, const DHdr& x0) {
        if (l == 0) {
            WalkRec x;
            x.pos = at_pos;
            x.hs = x0.hs;
            x.comp = x0.comp;
            x.uncomp = x0.uncomp;
            x.type = x0.type;
            x.nv = x0.type == PQ_DICTIONARY_PAGE ? x0.dictnv : x0.dnv;
            x.enc = x0.denc;
            x.flags = x0.flags;
            r[n] = x;
        }
        n++;
    };
    // Headers parsed 64 at a time, a lane each: every position of the staged
    // segment that opens like a PageHeader (the three bytes of the start
    // search) from the chain's position on is a candidate; the lanes parse
    // their candidates at once and the chain then steps through them by
    // position (one header parse per hop on the whole wave was ~5-7 us of
    // serial latency).  A chain position that is not a candidate takes the
    // one-wave parse below, which also reports a refused header.
    __shared__ uint64_t cand[kWave];
    auto rl64 = [](uint64_t v, uint32_t i) -> uint64_t {
        return (static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v >> 32), static_cast<int>(i)))) << 32) |
               static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(static_cast<uint32_t>(v)), static_cast<int>(i)));
    };
    auto rl32 = [](int32_t v, uint32_t i) -> int32_t { return __builtin_amdgcn_readlane(v, static_cast<int>(i)); };
    while (pos < hi && !fl) {
        const uint64_t rel0 = pos - base;
        if (sbytes && rel0 >= rlo && hi - base + kWin <= rlo + sbytes) {
            // up to 64 candidates from pos on (in position order)
            const uint64_t pos_before = pos;
            uint32_t got = 0;
            for (uint64_t c0 = pos; c0 < hi && got < static_cast<uint32_t>(kWave); c0 += kWave) {
                const uint64_t c = c0 + l;
                lds8c* q = segb + (c - base - rlo);
                const bool sig = c < hi && q[0] == 0x15u && (q[1] & 0xF9u) == 0u && q[2] == 0x15u;
                const uint64_t m = __ballot(sig);
                const uint32_t rank = __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(m >> 32),
                                                                 __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(m), 0u));
                if (sig && got + rank < static_cast<uint32_t>(kWave)) cand[got + rank] = c;
                got += static_cast<uint32_t>(__builtin_popcountll(m));
            }
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            const uint32_t nc = min(got, static_cast<uint32_t>(kWave));
            const uint64_t mc = l < nc ? cand[l] : ~0ull;
            DHdr hc{};
            bool okc = false;
            if (l < nc) okc = dev_parse(segb + (mc - base - rlo), kWin, hc) && hc.comp >= 0 && mc + hc.hs <= end;
            // the chain through this batch
            uint32_t j = 0;
            bool miss = false;
            while (pos < hi) {
                while (j < nc && rl64(mc, j) < pos) j++;
                if (j >= nc) break;             // past the batch: the next one from pos
                if (rl64(mc, j) != pos) { miss = true; break; }
                if (!__builtin_amdgcn_readlane(static_cast<int>(okc), static_cast<int>(j))) { fl |= 2u; break; }
                if (n == cap) { fl |= 1u; break; }
                DHdr x;
                x.type = rl32(hc.type, j);
                x.uncomp = rl32(hc.uncomp, j);
                x.comp = rl32(hc.comp, j);
                x.dnv = rl32(hc.dnv, j);
                x.denc = rl32(hc.denc, j);
                x.dictnv = rl32(hc.dictnv, j);
                x.hs = static_cast<uint32_t>(rl32(static_cast<int32_t>(hc.hs), j));
                x.flags = static_cast<uint32_t>(rl32(static_cast<int32_t>(hc.flags), j));
                emit(pos, x);
                pos += x.hs + static_cast<uint64_t>(x.comp);
                j++;
            }
            if (fl || (!miss && pos != pos_before)) continue;
            // (no candidate at or past pos, or pos is not one: one step below)
        }
        // one header on the whole wave (positions outside the staged segment
        // or not opening like a candidate)
        // a header reaching past the extent parsed zeros the host walk would
        // read as file bytes: refuse rather than emit a different table
        if (!dev_parse(at(pos), kWin, h) || h.comp < 0 || pos + h.hs > end) { fl |= 2u; break; }
        if (n == cap) { fl |= 1u; break; }
        emit(pos, h);
        pos += h.hs + static_cast<uint64_t>(h.comp);
    }
    if (l == 0) segs[k] = WalkSeg{pos, n, fl};
}

// Per segment on the chain: the record where the chain enters (found by the
// previous segment's exit), and the chain's pages / data values / last
// dictionary page (local index) / first invalid page from there.
struct WalkLink {
    int32_t entry;      // record index where the chain enters; -1: skipped (inside a page), -2: refused
    int32_t pages;
    int64_t values;
    int32_t last_dict;  // local (from entry), -1 none
    int32_t bad;        // local index of the first invalid page, -1 none
};

__device__ uint32_t rec_kind(const WalkRec& x, int64_t* v, bool* bad) {  // format.cpp linked_walk kind()
    *v = 0;
    *bad = false;
    if (x.comp < 0) { *bad = true; return 0; }
    if (x.type == PQ_DICTIONARY_PAGE) {
        *bad = !(x.flags & 2u) || x.nv < 0;
        return 1;
    }
    if (x.type == PQ_DATA_PAGE) {
        *bad = !(x.flags & 1u) || x.nv < 0;
        *v = x.nv;
        return 2;
    }
    return 0;
}

constexpr uint32_t kMaxSkip = 64;  // segments a page may span (a longer page refuses)

constexpr int kLinkWaves = 4;  // a wave per segment
__global__ void __launch_bounds__(kLinkWaves * kWave) k_walk_link(uint64_t start, uint64_t seg, uint32_t nseg, uint32_t cap, const WalkRec* __restrict__ recs,
                            const WalkSeg* __restrict__ segs, WalkLink* __restrict__ links) {
    const uint32_t k = blockIdx.x * kLinkWaves + threadIdx.x / kWave;
    const uint32_t ln = __lane_id();
    if (k >= nseg) return;
    const WalkSeg S = segs[k];
    const WalkRec* r = recs + static_cast<uint64_t>(k) * cap;
    WalkLink L{-2, 0, 0, -1, -1};
    // the chain arrives where the nearest earlier segment with records left
    // (segments inside a longer page find no header start: no records; one
    // whose records lie inside a page is refused below)
    uint64_t expect = start;
    bool have = k == 0;
    for (uint32_t j = k; j > 0 && k - j < kMaxSkip && !have; j--) {
        const WalkSeg P = segs[j - 1];
        if (P.n > 0 || j - 1 == 0) {
            expect = P.n > 0 ? P.exit : start;
            have = true;
        }
    }
    const uint64_t lo = start + seg * k, hi = lo + seg;
    if (have && expect >= hi) {  // inside a page that covers the segment
        L.entry = S.n == 0 ? -1 : -2;
    } else if (have && expect >= lo && !(S.flags & 1u)) {
        // the record at `expect` (records are in position order), then the
        // chain's values, its first invalid page and last dictionary page from
        // there, a lane per record
        int32_t entry = -1;
        for (uint32_t a0 = 0; a0 < S.n; a0 += kWave) {
            const uint32_t a = a0 + ln;
            const uint64_t p = a < S.n ? r[a].pos : ~0ull;
            const uint64_t m = __ballot(p >= expect);
            if (m) {
                const uint32_t f = static_cast<uint32_t>(__builtin_ctzll(m));
                const uint64_t pf = (static_cast<uint64_t>(static_cast<uint32_t>(__shfl(static_cast<int>(p >> 32), static_cast<int>(f)))) << 32) |
                                    static_cast<uint32_t>(__shfl(static_cast<int>(static_cast<uint32_t>(p)), static_cast<int>(f)));
                if (pf == expect) entry = static_cast<int32_t>(a0 + f);
                break;
            }
        }
        if (entry >= 0) {
            L.entry = entry;
            L.pages = static_cast<int32_t>(S.n - static_cast<uint32_t>(entry));
            for (uint32_t j0 = static_cast<uint32_t>(entry); j0 < S.n; j0 += kWave) {
                const uint32_t j = j0 + ln;
                const bool act = j < S.n;
                int64_t v = 0;
                bool bad = false;
                uint32_t kd = 0;
                if (act) kd = rec_kind(r[j], &v, &bad);
                const uint64_t mb = __ballot(act && bad);
                const uint32_t lim = mb ? static_cast<uint32_t>(__builtin_ctzll(mb)) : static_cast<uint32_t>(kWave);
                const bool take = act && ln < lim;
                int64_t sv = take ? v : 0;
#pragma unroll
                for (int o = 1; o < kWave; o <<= 1) sv += __shfl_xor(sv, o);
                L.values += sv;
                const uint64_t md = __ballot(take && kd == 1);
                if (md) L.last_dict = static_cast<int32_t>(j0 + 63u - static_cast<uint32_t>(__builtin_clzll(md)) - static_cast<uint32_t>(entry));
                if (mb) {
                    L.bad = static_cast<int32_t>(j0 + lim - static_cast<uint32_t>(entry));
                    break;
                }
            }
        }
    }
    if (ln == 0) links[k] = L;
}

// One workgroup: prefixes over the segments, the cut, the dictionary in force.
// out[0] = pages (or -1: refused), the per-segment page base / value base /
// dictionary-in base go to base_pg / base_val / dict_in.
constexpr int kScanThreads = 1024;
__global__ void __launch_bounds__(kScanThreads) k_walk_scan(int64_t num_values, uint32_t nseg, uint32_t cap,
                                                          const WalkRec* __restrict__ recs,
                                                          const WalkSeg* __restrict__ segs,
                                                          const WalkLink* __restrict__ links,
                                                          int64_t* __restrict__ base_pg, int64_t* __restrict__ base_val,
                                                          int64_t* __restrict__ dict_in, int64_t* __restrict__ out) {
    __shared__ int64_t sp[kScanThreads], sv[kScanThreads], sd[kScanThreads];
    __shared__ int64_t carry_p, carry_v, carry_d;
    __shared__ int32_t cut_seg, first;
    if (threadIdx.x == 0) { carry_p = 0; carry_v = 0; carry_d = -1; cut_seg = -1; first = 0x7FFFFFFF; }
    __syncthreads();
    for (uint32_t c0 = 0; c0 < nseg; c0 += kScanThreads) {
        const uint32_t k = c0 + threadIdx.x;
        const WalkLink L = k < nseg ? links[k] : WalkLink{-1, 0, 0, -1, -1};
        const bool on = L.entry >= 0;  // (-1: skipped inside a page, -2: refused)
        // (segments past the cut are unused; an unlinked one before it refuses)
        sp[threadIdx.x] = on ? L.pages : 0;
        sv[threadIdx.x] = on ? L.values : 0;
        __syncthreads();
        // inclusive scans (Hillis-Steele) of pages and values
        for (uint32_t o = 1; o < kScanThreads; o <<= 1) {
            const int64_t a = threadIdx.x >= o ? sp[threadIdx.x - o] : 0;
            const int64_t b = threadIdx.x >= o ? sv[threadIdx.x - o] : 0;
            __syncthreads();
            sp[threadIdx.x] += a;
            sv[threadIdx.x] += b;
            __syncthreads();
        }
        const int64_t pinc = sp[threadIdx.x], vinc = sv[threadIdx.x];
        const int64_t pex = carry_p + pinc - (on ? L.pages : 0), vex = carry_v + vinc - (on ? L.values : 0);
        // the last dictionary page at or before each segment's end (global index)
        sd[threadIdx.x] = (on && L.last_dict >= 0) ? pex + L.last_dict : -1;
        __syncthreads();
        for (uint32_t o = 1; o < kScanThreads; o <<= 1) {
            const int64_t a = threadIdx.x >= o ? sd[threadIdx.x - o] : -1;
            __syncthreads();
            sd[threadIdx.x] = max(sd[threadIdx.x], a);
            __syncthreads();
        }
        const int64_t dex = threadIdx.x > 0 ? max(carry_d, sd[threadIdx.x - 1]) : carry_d;
        if (k < nseg) {
            base_pg[k] = pex;
            base_val[k] = vex;
            dict_in[k] = dex;
        }
        // the cut: the first segment whose values reach num_values (or whose
        // chain holds an invalid page, or that is not linked: refused below)
        const bool stop = k < nseg && (L.entry == -2 || L.bad >= 0 || (on && vex + L.values >= num_values));
        if (stop) atomicMin(&first, static_cast<int32_t>(k));
        __syncthreads();
        if (threadIdx.x == 0) {
            if (first != 0x7FFFFFFF) cut_seg = first;
            carry_p += sp[kScanThreads - 1];
            carry_v += sv[kScanThreads - 1];
            carry_d = max(carry_d, sd[kScanThreads - 1]);
        }
        __syncthreads();
        if (cut_seg >= 0) break;
    }
    if (threadIdx.x != 0) return;
    int64_t npages = -1;
    const int32_t K = cut_seg;
    if (K >= 0) {
        const WalkLink L = links[K];
        if (L.entry >= 0) {
            // within segment K: the page at which the values reach num_values;
            // an invalid page before it refuses (the host reports the error)
            const WalkRec* r = recs + static_cast<uint64_t>(K) * cap;
            int64_t a = base_val[K];
            const uint32_t n = segs[K].n;
            for (uint32_t j = static_cast<uint32_t>(L.entry); j < n; j++) {
                int64_t v;
                bool bad;
                rec_kind(r[j], &v, &bad);
                if (bad) break;
                a += v;
                if (a >= num_values) { npages = base_pg[K] + (j - L.entry) + 1; break; }
            }
        }
    }
    out[0] = npages;
    out[1] = K;
    if (K >= 0) {  // (diagnostics: the stopping segment's link state, records, exit)
        out[2] = links[K].entry;
        out[3] = segs[K].n;
        out[4] = static_cast<int64_t>(segs[K].exit);
        out[5] = links[K].bad;
        out[6] = K > 0 ? static_cast<int64_t>(segs[K - 1].exit) : -1;
        out[7] = segs[K].n ? static_cast<int64_t>(recs[static_cast<uint64_t>(K) * cap].pos) : -1;
    }
}

// A wave per segment, a lane per record: the page's first row is an
// exclusive scan of the records' values, the dictionary in force an
// inclusive max-scan of the dictionary pages' indices (one thread walking a
// segment's records paid a dependent global load per record).
constexpr int kEmitWaves = 4;
__global__ void __launch_bounds__(kEmitWaves * kWave) k_walk_emit(uint32_t cap, const WalkRec* __restrict__ recs, const WalkSeg* __restrict__ segs,
                            const WalkLink* __restrict__ links, const int64_t* __restrict__ base_pg,
                            const int64_t* __restrict__ base_val, const int64_t* __restrict__ dict_in,
                            const int64_t* __restrict__ out, pq_page_desc* __restrict__ pages) {
    const int64_t npages = out[0];
    const int64_t K = out[1];
    const uint32_t k = blockIdx.x * kEmitWaves + threadIdx.x / kWave;
    const uint32_t ln = __lane_id();
    if (npages < 0 || static_cast<int64_t>(k) > K) return;
    const WalkLink L = links[k];
    if (L.entry < 0) return;
    const WalkRec* r = recs + static_cast<uint64_t>(k) * cap;
    const uint32_t n = segs[k].n;
    int64_t idx0 = base_pg[k], row = base_val[k], d = dict_in[k];
    for (uint32_t j0 = static_cast<uint32_t>(L.entry); j0 < n && idx0 < npages; j0 += kWave, idx0 += kWave) {
        const uint32_t j = j0 + ln;
        const int64_t idx = idx0 + ln;
        const bool act = j < n && idx < npages;
        WalkRec x{};
        int64_t v = 0;
        uint32_t kd = 0;
        if (act) {
            x = r[j];
            bool bad;
            kd = rec_kind(x, &v, &bad);
        }
        int64_t inc = v, dm = (act && kd == 1) ? idx : -1;
#pragma unroll
        for (int o = 1; o < kWave; o <<= 1) {
            const int64_t a = __shfl_up(inc, static_cast<unsigned>(o));
            const int64_t b = __shfl_up(dm, static_cast<unsigned>(o));
            if (ln >= static_cast<uint32_t>(o)) {
                inc += a;
                dm = max(dm, b);
            }
        }
        if (act) {
            pq_page_desc p{};
            p.header_offset = static_cast<int64_t>(x.pos);
            p.payload_offset = static_cast<int64_t>(x.pos + x.hs);
            p.payload_size = x.comp;
            p.page_type = x.type;
            p.first_row = row + inc - v;
            p.page_num = -1;
            p.uncompressed_size = x.uncomp;
            if (kd == 1) {
                p.num_values = x.nv;
                p.page_num = static_cast<int32_t>(idx);
            } else if (kd == 2) {
                p.num_values = x.nv;
                p.encoding = x.enc;
                p.page_num = static_cast<int32_t>(idx);
            }
            p.dict_page = static_cast<int32_t>(max(d, dm));
            pages[idx] = p;
        }
        row += __shfl(inc, kWave - 1);
        d = max(d, __shfl(dm, kWave - 1));
    }
}

}  // namespace

void launch_walk(hipStream_t s, const WalkLaunch& W) {
    const uint32_t nseg = W.nseg;
    // the segment staged in LDS when it is at most 32 KiB (+ one header window)
    const uint32_t stage = W.seg <= 32768u ? static_cast<uint32_t>(W.seg) + kWin + 32 : 0u;
    if (stage) ensure_dyn_lds(reinterpret_cast<const void*>(k_walk_seg), stage);
    hipLaunchKernelGGL(k_walk_seg, dim3(nseg), dim3(kWave), stage, s, W.bytes, W.base, W.len, W.start,
                       W.end, W.seg, nseg, W.cap, W.recs, reinterpret_cast<WalkSeg*>(W.segs), stage);
    hipLaunchKernelGGL(k_walk_link, dim3((nseg + kLinkWaves - 1) / kLinkWaves), dim3(kLinkWaves * kWave), 0, s, W.start, W.seg, nseg, W.cap, W.recs,
                       reinterpret_cast<const WalkSeg*>(W.segs), reinterpret_cast<WalkLink*>(W.links));
    hipLaunchKernelGGL(k_walk_scan, dim3(1), dim3(kScanThreads), 0, s, W.num_values, nseg, W.cap, W.recs,
                       reinterpret_cast<const WalkSeg*>(W.segs), reinterpret_cast<const WalkLink*>(W.links), W.base_pg,
                       W.base_val, W.dict_in, W.out);
    hipLaunchKernelGGL(k_walk_emit, dim3((nseg + kEmitWaves - 1) / kEmitWaves), dim3(kEmitWaves * kWave), 0, s, W.cap, W.recs,
                       reinterpret_cast<const WalkSeg*>(W.segs), reinterpret_cast<const WalkLink*>(W.links), W.base_pg,
                       W.base_val, W.dict_in, W.out, W.pages);
}

size_t walk_seg_bytes() { return sizeof(WalkSeg); }
size_t walk_link_bytes() { return sizeof(WalkLink); }

}  // namespace pqk
