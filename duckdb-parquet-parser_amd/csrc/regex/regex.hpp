// regex.hpp — the --regex-column page filter (README.md:54-64 of the
// reference; the reference ships no implementation, so the contract is
// SURVEY §8a R-REGEX).
//
// Patterns are compiled on the host into a Glushkov position automaton over
// bytes (<= 64 character positions) with ^/$ as zero-width assertion leaves,
// and run on the GPU as a bit-parallel NFA: one 64-bit state word per string,
// next = follow(D) & class[byte], follow(D) assembled from 8-bit chunk tables
// kept in LDS.  Match = Python `re.search(p, s, re.ASCII) is not None` on the
// supported subset (literals, ., [...], [^...], \d\w\s\D\W\S, * + ? {m,n},
// lazy forms, |, (...), (?:...), ^, $ with \Z semantics, \A, \Z).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "kernels/kernels.hpp"

namespace pqre {

constexpr int kMaxPos = 64;

struct Program {
    int npos = 0;                 // character positions
    uint64_t cls[256] = {};       // positions whose byte class contains c
    uint64_t follow[kMaxPos] = {};// follow set (character positions) of each position
    uint64_t first_at0 = 0;       // positions that may consume byte 0 (through ^)
    uint64_t first_mid = 0;       // positions that may start a match at byte i > 0
    uint64_t last = 0;            // positions after which the match may end anywhere
    uint64_t accept_end = 0;      // positions after which the match may end at end ($)
    bool nonempty_trivial = false;// every non-empty string matches (empty match exists)
    bool empty_string = false;    // the empty string matches
};

// Device image of a Program (18.5 KiB; staged into LDS by the kernels).
struct DevProg {
    uint64_t cls[256];
    uint64_t ftab[8][256];        // follow(D) = OR_k ftab[k][(D >> 8k) & 0xFF]
    uint64_t first_at0, first_mid, last, accept_end;
    uint32_t nchunks;             // ceil(npos / 8)
    uint32_t nonempty_trivial;
    uint32_t empty_string;
    uint32_t pad;
};

struct DeviceProgram {
    DevProg* d;
};

// The same automaton as a DFA over the Glushkov position sets (subset
// construction on the host, regex_host.cpp build_dfa).  Layout in device
// memory: this header, then u16 trans[nstates * nclasses]; an entry is the
// next state id with bit 15 set when that state accepts at the string end
// ($).  State ids: 0 DEAD (absorbing reject), 1 ACCEPT (absorbing match),
// 2 START (before the first byte), 3.. position sets.
constexpr uint32_t kDfaMaxBytes = 32768;
constexpr uint32_t kDfaRowBytes = 516;  // full-table row stride (129 dwords)
struct DevDfa {
    uint32_t nstates, nclasses;
    uint32_t empty_string;      // "" matches
    uint32_t nonempty_trivial;  // every non-empty string matches
    uint32_t bytes;             // header + table, multiple of 16
    uint32_t full;              // 1: one column per byte value, entries = next row's byte
                                // offset (rows kDfaRowBytes apart); column 256 of a row:
                                // the state accepts at the string end
    uint32_t pad[2];
    uint32_t sink_lo, sink_hi;  // full tables: absorbing states (every byte stays), bit = state
    uint32_t pad2;
    uint32_t anchored;          // matches start at byte 0 only (the DFA dies early on most strings)
    uint8_t cls_of[256];        // byte -> class
};
static_assert(sizeof(DevDfa) % 16 == 0, "table alignment");
enum : uint32_t { DFA_DEAD = 0, DFA_ACCEPT = 1, DFA_START = 2 };

// Builds the DFA image; false if it would exceed kDfaMaxBytes (the NFA
// kernel is used then).
bool build_dfa(const Program& p, std::vector<uint8_t>* image);

// Windowed PLAIN scan (chunks without dictionary pages).  Per wave: the
// window (+32 zero bytes), a u16 offset per possible string, per-page counts,
// list bases and kept counts, the hit mask.
constexpr uint32_t regex_plain_wave_lds(uint32_t win_bytes) { return win_bytes + 32 + win_bytes / 2 + 3 * 64 * 4 + 16; }
uint32_t regex_plain_waves(uint32_t dfa_bytes, uint32_t win_bytes);
uint32_t regex_plain_lds(uint32_t dfa_bytes, uint32_t win_bytes);
int regex_plain_occupancy(uint32_t lds);
bool regex_plain_lds_ok();  // k_regex_plain's constant-address LDS table is valid (no static LDS)
void launch_regex_plain(hipStream_t s, const uint8_t* dfa, uint32_t dfa_bytes, uint32_t win_bytes,
                        const uint8_t* bytes, const pqk::DevPage* pages, const pqk::DevBatch* wins, int nwins,
                        int32_t* ticket, int grid, pqk::ColumnParams cp, int neg, uint8_t* page_flags,
                        pqk::DevErr* page_err, int32_t* err_any,
                        const uint16_t* index_in = nullptr, uint16_t* index_out = nullptr, bool sink = false);

void launch_regex_lanes(hipStream_t s, const uint8_t* dfa, uint32_t dfa_bytes, const uint8_t* bytes,
                        const pqk::DevPage* pages, int npages, const pqk::DevDict* dicts,
                        const int32_t* dict_count, const uint8_t* dict_match, pqk::ColumnParams cp, int neg,
                        uint8_t* page_flags, pqk::DevErr* page_err, int32_t* err_any);

int check(const std::string& pattern, std::string* msg);
int compile(const std::string& pattern, Program* out, std::string* msg);
bool match_host(const Program& p, const uint8_t* s, size_t n);
void build_dev(const Program& p, DevProg* out);

DeviceProgram* upload_program(const Program& p, hipStream_t s);
void free_device_program(DeviceProgram* p);

// fill1/nfill1: bytes set to 1 (page flags), zero/nzero: u32 words cleared
// (the chunk's status words), both in the same launch (the scan over the
// codes of a checked decode then needs no fill kernels); may be null / 0.
void launch_regex_dict(hipStream_t s, const DeviceProgram* prog, const uint8_t* bytes,
                       const pqk::DevDict* dicts, int ndicts, const uint64_t* entries,
                       const int32_t* dict_count, uint8_t* dict_match, uint8_t* fill1 = nullptr,
                       int64_t nfill1 = 0, uint32_t* zero = nullptr, int64_t nzero = 0);

void launch_regex_pages(hipStream_t s, const DeviceProgram* prog, const uint8_t* bytes,
                        const pqk::DevPage* pages, int npages, const pqk::DevDict* dicts,
                        const uint64_t* entries, const int32_t* dict_count,
                        const uint8_t* dict_match, pqk::ColumnParams cp, int neg,
                        uint8_t* page_flags, pqk::DevErr* page_err, int32_t* err_any);

}  // namespace pqre
