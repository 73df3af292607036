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

int check(const std::string& pattern, std::string* msg);
int compile(const std::string& pattern, Program* out, std::string* msg);
bool match_host(const Program& p, const uint8_t* s, size_t n);
void build_dev(const Program& p, DevProg* out);

DeviceProgram* upload_program(const Program& p, hipStream_t s);
void free_device_program(DeviceProgram* p);

void launch_regex_dict(hipStream_t s, const DeviceProgram* prog, const uint8_t* bytes,
                       const pqk::DevDict* dicts, int ndicts, const uint64_t* entries,
                       const int32_t* dict_count, uint8_t* dict_match);

void launch_regex_pages(hipStream_t s, const DeviceProgram* prog, const uint8_t* bytes,
                        const pqk::DevPage* pages, int npages, const pqk::DevDict* dicts,
                        const uint64_t* entries, const int32_t* dict_count,
                        const uint8_t* dict_match, pqk::ColumnParams cp, int neg,
                        uint8_t* page_flags, pqk::DevErr* page_err, int32_t* err_any);

}  // namespace pqre
