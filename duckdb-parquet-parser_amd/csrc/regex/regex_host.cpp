// regex_host.cpp — pattern parser and Glushkov construction (host side).
//
// Supported subset (where RE2 and Python `re` agree on match
// existence): literals (UTF-8 literal characters become byte sequences),
// `.`, `[...]` / `[^...]` with ASCII items and ranges, `\d \w \s \D \W \S`,
// `\t \n \r \f \v \xhh`, escaped punctuation, `* + ? {m} {m,} {m,n}` and their
// lazy forms, `|`, `( )`, `(?: )`, `(?P<name> )`, `^`/`\A`, `$`/`\Z` (end of
// string only).  `.` and negated classes consume one UTF-8 code point
// (ASCII byte, or lead byte followed by continuation bytes).  Anything else is
// rejected with PQ_ERR_REGEX rather than guessed.
#include <bitset>
#include <cstring>
#include <stdexcept>
#include <vector>

#include "pq_gpu.h"
#include "regex/regex.hpp"

namespace pqre {
namespace {

constexpr int kMaxLeaves = 192;
using Set = std::bitset<kMaxLeaves>;
using Bytes = std::bitset<256>;

struct ReError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

enum Kind { CHAR, BOL, EOL, EMPTY, CAT, ALT, STAR };
struct Node {
    Kind k;
    Bytes set;
    std::vector<int> kids;
};

struct Parser {
    const std::string& p;
    size_t i = 0;
    std::vector<Node> nodes;
    explicit Parser(const std::string& s) : p(s) {}

    int add(Kind k, Bytes set = Bytes(), std::vector<int> kids = {}) {
        nodes.push_back(Node{k, set, std::move(kids)});
        return static_cast<int>(nodes.size()) - 1;
    }
    int copy(int n) {
        Node x = nodes[n];
        for (auto& c : x.kids) c = copy(c);
        nodes.push_back(x);
        return static_cast<int>(nodes.size()) - 1;
    }
    bool eof() const { return i >= p.size(); }
    char peek() const { return p[i]; }

    static Bytes ascii_range(int a, int b) {
        Bytes s;
        for (int c = a; c <= b; c++) s.set(c);
        return s;
    }
    static Bytes digit() { return ascii_range('0', '9'); }
    static Bytes word() { return ascii_range('a', 'z') | ascii_range('A', 'Z') | digit() | ascii_range('_', '_'); }
    static Bytes space() {
        Bytes s;
        for (char c : std::string(" \t\n\r\f\v")) s.set(static_cast<uint8_t>(c));
        return s;
    }
    static Bytes ascii_all() { return ascii_range(0, 127); }

    // a code point outside ASCII: lead byte then continuation bytes
    int multibyte() {
        int lead = add(CHAR, ascii_range(0xC0, 0xFF));
        int cont = add(CHAR, ascii_range(0x80, 0xBF));
        return add(CAT, Bytes(), {lead, add(STAR, Bytes(), {cont})});
    }
    int cls_node(const Bytes& ascii, bool nonascii) {
        int a = add(CHAR, ascii);
        if (!nonascii) return a;
        return add(ALT, Bytes(), {a, multibyte()});
    }

    int parse_alt() {
        std::vector<int> alts{parse_cat()};
        while (!eof() && peek() == '|') {
            i++;
            alts.push_back(parse_cat());
        }
        return alts.size() == 1 ? alts[0] : add(ALT, Bytes(), alts);
    }
    int parse_cat() {
        std::vector<int> items;
        while (!eof() && peek() != '|' && peek() != ')') items.push_back(parse_repeat());
        if (items.empty()) return add(EMPTY);
        return items.size() == 1 ? items[0] : add(CAT, Bytes(), items);
    }
    bool parse_braces(int* lo, int* hi) {  // at '{'; false = literal '{'
        size_t j = i + 1;
        auto num = [&](int* v) {
            size_t s = j;
            long x = 0;
            while (j < p.size() && p[j] >= '0' && p[j] <= '9') {
                x = x * 10 + (p[j] - '0');
                if (x > 1000) throw ReError("repeat count too large");
                j++;
            }
            *v = static_cast<int>(x);
            return j > s;
        };
        int a = 0, b = -1;
        bool ha = num(&a);
        if (j < p.size() && p[j] == '}') {
            if (!ha) return false;
            b = a;
        } else if (j < p.size() && p[j] == ',') {
            j++;
            bool hb = num(&b);
            if (!hb) b = -1;
            if (j >= p.size() || p[j] != '}') return false;
            if (!ha) throw ReError("{,n} repeat is not supported (RE2 and Python disagree)");
        } else {
            return false;
        }
        if (b >= 0 && b < a) throw ReError("min repeat greater than max repeat");
        *lo = a;
        *hi = b;
        i = j + 1;
        return true;
    }
    int parse_repeat() {
        size_t start = i;
        int atom = parse_atom();
        bool quantified = false;
        while (!eof()) {
            char c = peek();
            int lo, hi;
            if (c == '*' || c == '+' || c == '?') {
                i++;
                lo = c == '+' ? 1 : 0;
                hi = c == '?' ? 1 : -1;
            } else if (c == '{') {
                if (!parse_braces(&lo, &hi)) break;
            } else {
                break;
            }
            if (quantified) throw ReError("multiple repeat");
            Kind ak = nodes[atom].k;
            if (ak == BOL || ak == EOL || i == start) throw ReError("nothing to repeat");
            quantified = true;
            if (!eof() && peek() == '?') i++;  // lazy: same language
            atom = repeat(atom, lo, hi);
        }
        return atom;
    }
    int repeat(int a, int lo, int hi) {
        std::vector<int> parts;
        for (int k = 0; k < lo; k++) parts.push_back(k == 0 ? a : copy(a));
        if (hi < 0) {
            parts.push_back(add(STAR, Bytes(), {lo == 0 ? a : copy(a)}));
        } else {
            for (int k = lo; k < hi; k++) {
                int x = (k == 0 && lo == 0) ? a : copy(a);
                parts.push_back(add(ALT, Bytes(), {x, add(EMPTY)}));
            }
        }
        if (parts.empty()) return add(EMPTY);
        return parts.size() == 1 ? parts[0] : add(CAT, Bytes(), parts);
    }
    // class escape inside/outside brackets: returns true with (set, nonascii)
    bool class_escape(char e, Bytes* s, bool* nonascii) {
        *nonascii = false;
        switch (e) {
            case 'd': *s = digit(); return true;
            case 'w': *s = word(); return true;
            case 's': *s = space(); return true;
            case 'D': *s = ascii_all() & ~digit(); *nonascii = true; return true;
            case 'W': *s = ascii_all() & ~word(); *nonascii = true; return true;
            case 'S': *s = ascii_all() & ~space(); *nonascii = true; return true;
            default: return false;
        }
    }
    int escape_byte(char e) {  // single-character escapes; -1 = not one
        switch (e) {
            case 't': return '\t';
            case 'n': return '\n';
            case 'r': return '\r';
            case 'f': return '\f';
            case 'v': return '\v';
            case 'x': {
                if (i + 2 > p.size()) throw ReError("bad \\x escape");
                int v = 0;
                for (int k = 0; k < 2; k++) {
                    char h = p[i++];
                    int d = (h >= '0' && h <= '9') ? h - '0'
                            : (h >= 'a' && h <= 'f') ? h - 'a' + 10
                            : (h >= 'A' && h <= 'F') ? h - 'A' + 10 : -1;
                    if (d < 0) throw ReError("bad \\x escape");
                    v = v * 16 + d;
                }
                if (v >= 0x80) throw ReError("non-ASCII \\x escape is not supported");
                return v;
            }
            default:
                if ((e >= 'a' && e <= 'z') || (e >= 'A' && e <= 'Z') || (e >= '0' && e <= '9'))
                    return -1;
                if (static_cast<uint8_t>(e) >= 0x80) return -1;
                return static_cast<uint8_t>(e);  // escaped punctuation
        }
    }
    int parse_class() {  // after '['
        bool neg = false;
        if (!eof() && peek() == '^') { neg = true; i++; }
        Bytes s;
        bool nonascii = false, first = true;
        for (;;) {
            if (eof()) throw ReError("unterminated character set");
            char c = p[i];
            if (c == ']' && !first) { i++; break; }
            first = false;
            int lo;
            if (static_cast<uint8_t>(c) >= 0x80) throw ReError("non-ASCII character in a class");
            if (c == '\\') {
                i++;
                if (eof()) throw ReError("bad escape");
                char e = p[i++];
                Bytes es;
                bool na;
                if (class_escape(e, &es, &na)) {
                    s |= es;
                    nonascii |= na;
                    continue;
                }
                lo = escape_byte(e);
                if (lo < 0) throw ReError(std::string("unsupported escape \\") + e);
            } else {
                lo = static_cast<uint8_t>(c);
                i++;
            }
            if (i + 1 < p.size() && p[i] == '-' && p[i + 1] != ']') {
                i++;
                char d = p[i];
                int hi;
                if (static_cast<uint8_t>(d) >= 0x80) throw ReError("non-ASCII character in a class");
                if (d == '\\') {
                    i++;
                    if (eof()) throw ReError("bad escape");
                    char e = p[i++];
                    Bytes es;
                    bool na;
                    if (class_escape(e, &es, &na)) throw ReError("bad character range");
                    hi = escape_byte(e);
                    if (hi < 0) throw ReError(std::string("unsupported escape \\") + e);
                } else {
                    hi = static_cast<uint8_t>(d);
                    i++;
                }
                if (hi < lo) throw ReError("bad character range");
                s |= ascii_range(lo, hi);
            } else {
                s.set(lo);
            }
        }
        if (neg) return cls_node(ascii_all() & ~s, !nonascii);
        return cls_node(s, nonascii);
    }
    int parse_atom() {
        if (eof()) throw ReError("unexpected end of pattern");
        char c = p[i];
        switch (c) {
            case '(': {
                i++;
                if (!eof() && peek() == '?') {
                    if (i + 1 < p.size() && p[i + 1] == ':') {
                        i += 2;
                    } else if (i + 2 < p.size() && p[i + 1] == 'P' && p[i + 2] == '<') {
                        size_t e = p.find('>', i + 3);
                        if (e == std::string::npos || e == i + 3) throw ReError("bad group name");
                        i = e + 1;
                    } else {
                        throw ReError("unsupported group construct (?...)");
                    }
                }
                int a = parse_alt();
                if (eof() || peek() != ')') throw ReError("missing ), unterminated subpattern");
                i++;
                return a;
            }
            case ')': throw ReError("unbalanced parenthesis");
            case '*': case '+': case '?': throw ReError("nothing to repeat");
            case '[': i++; return parse_class();
            case '.': i++; return cls_node(ascii_all() & ~ascii_range('\n', '\n'), true);
            case '^': i++; return add(BOL);
            case '$': i++; return add(EOL);
            case '\\': {
                i++;
                if (eof()) throw ReError("bad escape (end of pattern)");
                char e = p[i++];
                if (e == 'A') return add(BOL);
                if (e == 'Z') return add(EOL);
                Bytes s;
                bool na;
                if (class_escape(e, &s, &na)) return cls_node(s, na);
                int b = escape_byte(e);
                if (b < 0) throw ReError(std::string("unsupported escape \\") + e);
                Bytes one;
                one.set(b);
                return add(CHAR, one);
            }
            default: {
                uint8_t u = static_cast<uint8_t>(c);
                if (u < 0x80) {
                    i++;
                    Bytes one;
                    one.set(u);
                    return add(CHAR, one);
                }
                // UTF-8 literal character -> its byte sequence
                int len = u >= 0xF0 ? 4 : u >= 0xE0 ? 3 : u >= 0xC0 ? 2 : 0;
                if (!len || i + len > p.size()) throw ReError("invalid UTF-8 in pattern");
                std::vector<int> seq;
                for (int k = 0; k < len; k++) {
                    Bytes one;
                    one.set(static_cast<uint8_t>(p[i + k]));
                    seq.push_back(add(CHAR, one));
                }
                i += len;
                return add(CAT, Bytes(), seq);
            }
        }
    }
};

struct Glushkov {
    const std::vector<Node>& nodes;
    std::vector<int> leaf_of_node;
    std::vector<Kind> leaf_kind;
    std::vector<Bytes> leaf_set;
    std::vector<Set> follow;
    explicit Glushkov(const std::vector<Node>& n) : nodes(n), leaf_of_node(n.size(), -1) {}

    struct Info {
        bool nullable;
        Set first, last;
    };
    Info walk(int n) {
        const Node& x = nodes[n];
        Info r{false, Set(), Set()};
        switch (x.k) {
            case CHAR: case BOL: case EOL: {
                int id = static_cast<int>(leaf_kind.size());
                if (id >= kMaxLeaves) throw ReError("pattern too large");
                leaf_kind.push_back(x.k);
                leaf_set.push_back(x.set);
                follow.push_back(Set());
                r.first.set(id);
                r.last.set(id);
                return r;
            }
            case EMPTY: r.nullable = true; return r;
            case ALT: {
                for (int k : x.kids) {
                    Info c = walk(k);
                    r.nullable |= c.nullable;
                    r.first |= c.first;
                    r.last |= c.last;
                }
                return r;
            }
            case CAT: {
                r.nullable = true;
                bool firstkid = true;
                for (int k : x.kids) {
                    Info c = walk(k);
                    if (firstkid) { r = c; firstkid = false; continue; }
                    for (size_t l = 0; l < follow.size(); l++)
                        if (r.last.test(l)) follow[l] |= c.first;
                    if (r.nullable) r.first |= c.first;
                    r.last = c.nullable ? (r.last | c.last) : c.last;
                    r.nullable = r.nullable && c.nullable;
                }
                return r;
            }
            case STAR: {
                Info c = walk(x.kids[0]);
                for (size_t l = 0; l < follow.size(); l++)
                    if (c.last.test(l)) follow[l] |= c.first;
                c.nullable = true;
                return c;
            }
        }
        return r;
    }
};

Set kind_mask(const std::vector<Kind>& kinds, Kind k) {
    Set s;
    for (size_t i = 0; i < kinds.size(); i++)
        if (kinds[i] == k) s.set(i);
    return s;
}

// closure of `from` under follow restricted to leaves in `allowed`
Set closure(const Set& from, const Set& allowed, const std::vector<Set>& follow) {
    Set cur = from & allowed, seen = cur;
    while (cur.any()) {
        Set nxt;
        for (size_t l = 0; l < follow.size(); l++)
            if (cur.test(l)) nxt |= follow[l] & allowed;
        cur = nxt & ~seen;
        seen |= cur;
    }
    return seen;
}

}  // namespace

int compile(const std::string& pattern, Program* out, std::string* msg) {
    try {
        Parser ps(pattern);
        int root = ps.parse_alt();
        if (!ps.eof()) throw ReError("unbalanced parenthesis");
        Glushkov g(ps.nodes);
        Glushkov::Info top = g.walk(root);
        const size_t L = g.leaf_kind.size();
        Set charm = kind_mask(g.leaf_kind, CHAR), bolm = kind_mask(g.leaf_kind, BOL),
            eolm = kind_mask(g.leaf_kind, EOL);
        if (charm.count() > static_cast<size_t>(kMaxPos))
            throw ReError("pattern needs more than 64 positions");
        std::vector<int> bit(L, -1);
        int nb = 0;
        for (size_t l = 0; l < L; l++)
            if (charm.test(l)) bit[l] = nb++;
        auto to_mask = [&](const Set& s) {
            uint64_t m = 0;
            for (size_t l = 0; l < L; l++)
                if (s.test(l) && bit[l] >= 0) m |= 1ull << bit[l];
            return m;
        };
        Program p;
        p.npos = nb;
        for (size_t l = 0; l < L; l++) {
            if (bit[l] < 0) continue;
            for (int c = 0; c < 256; c++)
                if (g.leaf_set[l].test(c)) p.cls[c] |= 1ull << bit[l];
            p.follow[bit[l]] = to_mask(g.follow[l]);
        }
        // starts: through ^ leaves at byte 0, directly elsewhere
        Set bol_reach = closure(top.first, bolm, g.follow);
        Set at0 = top.first;
        for (size_t l = 0; l < L; l++)
            if (bol_reach.test(l)) at0 |= g.follow[l];
        p.first_at0 = to_mask(at0);
        p.first_mid = to_mask(top.first);
        p.last = to_mask(top.last);
        for (size_t l = 0; l < L; l++) {
            if (bit[l] < 0) continue;
            bool acc = top.last.test(l);
            if (!acc) acc = (closure(g.follow[l], eolm, g.follow) & top.last).any();
            if (acc) p.accept_end |= 1ull << bit[l];
        }
        bool empty_at0 = (bol_reach & top.last).any();
        bool empty_at_end = (closure(top.first, eolm, g.follow) & top.last).any();
        bool empty_any = (closure(top.first, bolm | eolm, g.follow) & top.last).any();
        p.nonempty_trivial = top.nullable || empty_at0 || empty_at_end;
        p.empty_string = top.nullable || empty_any;
        *out = p;
        return 0;
    } catch (const ReError& e) {
        if (msg) *msg = e.what();
        return PQ_ERR_REGEX;
    }
}

int check(const std::string& pattern, std::string* msg) {
    Program p;
    return compile(pattern, &p, msg);
}

bool match_host(const Program& p, const uint8_t* s, size_t n) {
    if (n == 0) return p.empty_string;
    if (p.nonempty_trivial) return true;
    uint64_t D = 0;
    for (size_t i = 0; i < n; i++) {
        uint64_t f = i == 0 ? p.first_at0 : p.first_mid;
        for (int b = 0; b < p.npos; b++)
            if (D >> b & 1) f |= p.follow[b];
        D = f & p.cls[s[i]];
        if (D & p.last) return true;
    }
    return (D & p.accept_end) != 0;
}

void build_dev(const Program& p, DevProg* d) {
    std::memset(d, 0, sizeof *d);
    std::memcpy(d->cls, p.cls, sizeof p.cls);
    for (int k = 0; k < 8; k++)
        for (int v = 0; v < 256; v++) {
            uint64_t f = 0;
            for (int b = 0; b < 8; b++)
                if ((v >> b) & 1 && 8 * k + b < p.npos) f |= p.follow[8 * k + b];
            d->ftab[k][v] = f;
        }
    d->first_at0 = p.first_at0;
    d->first_mid = p.first_mid;
    d->last = p.last;
    d->accept_end = p.accept_end;
    d->nchunks = static_cast<uint32_t>((p.npos + 7) / 8);
    d->nonempty_trivial = p.nonempty_trivial;
    d->empty_string = p.empty_string;
}

bool build_dfa(const Program& p, std::vector<uint8_t>* image) {
    // byte classes: bytes with the same position mask behave alike
    std::vector<uint64_t> cmask;
    uint8_t cls_of[256];
    for (int b = 0; b < 256; b++) {
        size_t c = 0;
        while (c < cmask.size() && cmask[c] != p.cls[b]) c++;
        if (c == cmask.size()) cmask.push_back(p.cls[b]);
        cls_of[b] = static_cast<uint8_t>(c);
    }
    uint32_t nc = static_cast<uint32_t>(cmask.size());
    const size_t max_states = (kDfaMaxBytes - sizeof(DevDfa)) / (2 * nc);
    auto follow = [&](uint64_t D) {
        uint64_t f = 0;
        for (int b = 0; b < p.npos; b++)
            if (D >> b & 1) f |= p.follow[b];
        return f;
    };
    std::vector<uint64_t> sets = {0, 0, 0};  // DEAD, ACCEPT, START (sets unused)
    std::vector<uint16_t> trans;
    std::vector<std::pair<uint64_t, uint32_t>> index;  // set -> id (linear; state counts are small)
    auto id_of = [&](uint64_t D, bool& overflow) -> uint32_t {
        if (D & p.last) return DFA_ACCEPT;
        if (D == 0 && p.first_mid == 0) return DFA_DEAD;
        for (auto& e : index)
            if (e.first == D) return e.second;
        if (sets.size() >= max_states || sets.size() >= 0x7FFF) { overflow = true; return DFA_DEAD; }
        const uint32_t id = static_cast<uint32_t>(sets.size());
        sets.push_back(D);
        index.push_back({D, id});
        return id;
    };
    auto entry = [&](uint32_t id) -> uint16_t {
        const bool acc = id == DFA_ACCEPT || (id >= 3 && (sets[id] & p.accept_end) != 0);
        return static_cast<uint16_t>(id | (acc ? 0x8000u : 0u));
    };
    bool overflow = false;
    trans.assign(3 * nc, 0);
    for (uint32_t c = 0; c < nc; c++) {
        trans[DFA_DEAD * nc + c] = entry(DFA_DEAD);
        trans[DFA_ACCEPT * nc + c] = entry(DFA_ACCEPT);
    }
    for (uint32_t c = 0; c < nc; c++) {
        const uint32_t id = id_of(p.first_at0 & cmask[c], overflow);
        trans[DFA_START * nc + c] = static_cast<uint16_t>(id);  // flags patched below
    }
    for (size_t s = 3; s < sets.size() && !overflow; s++) {
        trans.resize((s + 1) * nc);
        const uint64_t f = p.first_mid | follow(sets[s]);
        for (uint32_t c = 0; c < nc; c++) trans[s * nc + c] = static_cast<uint16_t>(id_of(f & cmask[c], overflow));
    }
    if (overflow) return false;
    trans.resize(sets.size() * nc);
    for (auto& t : trans) t = entry(t & 0x7FFFu);
    bool is_full = false;
    // few states: expand to one column per byte value (no class lookup on
    // the device's dependent chain)
    if (sets.size() * kDfaRowBytes < 0x8000u && sizeof(DevDfa) + sets.size() * kDfaRowBytes <= kDfaMaxBytes) {
        std::vector<uint16_t> full(sets.size() * 256);
        for (size_t st = 0; st < sets.size(); st++)
            for (int b = 0; b < 256; b++) full[st * 256 + b] = trans[st * nc + cls_of[b]];
        // entries hold the next state's row byte offset, so the device forms
        // the next address with one mask and one add.  Rows are 516 bytes
        // apart (129 dwords): the LDS bank of an entry is (state + byte/2) mod
        // 32, so lanes in different states spread over the banks.
        // Entries are bare offsets (no flag bits to mask on the chain);
        // column 256 of a row holds whether that state accepts at the string
        // end ($), read once per string.
        std::vector<uint16_t> pad(sets.size() * (kDfaRowBytes / 2), 0);
        for (size_t st = 0; st < sets.size(); st++) {
            for (int b = 0; b < 256; b++) {
                const uint32_t t = full[st * 256 + b];
                pad[st * (kDfaRowBytes / 2) + b] = static_cast<uint16_t>((t & 0x7FFFu) * kDfaRowBytes);
            }
            const bool acc = st == DFA_ACCEPT || (st >= 3 && (sets[st] & p.accept_end) != 0);
            pad[st * (kDfaRowBytes / 2) + 256] = acc ? 1 : 0;
        }
        full.swap(pad);
        trans.swap(full);
        nc = 256;
        for (int b = 0; b < 256; b++) cls_of[b] = static_cast<uint8_t>(b);
        is_full = true;
    }
    DevDfa h{};
    h.anchored = p.first_mid == 0 ? 1u : 0u;
    if (is_full) {  // absorbing states (the device stops a batch once every string sits in one)
        for (size_t st = 0; st < sets.size() && st < 64; st++) {
            bool stay = true;
            for (int b = 0; b < 256 && stay; b++) stay = trans[st * (kDfaRowBytes / 2) + b] == st * kDfaRowBytes;
            if (stay) (st < 32 ? h.sink_lo : h.sink_hi) |= 1u << (st & 31);
        }
    }
    h.nstates = static_cast<uint32_t>(sets.size());
    h.nclasses = nc;
    h.empty_string = p.empty_string;
    h.nonempty_trivial = p.nonempty_trivial;
    h.full = is_full;
    h.bytes = static_cast<uint32_t>((sizeof(DevDfa) + 2 * trans.size() + 15) / 16 * 16);
    std::memcpy(h.cls_of, cls_of, 256);
    image->assign(h.bytes, 0);
    std::memcpy(image->data(), &h, sizeof h);
    std::memcpy(image->data() + sizeof h, trans.data(), 2 * trans.size());
    return true;
}

}  // namespace pqre

// DFA form of the same match (test hook: the kernel's automaton on the host).
// Returns 1/0, PQ_ERR_REGEX for a bad pattern, or PQ_ERR_UNSUPPORTED when the
// DFA exceeds its size cap.
extern "C" int pq_regex_match_host_dfa(const char* pattern, const uint8_t* s, size_t n) {
    pqre::Program p;
    std::string msg;
    if (pqre::compile(pattern ? pattern : "", &p, &msg)) return PQ_ERR_REGEX;
    std::vector<uint8_t> img;
    if (!pqre::build_dfa(p, &img)) return PQ_ERR_UNSUPPORTED;
    pqre::DevDfa h;
    std::memcpy(&h, img.data(), sizeof h);
    const uint16_t* t = reinterpret_cast<const uint16_t*>(img.data() + sizeof h);
    if (n == 0) return h.empty_string ? 1 : 0;
    if (h.nonempty_trivial) return 1;
    if (h.full) {
        const uint8_t* tb = reinterpret_cast<const uint8_t*>(t);
        uint32_t e = pqre::DFA_START * pqre::kDfaRowBytes;
        for (size_t i = 0; i < n; i++) {
            uint16_t v;
            std::memcpy(&v, tb + e + 2 * s[i], 2);
            e = v;
        }
        uint16_t acc;
        std::memcpy(&acc, tb + e + 512, 2);
        return (e == pqre::DFA_ACCEPT * pqre::kDfaRowBytes || acc) ? 1 : 0;
    }
    uint32_t e = pqre::DFA_START;
    for (size_t i = 0; i < n; i++) e = t[(e & 0x7FFFu) * h.nclasses + h.cls_of[s[i]]];
    return ((e & 0x7FFFu) == pqre::DFA_ACCEPT || (e >> 15)) ? 1 : 0;
}

// DFA statistics of a pattern (diagnostics): states, byte classes, full table.
extern "C" int pq_regex_dfa_info(const char* pattern, int* nstates, int* nclasses, int* full, int* bytes) {
    pqre::Program p;
    std::string msg;
    if (pqre::compile(pattern ? pattern : "", &p, &msg)) return PQ_ERR_REGEX;
    std::vector<uint8_t> img;
    if (!pqre::build_dfa(p, &img)) return PQ_ERR_UNSUPPORTED;
    pqre::DevDfa h;
    std::memcpy(&h, img.data(), sizeof h);
    if (nstates) *nstates = static_cast<int>(h.nstates);
    if (nclasses) *nclasses = static_cast<int>(h.nclasses);
    if (full) *full = static_cast<int>(h.full);
    if (bytes) *bytes = static_cast<int>(h.bytes);
    return 0;
}

// The DFA's absorbing-state masks (test hook; k_regex_plain<true> stops a
// batch once every string sits in one).  PQ_ERR_REGEX / PQ_ERR_UNSUPPORTED
// as above.
extern "C" int pq_regex_dfa_sinks(const char* pattern, uint32_t* sink_lo, uint32_t* sink_hi) {
    pqre::Program p;
    std::string msg;
    if (pqre::compile(pattern ? pattern : "", &p, &msg)) return PQ_ERR_REGEX;
    std::vector<uint8_t> img;
    if (!pqre::build_dfa(p, &img)) return PQ_ERR_UNSUPPORTED;
    pqre::DevDfa h;
    std::memcpy(&h, img.data(), sizeof h);
    if (sink_lo) *sink_lo = h.sink_lo;
    if (sink_hi) *sink_hi = h.sink_hi;
    return 0;
}

extern "C" int pq_regex_match_host(const char* pattern, const uint8_t* s, size_t n) {
    pqre::Program p;
    std::string msg;
    if (pqre::compile(pattern ? pattern : "", &p, &msg)) return PQ_ERR_REGEX;
    return pqre::match_host(p, s, n) ? 1 : 0;
}

// Prebuilt host DFA handle (the same table k_regex_plain walks), for the CPU
// regex baseline (bench.py cpu_baseline: the reference ColumnReader's values
// matched with this DFA on the host's threads).  Not used by any product
// path.  pq_regex_host_new returns NULL for a bad pattern or an oversized DFA.
struct pq_regex_host {
    pqre::DevDfa h;
    std::vector<uint8_t> img;
};

extern "C" pq_regex_host* pq_regex_host_new(const char* pattern) {
    pqre::Program p;
    std::string msg;
    if (pqre::compile(pattern ? pattern : "", &p, &msg)) return nullptr;
    auto* r = new pq_regex_host;
    if (!pqre::build_dfa(p, &r->img)) {
        delete r;
        return nullptr;
    }
    std::memcpy(&r->h, r->img.data(), sizeof r->h);
    return r;
}

extern "C" void pq_regex_host_free(pq_regex_host* r) { delete r; }

extern "C" int pq_regex_host_match(const pq_regex_host* r, const uint8_t* s, size_t n) {
    const pqre::DevDfa& h = r->h;
    if (n == 0) return h.empty_string ? 1 : 0;
    if (h.nonempty_trivial) return 1;
    const uint8_t* tb = r->img.data() + sizeof h;
    if (h.full) {
        constexpr uint32_t kAcc = pqre::DFA_ACCEPT * pqre::kDfaRowBytes;
        uint32_t e = pqre::DFA_START * pqre::kDfaRowBytes;
        for (size_t i = 0; i < n; i++) {
            uint16_t v;
            std::memcpy(&v, tb + e + 2 * s[i], 2);
            e = v;
            if (e == kAcc) return 1;  // ACCEPT absorbs
        }
        uint16_t acc;
        std::memcpy(&acc, tb + e + 512, 2);
        return acc ? 1 : 0;
    }
    const uint16_t* t = reinterpret_cast<const uint16_t*>(tb);
    uint32_t e = pqre::DFA_START;
    for (size_t i = 0; i < n; i++) {
        e = t[(e & 0x7FFFu) * h.nclasses + h.cls_of[s[i]]];
        if ((e & 0x7FFFu) == pqre::DFA_ACCEPT) return 1;
    }
    return (e >> 15) ? 1 : 0;
}
