// plan.cpp — host-side planning of a device chunk's launches: which kernel
// path a chunk takes (dict_pipe.hip, plain_ba.hip, dict_fused.hip), its
// LDS carve-up and grid, the page tables of a walk, and the windows of the
// windowed regex scan.  No launches here (capi.hip runs them).
#include <algorithm>
#include <cstring>

#include "host/capi_state.hpp"

namespace pqcapi {

// The three-pass dictionary path (dict_pipe.hip) takes a BYTE_ARRAY chunk
// whose data pages all use one dictionary page that fits in LDS.
// Dictionaries the writer's LDS cannot hold (or of more than 65,535 entries):
// every page through k_pipe_big<true> (32-bit codes, index bit widths up to
// 24, entry lengths from HBM), then k_pipe_wwide, which reads the entry words
// and characters from HBM/L2.  Called by plan_pipe after its page checks
// (dictionary-encoded pages of one dictionary).
static void plan_pipe_wide(pq_ctx* ctx, pq_chunk* c, const PVec<DevPage>& pages, const DevDict& d, int32_t dict_id) {
    if (!ctx->opt_pipe_wide) return;
    std::vector<int32_t> big;
    uint32_t big_bytes = 0;
    big.reserve(pages.size());
    for (size_t i = 0; i < pages.size(); i++) {
        const DevPage& pg = pages[i];
        if (pg.nvals > pqk::kBigTiles * pqk::kTileRows || static_cast<uint32_t>(pg.size) > pqk::kBigMaxBytes) return;
        big.push_back(static_cast<int32_t>(i));
        big_bytes = std::max(big_bytes, static_cast<uint32_t>(pg.size));
    }
    if (pqk::pipe_big_lds(big_bytes, 0) > 160u * 1024) return;
    // a dictionary page past k_dict_index's LDS decodes in launch_dict_big,
    // which also files its 16-byte entry slots: the writer keeps one per row
    // of its tile in LDS (10 KiB per wave: four waves per workgroup, three
    // workgroups per CU; five per workgroup measured 82 vs 58 µs, r4e)
    const bool pad = static_cast<uint64_t>(std::max(d.size, 0)) + 32 > pqk::kDictLdsCap;
    const int wpw = std::max(1, std::min(pad ? 4 : 16, ctx->opt_write_waves));
    pqk::PipePlan pl = pqk::plan_pipe_wide(wpw, pad);
    if (pl.blocks_per_cu == 0) return;
    if (ctx->opt_write_bpc > 0) pl.blocks_per_cu = std::min(pl.blocks_per_cu, ctx->opt_write_bpc);
    c->pipe = true;
    c->pipe_wide = true;
    c->pipe_small = false;
    c->pipe_small_bytes = 0;
    c->pipe_count = false;
    c->hbig = std::move(big);
    c->big_max_bytes = big_bytes;
    c->pipe_dict = dict_id;
    c->pipe_dict_payload = static_cast<uint32_t>(d.size);
    c->pipe_entry_base = d.entry_base;
    c->pipe_dict_chars_bytes = 0;
    c->pipe_dict_bytes = 0;
    c->pipe_lds = pl.lds;
    c->pipe_grid = ctx->cus * pl.blocks_per_cu;
    c->pipe_ecap = static_cast<uint32_t>(std::min<int64_t>(d.nvals, d.size / 4 + 1));
    c->pipe_cus = ctx->cus;
    c->pipe_wpw = wpw;
}

void plan_pipe(pq_ctx* ctx, pq_chunk* c, const PVec<DevPage>& pages, const std::vector<DevDict>& dicts) {
    c->pipe = false;
    c->pipe_wide = false;
    c->pipe_count = false;
    c->pipe_small = false;
    c->hbig.clear();
    c->big_max_bytes = 0;
    if (c->type != PQ_BYTE_ARRAY || c->max_def > 254 || c->max_def < 0 || c->max_rep < 0 || pages.empty()) return;
    int32_t dict_id = -1;
    bool multi = false, small = false;
    std::vector<int32_t> big;
    uint32_t big_bytes = 0, small_bytes = 0;
    for (size_t i = 0; i < pages.size(); i++) {
        const DevPage& pg = pages[i];
        if (pg.mode != pqk::MODE_DICT || pg.size > (1 << 27) || pg.size < 0) return;
        if (pg.nvals > pqk::kPipeSmallRows || ctx->opt_big_all) {
            // k_pipe_big: the page's jump table and up to kBigTiles tiles in one workgroup
            if (pg.nvals > pqk::kBigTiles * pqk::kTileRows || static_cast<uint32_t>(pg.size) > pqk::kBigMaxBytes) return;
            big.push_back(static_cast<int32_t>(i));
            big_bytes = std::max(big_bytes, static_cast<uint32_t>(pg.size));
        } else {
            small = true;
            multi |= pg.nvals > pqk::kTileRows;
            small_bytes = std::max(small_bytes, static_cast<uint32_t>(pg.size));
        }
        if (dict_id >= 0 && pg.dict != dict_id) return;
        dict_id = pg.dict;
    }
    const DevDict& d = dicts[dict_id];
    if (d.size < 0 || d.nvals < 0) return;
    if (d.size > 65536 - 64 || d.nvals > 65535) return plan_pipe_wide(ctx, c, pages, d, dict_id);
    const int64_t ecap = std::min<int64_t>(d.nvals, d.size / 4 + 1);
    if (!big.empty() && pqk::pipe_big_lds(big_bytes, std::min<uint32_t>(static_cast<uint32_t>(ecap), pqk::kBigLens)) > 160u * 1024)
        return;
    const uint32_t chars_bytes = (static_cast<uint32_t>(d.size) + 15) / 16 * 16 + 16;
    const uint32_t dict_bytes = 16 + chars_bytes + static_cast<uint32_t>((4 * ecap + 15) / 16 * 16);
    const int wpw = std::max(1, std::min(16, ctx->opt_write_waves));
    pqk::PipePlan pl = pqk::plan_pipe_lds(dict_bytes, wpw);
    if (pl.blocks_per_cu == 0) return plan_pipe_wide(ctx, c, pages, d, dict_id);
    if (ctx->opt_write_bpc > 0) pl.blocks_per_cu = std::min(pl.blocks_per_cu, ctx->opt_write_bpc);
    const int cus = ctx->cus;
    c->pipe = true;
    c->pipe_small = small;
    c->pipe_small_bytes = small_bytes;
    c->pipe_count = multi && c->max_def > 0;
    c->hbig = std::move(big);
    c->big_max_bytes = big_bytes;
    c->pipe_dict = dict_id;
    c->pipe_dict_payload = static_cast<uint32_t>(d.size);
    c->pipe_entry_base = d.entry_base;
    c->pipe_dict_chars_bytes = chars_bytes;
    c->pipe_dict_bytes = dict_bytes;
    c->pipe_lds = pl.lds;
    c->pipe_grid = cus * pl.blocks_per_cu;
    c->pipe_ecap = static_cast<uint32_t>(ecap);
    c->pipe_cus = cus;
    c->pipe_wpw = wpw;
}

// PLAIN BYTE_ARRAY chunks without levels go through plain_ba.hip: windows of
// consecutive page slots of at most kPWin bytes.
void plan_plain(pq_ctx* ctx, pq_chunk* c, const PVec<DevPage>& pages) {
    c->plain = false;
    c->plain_spec = false;
    c->plain_opt = false;
    c->hpwins.clear();
    c->hpwbase.clear();
    c->hpwpage.clear();
    c->hchunk_base.clear();
    c->hchunks.clear();
    if (c->type != PQ_BYTE_ARRAY || c->max_def < 0 || c->max_rep != 0 || pages.empty()) return;
    // OPTIONAL: the value sections (after the levels) are decoded as
    // REQUIRED-shaped pages of their non-null values; the windows and chunks
    // below cover the whole slots, which hold them
    const bool opt = c->max_def > 0;
    auto slot = [](const DevPage& p) {
        return (static_cast<uint64_t>(std::max(p.size, 0)) + 15) / 16 * 16 + 16;
    };
    bool big = false;
    for (const auto& pg : pages) {
        if (pg.mode != pqk::MODE_PLAIN || pg.nvals < 0) return;
        big |= slot(pg) > pqk::kPWin;
    }
    if (big) {
        // every page in kPChunk-byte chunks, windows of kPChunkGroup chunks
        // (the pseudo pages k_plain_link writes, one per chunk)
        if (pages.size() > (1u << 24)) return;
        int64_t nch = 0;
        for (size_t p = 0; p < pages.size(); p++) {
            const uint32_t size = static_cast<uint32_t>(std::max(pages[p].size, 0));
            const uint32_t k = std::max<uint32_t>(1, (size + pqk::kPChunk - 1) / pqk::kPChunk);
            c->hchunk_base.push_back(static_cast<int32_t>(nch));
            for (uint32_t i = 0; i < k; i++) {
                c->hchunks.push_back(make_uint2(static_cast<uint32_t>(p), i));
            }
            const uint64_t se = pages[p].off + slot(pages[p]);
            for (uint32_t g = 0; g < k; g += pqk::kPChunkGroup) {
                pqk::DevBatch b{};
                b.p0 = static_cast<int32_t>(nch + g);
                b.np = static_cast<int32_t>(std::min(pqk::kPChunkGroup, k - g));
                b.img_lo = pages[p].off + static_cast<uint64_t>(g) * pqk::kPChunk;
                b.img_bytes = static_cast<uint32_t>(std::min<uint64_t>(pqk::kPWin, se - b.img_lo));
                c->hpwins.push_back(b);
            }
            nch += k;
            if (nch > (1ll << 30)) return;
        }
        c->hchunk_base.push_back(static_cast<int32_t>(nch));
        c->plain_spec = true;
        for (const auto& b : c->hpwins) c->hpwpage.push_back(static_cast<int32_t>(c->hchunks[static_cast<size_t>(b.p0)].x));
        // one-pass form over the pseudo pages (k_plain_fused, kWinPseudo): per
        // window, its page's first output byte (pages whose strings fill them
        // exactly: size - 4 * num_values each, verified on the device) minus
        // the page's image offset plus 4 x its first row
        bool known = true;
        std::vector<int64_t> pbase(pages.size());
        int64_t acc = 0;
        for (size_t p = 0; p < pages.size(); p++) {
            pbase[p] = acc;
            const int64_t x = static_cast<int64_t>(pages[p].size) - 4 * static_cast<int64_t>(pages[p].nvals);
            known &= x >= 0;
            acc += x;
        }
        if (known && !opt) {
            c->hpwbase.reserve(c->hpwins.size());
            for (const auto& b : c->hpwins) {
                const uint2 ch = c->hchunks[static_cast<size_t>(b.p0)];
                const DevPage& pg = pages[ch.x];
                c->hpwbase.push_back(pbase[ch.x] - static_cast<int64_t>(pg.off) + 4 * pg.first_row);
            }
        }
    } else {
        // greedy windows from the start of each page range (one range per
        // host thread; a range start also starts a window), with each
        // window's characters for the one-pass form (k_plain_fused): a page's
        // strings fill it exactly, so its characters are size - 4 *
        // num_values; verified on the device
        const size_t NP = pages.size();
        const int T = static_cast<int>(std::min<size_t>(16, std::max<size_t>(1, NP / 16384)));
        const size_t per = (NP + static_cast<size_t>(T) - 1) / static_cast<size_t>(T);
        std::vector<std::vector<pqk::DevBatch>> wparts(static_cast<size_t>(T));
        std::vector<std::vector<int64_t>> cparts(static_cast<size_t>(T));
        std::vector<char> kparts(static_cast<size_t>(T), 1);
        pqfmt::parallel_run(T, T, [&](int t) {
            auto& W = wparts[static_cast<size_t>(t)];
            auto& C = cparts[static_cast<size_t>(t)];
            const size_t end = std::min(NP, (static_cast<size_t>(t) + 1) * per);
            W.reserve((end - std::min(end, static_cast<size_t>(t) * per)) / 4 + 1);
            C.reserve(W.capacity());
            bool known = true;
            size_t p = static_cast<size_t>(t) * per;
            while (p < end) {
                pqk::DevBatch b{};
                b.p0 = static_cast<int32_t>(p);
                b.img_lo = pages[p].off;
                uint64_t hi = b.img_lo;
                size_t q = p;
                int64_t ch = 0;
                while (q < end && q - p < 64 && pages[q].off >= b.img_lo) {
                    const uint64_t e = pages[q].off + slot(pages[q]);
                    if (e - b.img_lo > pqk::kPWin) break;
                    hi = e;
                    const int64_t x = static_cast<int64_t>(pages[q].size) - 4 * static_cast<int64_t>(pages[q].nvals);
                    known &= x >= 0;
                    ch += x;
                    b.nrows += static_cast<uint32_t>(std::max(pages[q].nvals, 0));
                    q++;
                }
                b.row0 = pages[p].first_row;
                b.np = static_cast<int32_t>(q - p);
                b.img_bytes = static_cast<uint32_t>(hi - b.img_lo);
                W.push_back(b);
                C.push_back(ch);
                p = q;
            }
            kparts[static_cast<size_t>(t)] = known;
        });
        bool known = true;
        size_t nw = 0;
        for (int t = 0; t < T; t++) {
            nw += wparts[static_cast<size_t>(t)].size();
            known &= kparts[static_cast<size_t>(t)] != 0;
        }
        c->hpwins.reserve(nw);
        for (const auto& W : wparts) c->hpwins.insert(c->hpwins.end(), W.begin(), W.end());
        if (known && !opt) {
            c->hpwbase.reserve(nw + 1);
            c->hpwbase.push_back(0);
            for (const auto& C : cparts)
                for (int64_t ch : C) c->hpwbase.push_back(c->hpwbase.back() + ch);
        }
    }
    c->plain_opt = opt;
    c->opt_lane_levels = true;
    for (const auto& pg : pages) c->opt_lane_levels &= pg.nvals <= pqk::kOptLaneRows;
    const int cus = ctx->cus;
    c->plain_grid = cus * pqk::plain_write_blocks_per_cu();
    c->plain = true;
}

// Decide whether every chunk of the column can take the fused BYTE_ARRAY
// path (dict_fused.hip) and size its LDS carve-up; otherwise the generic
// rows -> scan -> gather path runs.
void plan_fused(pq_ctx* ctx, pq_chunk* c, const PVec<DevPage>& pages,
                const std::vector<DevDict>& dicts) {
    c->fused = false;
    if (!ctx->opt_fused || c->type != PQ_BYTE_ARRAY || c->max_def > 255 || c->max_def < 0 || c->ranges.empty()) return;
    const int cus = ctx->cus;
    const uint32_t kLds = 160 * 1024;
    for (auto& r : c->ranges) {
        int32_t dict_id = -1;
        uint32_t maxn = 0, maxs = 0;
        for (int p = r.p0; p < r.p0 + r.np; p++) {
            const DevPage& pg = pages[p];
            if (pg.mode == pqk::MODE_DICT) {
                if (dict_id >= 0 && pg.dict != dict_id) return;  // several dictionaries in force
                dict_id = pg.dict;
            }
            maxn = std::max(maxn, static_cast<uint32_t>(std::max(pg.nvals, 0)));
            maxs = std::max(maxs, static_cast<uint32_t>(std::max(pg.size, 0)));
        }
        if (maxn > 4096 || maxs > 16384) return;
        r.dict_id = dict_id;
        r.rows_cap = (std::max(maxn, 64u) + 63) / 64 * 64;
        r.stage_bytes = (maxs + 15) / 16 * 16 + 16;
        r.wave_bytes = pqk::fused_wave_bytes(r.rows_cap, r.stage_bytes);
        r.dict_chars_bytes = r.dict_bytes = 0;
        if (dict_id >= 0) {
            const DevDict& d = dicts[dict_id];
            if (d.size > 65536 - 64 || d.nvals < 0 || d.nvals > 65535) return;
            int64_t ecap = std::min<int64_t>(d.nvals, d.size / 4 + 1);
            r.dict_chars_bytes = (static_cast<uint32_t>(d.size) + 15) / 16 * 16 + 16;
            r.dict_bytes = r.dict_chars_bytes + static_cast<uint32_t>((4 * ecap + 15) / 16 * 16);
        }
        if (r.dict_bytes + r.wave_bytes > kLds) return;
        // producer/writer pairs per workgroup (dict_fused.hip)
        int pairs = static_cast<int>(std::min<uint32_t>(8, (kLds - r.dict_bytes) / r.wave_bytes));
        if (ctx->opt_waves > 0) pairs = std::max(1, std::min(pairs, ctx->opt_waves / 2));
        const int W = 2 * pairs;
        r.waves = W;
        uint32_t lds = r.dict_bytes + static_cast<uint32_t>(pairs) * r.wave_bytes;
        int per_cu = pqk::fused_occupancy_waves(lds, W);
        if (per_cu < 1) per_cu = 1;
        int need = (r.np + pairs - 1) / pairs;
        r.grid = std::max(1, std::min(per_cu * cus, need));
    }
    c->fused = true;
}

// The host page tables of one walk (dictionary and data pages, their image
// slots and copy list) on host threads: per-range counts, then every page
// written at its index.  Same tables as upload_walked's page loop, which
// runs instead when a page goes through the codec pass (returns false).
bool plan_pages_parallel(pq_chunk* c, const pq_chunk_desc& desc, const pqfmt::WalkResult& w, bool keep_walk,
                                int hw, int64_t seq, int64_t& row_base, int64_t& img, PVec<DevPage>& hpages,
                                std::vector<DevDict>& hdicts, HVec<std::pair<int64_t, int64_t>>& copies,
                                HVec<int32_t>& copy_size) {
    const size_t N = w.pages.size();
    const int T = static_cast<int>(std::min<size_t>(static_cast<size_t>(hw), std::max<size_t>(1, N / 16384)));
    const size_t per = (N + static_cast<size_t>(T) - 1) / static_cast<size_t>(T);
    struct Part {
        int64_t nslot = 0, ndata = 0, bytes = 0, rows = 0, payload = 0;
        bool codec = false;
        std::vector<size_t> dicts;
    };
    std::vector<Part> parts(static_cast<size_t>(T));
    auto slot_bytes = [](int32_t size) { return (static_cast<int64_t>(size) + 15) / 16 * 16 + 16; };
    pqfmt::parallel_run(T, T, [&](int t) {
        Part& P = parts[static_cast<size_t>(t)];
        const size_t a = static_cast<size_t>(t) * per, b = std::min(N, a + per);
        for (size_t i = a; i < b; i++) {
            const pq_page_desc& p = w.pages[i];
            const bool dict = p.page_type == PQ_DICTIONARY_PAGE, data = p.page_type == PQ_DATA_PAGE;
            if (!dict && !data) continue;
            P.codec |= (p.flags & (PQ_PAGE_COMPRESSED | PQ_PAGE_V2)) != 0;
            P.nslot++;
            P.bytes += slot_bytes(p.payload_size);
            P.payload += p.payload_size;
            if (dict) P.dicts.push_back(i);
            else {
                P.ndata++;
                P.rows += p.num_values;
            }
        }
    });
    for (const auto& P : parts)
        if (P.codec) return false;
    // dictionary pages (few) in walk order: device index, entry base
    std::vector<size_t> dpos;  // walk index of each, ascending
    const int32_t d0 = static_cast<int32_t>(hdicts.size());
    for (const auto& P : parts)
        for (size_t i : P.dicts) {
            const pq_page_desc& p = w.pages[i];
            DevDict d{};
            d.size = p.payload_size;
            d.nvals = p.num_values;
            d.entry_base = static_cast<int32_t>(c->nentries);
            c->max_dict_bytes = std::max<uint32_t>(c->max_dict_bytes, static_cast<uint32_t>(std::max(p.payload_size, 0)));
            const int64_t cap = c->type == PQ_BYTE_ARRAY ? std::min<int64_t>(p.num_values, p.payload_size / 4 + 1) : 0;
            c->nentries += std::max<int64_t>(cap, 0);
            hdicts.push_back(d);
            c->dict_seq.push_back(seq + static_cast<int64_t>(i));
            dpos.push_back(i);
        }
    auto dict_dev = [&](int64_t walk_idx) -> int32_t {
        auto it = std::lower_bound(dpos.begin(), dpos.end(), static_cast<size_t>(walk_idx));
        return (walk_idx >= 0 && it != dpos.end() && *it == static_cast<size_t>(walk_idx))
                   ? d0 + static_cast<int32_t>(it - dpos.begin())
                   : -1;
    };
    // bases of each range
    std::vector<int64_t> img0(static_cast<size_t>(T)), slot0(static_cast<size_t>(T)), data0(static_cast<size_t>(T));
    int64_t ti = 0, ts = 0, td = 0, rows = 0;
    for (int t = 0; t < T; t++) {
        const Part& P = parts[static_cast<size_t>(t)];
        img0[static_cast<size_t>(t)] = ti;
        slot0[static_cast<size_t>(t)] = ts;
        data0[static_cast<size_t>(t)] = td;
        ti += P.bytes;
        ts += P.nslot;
        td += P.ndata;
        rows += P.rows;
        c->payload_bytes += P.payload;
    }
    const size_t cp0 = copies.size(), hp0 = hpages.size(), ps0 = c->page_seq.size(), wk0 = c->walked.size();
    copies.resize(cp0 + static_cast<size_t>(ts));
    copy_size.resize(cp0 + static_cast<size_t>(ts));
    hpages.resize(hp0 + static_cast<size_t>(td));
    c->page_seq.resize(ps0 + static_cast<size_t>(td));
    if (keep_walk) c->walked.resize(wk0 + N);
    const int64_t img_base = img, rb = row_base;
    pqfmt::parallel_run(T, T, [&](int t) {
        const size_t a = static_cast<size_t>(t) * per, b = std::min(N, a + per);
        int64_t at = img_base + img0[static_cast<size_t>(t)];
        size_t si = cp0 + static_cast<size_t>(slot0[static_cast<size_t>(t)]);
        size_t di = hp0 + static_cast<size_t>(data0[static_cast<size_t>(t)]);
        for (size_t i = a; i < b; i++) {
            pq_page_desc p = w.pages[i];
            if (p.page_type == PQ_DICTIONARY_PAGE || p.page_type == PQ_DATA_PAGE) {
                copies[si] = {p.payload_offset, at};
                copy_size[si] = p.payload_size;
                si++;
                if (p.page_type == PQ_DICTIONARY_PAGE) {
                    hdicts[static_cast<size_t>(dict_dev(static_cast<int64_t>(i)))].off = static_cast<uint64_t>(at);
                } else {
                    DevPage d{};
                    d.off = static_cast<uint64_t>(at);
                    d.size = p.payload_size;
                    d.nvals = p.num_values;
                    d.first_row = rb + p.first_row;
                    const int32_t dd = p.dict_page >= 0 ? dict_dev(p.dict_page) : -1;
                    const bool enc_dict = p.encoding == 2 || p.encoding == 8;
                    d.mode = (enc_dict && dd >= 0) ? pqk::MODE_DICT
                             : (c->type == PQ_BOOLEAN ? ((desc.ext_flags && p.encoding == 3) ? pqk::MODE_BOOL_RLE : pqk::MODE_BOOL)
                                                      : pqk::MODE_PLAIN);
                    d.dict = d.mode == pqk::MODE_DICT ? dd : -1;
                    c->page_seq[ps0 + (di - hp0)] = seq + static_cast<int64_t>(i);
                    hpages[di++] = d;
                }
                at += slot_bytes(p.payload_size);
            }
            if (keep_walk) {
                p.first_row += rb;
                c->walked[wk0 + i] = p;
            }
        }
    });
    img += ti;
    row_base += rows;
    return true;
}
// Windows of consecutive pages for the windowed PLAIN regex kernel (regex.hip
// k_regex_plain): <= 64 pages and <= win bytes of image each.  False when a
// page does not fit (the lane-per-page kernel runs then).
bool plan_regex_windows(pq_ctx* ctx, pq_chunk* c) {
    if (c->d_rwins && c->rwin_for_dfa == c->dfa_bytes && c->rwin_opt == ctx->opt_regex_win) return true;
    const uint32_t maxslot = c->npages ? (c->max_page_bytes + 15) / 16 * 16 + 16 : 0u;
    const uint32_t win = std::max<uint32_t>(static_cast<uint32_t>(ctx->opt_regex_win), maxslot);
    // the kernel lists strings by u16 window offsets (and the string index
    // keeps them): pages whose slot leaves no room take k_regex_lanes
    if (win + 32 > 65535u) return false;
    if (pqre::regex_plain_waves(c->dfa_bytes, win) == 0) return false;
    const uint32_t lds = pqre::regex_plain_lds(c->dfa_bytes, win);
    if (lds > 160 * 1024) return false;
    c->hrwins.clear();
    // the PLAIN decode's windows are the same kind (<= 64 consecutive page
    // slots, <= kPWin bytes; planned on host threads at upload): no page
    // table read back
    const bool same = c->plain && !c->plain_spec && win == pqk::kPWin && !c->hpwins.empty();
    std::vector<DevPage> hp(same ? 0 : static_cast<size_t>(c->npages));
    if (same) c->hrwins = c->hpwins;
    else if (c->npages && hipMemcpy(hp.data(), c->d_pages, hp.size() * sizeof(DevPage), hipMemcpyDeviceToHost) != hipSuccess)
        return false;
    size_t p = 0;
    while (p < hp.size()) {
        pqk::DevBatch b{};
        b.p0 = static_cast<int32_t>(p);
        b.img_lo = hp[p].off;
        uint64_t hi = b.img_lo;
        size_t q = p;
        while (q < hp.size() && q - p < 64) {
            const uint64_t e = hp[q].off + (static_cast<uint64_t>(std::max(hp[q].size, 0)) + 15) / 16 * 16 + 16;
            if (e - b.img_lo > win) break;
            hi = e;
            b.nrows += static_cast<uint32_t>(std::max(hp[q].nvals, 0));
            q++;
        }
        b.row0 = hp[p].first_row;
        b.np = static_cast<int32_t>(q - p);
        b.img_bytes = static_cast<uint32_t>(hi - b.img_lo);
        c->hrwins.push_back(b);
        p = q;
    }
    dfree(c->d_rwins);
    if (!c->d_rwin_ticket && dalloc(&c->d_rwin_ticket, 1)) return false;
    if (dalloc(&c->d_rwins, std::max<size_t>(c->hrwins.size(), 1))) return false;
    if (!c->hrwins.empty() &&
        hipMemcpy(c->d_rwins, c->hrwins.data(), c->hrwins.size() * sizeof(pqk::DevBatch), hipMemcpyHostToDevice) != hipSuccess)
        return false;
    const int cus = ctx->cus;
    const int per_cu = std::max(1, pqre::regex_plain_occupancy(lds));
    c->rwin_bytes = win;
    c->rwin_for_dfa = c->dfa_bytes;
    c->rwin_opt = ctx->opt_regex_win;
    const int scan = static_cast<int>(pqre::regex_plain_waves(c->dfa_bytes, win));  // waves per workgroup
    c->rwin_grid = std::max(1, std::min<int>(per_cu * cus, static_cast<int>((c->hrwins.size() + scan - 1) / scan)));
    (void)cus;
    return true;
}
}  // namespace pqcapi
