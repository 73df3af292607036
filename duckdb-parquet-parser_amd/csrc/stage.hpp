// stage.hpp — pinned, multi-buffered host→HBM staging.
//
// Replaces the reference's ReadRangeFunc / ifstream byte supply
// (include/reader/column_reader.hpp:10, src/reader/parquet_reader.cpp:173-178)
// on the way into HBM.  A transfer of n bytes is cut into pieces of kPiece
// bytes; host threads take pieces in order, fill a pinned buffer of the ring
// (the caller's fill function writes the piece's bytes: payload copies, zero
// padding) and queue its hipMemcpyAsync on the context's copy stream, so the
// fill of piece i+1.. overlaps the DMA of piece i.  A buffer is refilled only
// after the event recorded behind its previous copy has completed.  Pageable
// copies would go through the runtime's own bounce buffer at a fraction of
// PCIe bandwidth and serialise with the fill.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <mutex>
#include <thread>
#include <vector>

namespace pqstage {

constexpr int kMaxBufs = 16;

class Stager {
public:
    ~Stager() { release(); }

    // Ring shape (pq_ctx_set_option "stage_bufs" / "stage_piece_kb"); takes
    // effect at the next upload.
    void configure(int bufs, size_t piece) {
        release();
        bufs_ = std::max(2, std::min(kMaxBufs, bufs));
        piece_ = std::max<size_t>(64u << 10, piece);
    }
    size_t piece() const { return piece_; }
    double fill_ms = 0, wait_ms = 0;  // last upload: summed fill time over threads, final sync wait

    void release() {
        for (int b = 0; b < kMaxBufs; b++) {
            if (ev_[b]) (void)hipEventSynchronize(ev_[b]);
            if (buf_[b]) (void)hipHostFree(buf_[b]);
            if (ev_[b]) (void)hipEventDestroy(ev_[b]);
            buf_[b] = nullptr;
            ev_[b] = nullptr;
        }
    }

    // fill(dst, a, b): write bytes [a, b) of the transfer to dst (b - a <= kPiece).
    // Returns a hipError_t; the copies are complete when it returns.
    template <class Fill>
    hipError_t upload(uint8_t* d_dst, size_t n, hipStream_t stream, int threads, Fill&& fill,
                      hipStream_t stream2 = nullptr) {
        if (n == 0) return hipSuccess;
        hipError_t e = ensure();
        if (e != hipSuccess) return e;
        const size_t kPiece = piece_;
        const int kBufs = bufs_;
        const size_t npieces = (n + kPiece - 1) / kPiece;
        std::atomic<int64_t> fill_ns{0};
        threads = static_cast<int>(std::max<size_t>(1, std::min<size_t>(static_cast<size_t>(threads), npieces)));
        std::atomic<size_t> next{0};
        std::atomic<int> err{hipSuccess};
        std::mutex m;
        std::condition_variable cv;
        size_t queued = 0;  // pieces whose copy is queued, in order (a buffer's previous use is queued first)
        auto worker = [&]() {
            for (size_t i = next.fetch_add(1); i < npieces; i = next.fetch_add(1)) {
                const int b = static_cast<int>(i % kBufs);
                {   // the previous piece on this buffer must have queued its copy
                    std::unique_lock<std::mutex> lk(m);
                    cv.wait(lk, [&] { return queued + static_cast<size_t>(kBufs) > i || err.load() != hipSuccess; });
                }
                if (err.load() != hipSuccess) return;
                if (i >= static_cast<size_t>(kBufs)) (void)hipEventSynchronize(ev_[b]);
                const size_t a = i * kPiece, z = std::min(n, a + kPiece);
                auto f0 = std::chrono::steady_clock::now();
                fill(buf_[b], a, z);
                fill_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - f0).count();
                std::unique_lock<std::mutex> lk(m);
                cv.wait(lk, [&] { return queued == i || err.load() != hipSuccess; });  // copies queue in order
                hipStream_t st = (stream2 && (i & 1)) ? stream2 : stream;  // two DMA queues
                hipError_t r = hipMemcpyAsync(d_dst + a, buf_[b], z - a, hipMemcpyHostToDevice, st);
                if (r == hipSuccess) r = hipEventRecord(ev_[b], st);
                if (r != hipSuccess) err.store(r);
                queued++;
                cv.notify_all();
            }
        };
        std::vector<std::thread> th;
        for (int t = 1; t < threads; t++) th.emplace_back(worker);
        worker();
        for (auto& x : th) x.join();
        if (err.load() != hipSuccess) return static_cast<hipError_t>(err.load());
        auto w0 = std::chrono::steady_clock::now();
        hipError_t e2 = hipStreamSynchronize(stream);
        if (e2 == hipSuccess && stream2) e2 = hipStreamSynchronize(stream2);
        wait_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - w0).count();
        fill_ms = static_cast<double>(fill_ns.load()) * 1e-6;
        return e2;
    }

    // The reverse direction: n bytes from HBM at d_src in pieces through the
    // ring; sink(src, a, b) consumes bytes [a, b) from the pinned buffer src
    // (b - a <= the piece) on one of `threads` host threads, and the thread
    // that drained a buffer queues the next piece into it.  Returns when every
    // piece is consumed.
    template <class Sink>
    hipError_t download(const uint8_t* d_src, size_t n, hipStream_t stream, int threads, Sink&& sink) {
        if (n == 0) return hipSuccess;
        hipError_t e = ensure();
        if (e != hipSuccess) return e;
        const size_t kPiece = piece_;
        const size_t kBufs = static_cast<size_t>(bufs_);
        const size_t npieces = (n + kPiece - 1) / kPiece;
        std::mutex m;
        std::condition_variable cv;
        std::vector<char> queued(npieces, 0);
        std::atomic<int> err{hipSuccess};
        auto queue = [&](size_t i) {  // (under m)
            const size_t a = i * kPiece, z = std::min(n, a + kPiece);
            hipError_t r = hipMemcpyAsync(buf_[i % kBufs], d_src + a, z - a, hipMemcpyDeviceToHost, stream);
            if (r == hipSuccess) r = hipEventRecord(ev_[i % kBufs], stream);
            if (r != hipSuccess) err.store(r);
            queued[i] = 1;
        };
        {
            std::lock_guard<std::mutex> lk(m);
            for (size_t i = 0; i < std::min(kBufs, npieces); i++) queue(i);
        }
        std::atomic<size_t> next{0};
        auto worker = [&]() {
            for (size_t i = next.fetch_add(1); i < npieces; i = next.fetch_add(1)) {
                {
                    std::unique_lock<std::mutex> lk(m);
                    cv.wait(lk, [&] { return queued[i] != 0 || err.load() != hipSuccess; });
                }
                if (err.load() != hipSuccess) return;
                const int b = static_cast<int>(i % kBufs);
                hipError_t r = hipEventSynchronize(ev_[b]);
                if (r != hipSuccess) { err.store(r); cv.notify_all(); return; }
                const size_t a = i * kPiece, z = std::min(n, a + kPiece);
                sink(buf_[b], a, z);
                std::lock_guard<std::mutex> lk(m);
                if (i + kBufs < npieces) queue(i + kBufs);
                cv.notify_all();
            }
        };
        threads = static_cast<int>(std::max<size_t>(1, std::min<size_t>(static_cast<size_t>(threads), npieces)));
        std::vector<std::thread> th;
        for (int t = 1; t < threads; t++) th.emplace_back(worker);
        worker();
        for (auto& x : th) x.join();
        return static_cast<hipError_t>(err.load());
    }

private:
    hipError_t ensure() {
        for (int b = 0; b < bufs_; b++) {
            if (buf_[b]) continue;
            hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&buf_[b]), piece_, hipHostMallocDefault);
            if (e != hipSuccess) { buf_[b] = nullptr; return e; }
            e = hipEventCreateWithFlags(&ev_[b], hipEventDisableTiming);
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
    int bufs_ = 6;
    size_t piece_ = 8u << 20;
    uint8_t* buf_[kMaxBufs] = {};
    hipEvent_t ev_[kMaxBufs] = {};
};

}  // namespace pqstage
