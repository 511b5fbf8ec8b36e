// hostcopy.cpp -- parallel host memory copies for the ingest pipeline
// (tlsgpu/ingest.py; tlsgpu.h tg_host_copy / tg_host_copy_rows).
//
// The record pipeline's host side moves every byte of application data and
// wire records between the caller's buffers and pinned staging once
// (RecordSocket.recv / send, recordlayer.py:80-237, copy socket bytes the
// same way).  One core copies 13-20 GiB/s into pinned memory
// (profiles/r05/final/bench_ingest.json), well below the PCIe rate the
// staging feeds, so a copy is split into row ranges over a small pool of
// worker threads; the calling thread takes one range itself.  Callers from
// several threads share the pool (each call waits only for its own ranges).
// Plain C++ (no HIP): built by g++ into the library and, under
// AddressSanitizer + UBSan, into tests/native/host_check.cpp.
#include "host.h"

#include <string.h>

#include <algorithm>
#include <condition_variable>
#include <deque>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace tg {
namespace host {
namespace {

struct Call {
    std::mutex mu;
    std::condition_variable cv;
    int left = 0;
};

struct Task {
    std::function<void()> fn;
    Call* call;
};

class Pool {
  public:
    // grows to ``n`` workers (never shrinks; at most kMaxWorkers)
    void ensure(int n) {
        std::lock_guard<std::mutex> g(mu_);
        while ((int)workers_.size() < n && (int)workers_.size() < kMaxWorkers)
            workers_.emplace_back([this] { loop(); });
    }
    void post(Task t) {
        {
            std::lock_guard<std::mutex> g(mu_);
            q_.push_back(std::move(t));
        }
        cv_.notify_one();
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& w : workers_) w.join();
    }
    static constexpr int kMaxWorkers = 31;

  private:
    void loop() {
        for (;;) {
            Task t;
            {
                std::unique_lock<std::mutex> g(mu_);
                cv_.wait(g, [this] { return stop_ || !q_.empty(); });
                if (q_.empty()) return;   // stop_ with nothing left
                t = std::move(q_.front());
                q_.pop_front();
            }
            t.fn();
            std::lock_guard<std::mutex> g(t.call->mu);
            if (--t.call->left == 0) t.call->cv.notify_all();
        }
    }
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<Task> q_;
    std::vector<std::thread> workers_;
    bool stop_ = false;
};

Pool& pool() {
    static Pool p;
    return p;
}

// Ranges below this many bytes are not worth a thread hand-off.
constexpr size_t kMinChunk = 1u << 20;

}  // namespace

int copy_threads_default() {
    const unsigned hc = std::thread::hardware_concurrency();
    return (int)std::max(1u, std::min(8u, hc ? hc : 1u));
}

void parallel_copy_rows(uint8_t* dst, size_t dst_stride, const uint8_t* src, size_t src_stride, size_t row,
                        size_t rows, int nthreads) {
    if (!rows || !row) return;
    if (nthreads <= 0) nthreads = copy_threads_default();
    nthreads = std::min(nthreads, Pool::kMaxWorkers + 1);
    const size_t total = row * rows;
    size_t parts = std::min((size_t)nthreads, std::max<size_t>(1, total / kMinChunk));
    parts = std::min(parts, rows == 1 ? total / 4096 + 1 : rows);
    auto copy_range = [=](size_t r0, size_t r1) {
        if (rows == 1) {   // one row: split it by bytes
            memcpy(dst + r0, src + r0, r1 - r0);
            return;
        }
        if (dst_stride == row && src_stride == row) {
            memcpy(dst + r0 * row, src + r0 * row, (r1 - r0) * row);
            return;
        }
        for (size_t r = r0; r < r1; ++r) memcpy(dst + r * dst_stride, src + r * src_stride, row);
    };
    const size_t units = rows == 1 ? row : rows;
    if (parts <= 1) {
        copy_range(0, units);
        return;
    }
    pool().ensure((int)parts - 1);
    Call call;
    call.left = (int)parts - 1;
    // unit ranges; one-row copies split at 4 KiB boundaries
    auto bound = [&](size_t k) {
        size_t b = units * k / parts;
        if (rows == 1 && k != parts) b &= ~(size_t)4095;
        return b;
    };
    for (size_t k = 1; k < parts; ++k) {
        const size_t a = bound(k), b = bound(k + 1);
        pool().post(Task{[=] { copy_range(a, b); }, &call});
    }
    copy_range(0, bound(1));
    std::unique_lock<std::mutex> g(call.mu);
    call.cv.wait(g, [&] { return call.left == 0; });
}

void parallel_copy(void* dst, const void* src, size_t bytes, int nthreads) {
    parallel_copy_rows(static_cast<uint8_t*>(dst), bytes, static_cast<const uint8_t*>(src), bytes, bytes, 1,
                       nthreads);
}

}  // namespace host
}  // namespace tg
