// tdt_copypool.h — host threads for the host pipeline's staging copies (host code only).
//
// A pageable caller buffer reaches the GPU through pinned staging: one thread's memcpy moves
// ~10 GB/s, well below what PCIe takes, so large copies are split over a small pool of
// threads (the caller's thread takes a share too).  Copies below kParMin run inline.
#pragma once

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#if defined(__x86_64__) && !defined(__HIP_DEVICE_COMPILE__)
#include <immintrin.h>
// Large copies into the pinned staging (and out of it into the caller's buffer) stream past
// the caches: 32-byte non-temporal stores, no read-for-ownership of the destination.
__attribute__((target("avx2"))) inline void nt_copy_avx2(uint8_t *d, const uint8_t *s, size_t n) {
    size_t head = (32 - ((uintptr_t)d & 31)) & 31;
    if (head > n) head = n;
    std::memcpy(d, s, head);
    d += head;
    s += head;
    n -= head;
    size_t i = 0;
    for (; i + 128 <= n; i += 128) {
        const __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(s + i));
        const __m256i b = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(s + i + 32));
        const __m256i c = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(s + i + 64));
        const __m256i e = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(s + i + 96));
        _mm256_stream_si256(reinterpret_cast<__m256i *>(d + i), a);
        _mm256_stream_si256(reinterpret_cast<__m256i *>(d + i + 32), b);
        _mm256_stream_si256(reinterpret_cast<__m256i *>(d + i + 64), c);
        _mm256_stream_si256(reinterpret_cast<__m256i *>(d + i + 96), e);
    }
    std::memcpy(d + i, s + i, n - i);
    _mm_sfence();
}
inline void part_copy(uint8_t *d, const uint8_t *s, size_t n) {
    static const bool avx2 = __builtin_cpu_supports("avx2");
    if (avx2) nt_copy_avx2(d, s, n);
    else std::memcpy(d, s, n);
}
#else
inline void part_copy(uint8_t *d, const uint8_t *s, size_t n) { std::memcpy(d, s, n); }
#endif

class CopyPool {
  public:
    explicit CopyPool(int threads) {
        const int n = std::max(0, threads - 1);  // the caller copies a share itself
        for (int i = 0; i < n; ++i) th_.emplace_back([this] { work(); });
    }
    ~CopyPool() {
        {
            std::lock_guard<std::mutex> lk(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto &t : th_) t.join();
    }
    CopyPool(const CopyPool &) = delete;
    CopyPool &operator=(const CopyPool &) = delete;

    // dst[0, bytes) = src[0, bytes); returns when every part is copied.  Thread-safe: the pool
    // runs one job at a time (job_ is shared), so concurrent callers take turns.
    void copy(void *dst, const void *src, size_t bytes) {
        if (bytes < kParMin || th_.empty()) {
            std::memcpy(dst, src, bytes);
            return;
        }
        std::lock_guard<std::mutex> one(call_);
        auto job = std::make_shared<Job>();
        job->d = static_cast<uint8_t *>(dst);
        job->s = static_cast<const uint8_t *>(src);
        job->bytes = bytes;
        job->parts = std::min<size_t>(bytes / kPart + 1, 4 * (th_.size() + 1));
        submit(job);
    }

    // Gather: dst = msgs[0][0 .. sizes[0]) ++ msgs[1][...] ++ ... (n messages back to back).
    // Messages are grouped into pieces of about kPart bytes (a large message is split).
    void gather(void *dst, const uint8_t *const *msgs, const uint64_t *sizes, size_t n) {
        uint64_t total = 0;
        for (size_t i = 0; i < n; ++i) total += sizes[i];
        if (total < kParMin || th_.empty()) {
            uint8_t *d = static_cast<uint8_t *>(dst);
            for (size_t i = 0; i < n; ++i) {
                std::memcpy(d, msgs[i], sizes[i]);
                d += sizes[i];
            }
            return;
        }
        std::lock_guard<std::mutex> one(call_);
        auto job = std::make_shared<Job>();
        uint8_t *d = static_cast<uint8_t *>(dst);
        size_t k = 0;  // first message of the open piece
        uint64_t acc = 0;
        for (size_t i = 0; i < n; ++i) {
            if (sizes[i] >= kPart) {  // a large message: its own pieces
                if (i > k) job->pieces.push_back({d - acc, nullptr, acc, k, i});
                for (uint64_t o = 0; o < sizes[i]; o += kPart)
                    job->pieces.push_back({d + o, msgs[i] + o, std::min<uint64_t>(kPart, sizes[i] - o), 0, 0});
                d += sizes[i];
                acc = 0;
                k = i + 1;
                continue;
            }
            d += sizes[i];
            acc += sizes[i];
            if (acc >= kPart) {
                job->pieces.push_back({d - acc, nullptr, acc, k, i + 1});
                acc = 0;
                k = i + 1;
            }
        }
        if (k < n) job->pieces.push_back({d - acc, nullptr, acc, k, n});
        job->msgs = msgs;
        job->sizes = sizes;
        job->parts = job->pieces.size();
        submit(job);
    }

  private:
    static constexpr size_t kParMin = 1u << 20, kPart = 2u << 20;
    // one copy call; a worker that wakes late holds a finished job and finds no part left
    // a gather piece: bytes [d, d + len) from src (one message's part), or from messages
    // [m0, m1) back to back (src null)
    struct Piece {
        uint8_t *d;
        const uint8_t *src;
        uint64_t len;
        size_t m0, m1;
    };
    struct Job {
        uint8_t *d = nullptr;
        const uint8_t *s = nullptr;
        size_t bytes = 0, parts = 0;
        std::vector<Piece> pieces;  // gather jobs
        const uint8_t *const *msgs = nullptr;
        const uint64_t *sizes = nullptr;
        std::atomic<size_t> next{0}, left{0};
    };

    void submit(const std::shared_ptr<Job> &job) {
        job->left.store(job->parts);
        {
            std::lock_guard<std::mutex> lk(m_);
            job_ = job;
            ++gen_;
        }
        cv_.notify_all();
        run(*job);
        std::unique_lock<std::mutex> lk(m_);
        done_.wait(lk, [&] { return job->left.load() == 0; });
        job_.reset();
    }

    void run(Job &j) {
        const size_t per = j.pieces.empty() ? (j.bytes + j.parts - 1) / j.parts : 0;
        for (;;) {
            const size_t i = j.next.fetch_add(1);
            if (i >= j.parts) return;
            if (!j.pieces.empty()) {
                const Piece &p = j.pieces[i];
                if (p.src) {
                    part_copy(p.d, p.src, p.len);
                } else {
                    uint8_t *d = p.d;
                    for (size_t m = p.m0; m < p.m1; ++m) {
                        std::memcpy(d, j.msgs[m], j.sizes[m]);
                        d += j.sizes[m];
                    }
                }
            } else {
                const size_t b = i * per, e = std::min(j.bytes, b + per);
                if (b < e) part_copy(j.d + b, j.s + b, e - b);
            }
            if (j.left.fetch_sub(1) == 1) {
                std::lock_guard<std::mutex> lk(m_);
                done_.notify_all();
            }
        }
    }
    void work() {
        uint64_t seen = 0;
        for (;;) {
            std::shared_ptr<Job> j;
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
                j = job_;
            }
            if (j) run(*j);
        }
    }

    std::vector<std::thread> th_;
    std::mutex call_;  // one copy() at a time
    std::mutex m_;
    std::condition_variable cv_, done_;
    bool stop_ = false;
    uint64_t gen_ = 0;
    std::shared_ptr<Job> job_;
};
