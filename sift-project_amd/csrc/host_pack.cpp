// host_pack.cpp — the front end's host pass over a reference Image buffer
// (HWC doubles, reference src/image_io.hh:22-26; stb decodes bytes into it,
// image_io.cpp:20-35): when every value is an integer 0..255 the image goes
// to the device as bytes (8x less PCIe traffic, converted back exactly on
// the device). One pass reads the doubles, checks that each survives the
// u8 round trip bit for bit and writes the bytes into pinned staging.
//
// The pass is memory-bound (8 B read + 1 B written per pixel), so it runs on
// a persistent pool of host threads (no thread creation per image) with an
// AVX2 body where the CPU has it.
#include <immintrin.h>

#include <algorithm>
#include <cmath>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "sift_host.h"

namespace sift_amd {
namespace {

// scalar reference of the check: the byte's double has the same bits as v
// (rejects fractions, out-of-range values, NaN and -0.0)
bool pack_scalar(const double* src, size_t n, uint8_t* dst) {
    bool ok = true;
    for (size_t i = 0; i < n; ++i) {
        const double v = src[i];
        const uint8_t u = (v >= 0.0 && v <= 255.0) ? (uint8_t)v : 0;
        const double back = (double)u;
        uint64_t a, b;
        std::memcpy(&a, &v, 8);
        std::memcpy(&b, &back, 8);
        ok &= a == b;
        dst[i] = u;
    }
    return ok;
}

__attribute__((target("avx2"))) bool pack_avx2(const double* src, size_t n, uint8_t* dst) {
    size_t i = 0;
    __m256i bad = _mm256_setzero_si256();
    const __m128i lim = _mm_set1_epi32(255);
    for (; i + 16 <= n; i += 16) {
        __m128i q[4];
        for (int k = 0; k < 4; ++k) {
            const __m256d v = _mm256_loadu_pd(src + i + 4 * k);
            const __m128i t = _mm256_cvttpd_epi32(v);  // out of range: 0x80000000
            // 0..255 and bit-identical after the round trip: the converted
            // value compares equal and no sign bit is set (-0.0, negatives)
            const __m256d back = _mm256_cvtepi32_pd(t);
            const __m256d ne = _mm256_cmp_pd(back, v, _CMP_NEQ_UQ);
            const __m256i sign = _mm256_castpd_si256(v);
            bad = _mm256_or_si256(bad, _mm256_castpd_si256(ne));
            bad = _mm256_or_si256(bad, _mm256_srai_epi32(sign, 31));
            bad = _mm256_or_si256(bad, _mm256_castsi128_si256(_mm_cmpgt_epi32(t, lim)));
            q[k] = t;
        }
        const __m128i w01 = _mm_packus_epi32(q[0], q[1]);
        const __m128i w23 = _mm_packus_epi32(q[2], q[3]);
        _mm_storeu_si128(reinterpret_cast<__m128i*>(dst + i), _mm_packus_epi16(w01, w23));
    }
    const bool ok = _mm256_testz_si256(bad, bad);
    return pack_scalar(src + i, n - i, dst + i) && ok;
}

bool pack_range(const double* src, size_t n, uint8_t* dst) {
    static const bool avx2 = __builtin_cpu_supports("avx2");
    return avx2 ? pack_avx2(src, n, dst) : pack_scalar(src, n, dst);
}

// Persistent worker threads: run(n_tasks, fn) calls fn(t) for every task,
// the caller included, and returns when all are done. One caller at a time;
// a concurrent caller (another context on another thread) runs its tasks
// itself.
class Pool {
public:
    Pool() {
        const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
        const unsigned n = std::min(7u, hw > 1 ? hw - 1 : 0u);
        for (unsigned k = 0; k < n; ++k) workers_.emplace_back([this] { loop(); });
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : workers_) t.join();
    }
    unsigned threads() const { return (unsigned)workers_.size() + 1; }
    void run(unsigned n_tasks, const std::function<void(unsigned)>& fn) {
        std::unique_lock<std::mutex> busy(run_m_, std::try_to_lock);
        if (!busy.owns_lock() || workers_.empty()) {
            for (unsigned t = 0; t < n_tasks; ++t) fn(t);
            return;
        }
        unsigned gen;
        {
            std::lock_guard<std::mutex> g(m_);
            gen = ++gen_;
            fn_ = &fn;
            n_tasks_ = n_tasks;
            pending_ = n_tasks;
            claim_.store((uint64_t)gen << 32);
        }
        cv_.notify_all();
        work(gen, n_tasks, &fn);
        std::unique_lock<std::mutex> g(m_);
        done_cv_.wait(g, [this] { return pending_ == 0; });
        fn_ = nullptr;
    }

private:
    // Claims carry the generation: claim_ = gen << 32 | next task index, and
    // a task is taken only by a compare-exchange that still sees the
    // worker's own generation. A worker that wakes late (its generation
    // already finished and the next one posted) fails the exchange and
    // returns, so it never runs, or counts down, another generation's task.
    void work(unsigned gen, unsigned n_tasks, const std::function<void(unsigned)>* fn) {
        for (;;) {
            uint64_t c = claim_.load();
            unsigned t;
            do {
                if ((unsigned)(c >> 32) != gen) return;
                t = (unsigned)c;
                if (t >= n_tasks) return;
            } while (!claim_.compare_exchange_weak(c, c + 1));
            (*fn)(t);
            std::lock_guard<std::mutex> g(m_);
            if (--pending_ == 0) done_cv_.notify_all();
        }
    }
    void loop() {
        unsigned seen = 0;
        for (;;) {
            unsigned gen, n;
            const std::function<void(unsigned)>* fn;
            {
                std::unique_lock<std::mutex> g(m_);
                cv_.wait(g, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen = gen_;
                n = n_tasks_;
                fn = fn_;
            }
            work(gen, n, fn);
        }
    }
    std::vector<std::thread> workers_;
    std::mutex m_, run_m_;
    std::condition_variable cv_, done_cv_;
    const std::function<void(unsigned)>* fn_ = nullptr;  // guarded by m_
    unsigned pending_ = 0, gen_ = 0, n_tasks_ = 0;       // guarded by m_
    std::atomic<uint64_t> claim_{0};
    bool stop_ = false;
};

Pool& pool() {
    static Pool p;
    return p;
}

}  // namespace

bool host_pack_u8(const double* src, size_t n, uint8_t* dst) {
    const size_t kChunk = (size_t)1 << 17;  // 1 MiB of doubles per task
    if (n <= kChunk) return pack_range(src, n, dst);
    const unsigned tasks = (unsigned)((n + kChunk - 1) / kChunk);
    std::vector<char> ok(tasks, 1);
    pool().run(tasks, [&](unsigned t) {
        const size_t b = (size_t)t * kChunk, e = std::min(n, b + kChunk);
        ok[t] = pack_range(src + b, e - b, dst + b);
    });
    for (char c : ok)
        if (!c) return false;
    return true;
}

bool host_copy_finite(const double* src, size_t n, double* dst) {
    const size_t kChunk = (size_t)1 << 17;
    const unsigned tasks = (unsigned)((n + kChunk - 1) / kChunk);
    std::vector<char> ok(std::max(tasks, 1u), 1);
    auto part = [&](unsigned t) {
        const size_t b = (size_t)t * kChunk, e = std::min(n, b + kChunk);
        std::memcpy(dst + b, src + b, (e - b) * sizeof(double));
        bool fin = true;
        for (size_t i = b; i < e; ++i) fin &= std::isfinite(src[i]);
        ok[t] = fin;
    };
    if (tasks <= 1) {
        if (n) part(0);
    } else {
        pool().run(tasks, part);
    }
    for (char c : ok)
        if (!c) return false;
    return true;
}

void host_parallel(unsigned n_tasks, const std::function<void(unsigned)>& fn) {
    pool().run(n_tasks, fn);
}

}  // namespace sift_amd
