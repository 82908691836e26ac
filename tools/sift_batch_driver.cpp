// sift_batch_driver.cpp — BASELINE config 4 as a plain C++ program over the
// C-ABI (no torch): a batch of synthetic 1920x1080-class images sharded one
// image per GPU (image i -> GPU i % n_gpus), each GPU driven by
// its own host thread (sift_hip_submit / sift_hip_wait /
// sift_hip_fetch_device into HBM), then the native RCCL exchange
// (sift_hip_comm_init_all + sift_hip_allgather_records) so that every GPU
// holds every image's final records. Rank 0 prints one JSON line: per-image
// record counts (global image order), the 64-bit word sum of the exchanged
// buffer (rank-major) and the wall times.
//
//   sift_batch_driver <n_images> [width=1920] [height=1080] [n_gpus=all]
//
// Built by __graft_entry__.build(); tests/test_gpu_comm.py runs it. This is
// the C++ caller INTEGRATION.md shows.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "../include/sift_hip.h"

namespace {

struct Rank {
    int device = 0;
    std::vector<int64_t> ids;      // global image indices of this rank
    std::vector<size_t> counts;    // records per local image
    sift_kp* d_recs = nullptr;     // local records, image-major
    sift_kp* d_all = nullptr;      // every rank's records after the exchange
    size_t cap_all = 0, n_all = 0;
    std::vector<int64_t> all_ids;
    std::vector<size_t> all_counts;
    int status = SIFT_OK;
    double ms_detect = 0, ms_exchange = 0;
};

#define CHECK(expr)                                                               \
    do {                                                                          \
        const int st_ = (expr);                                                   \
        if (st_ != SIFT_OK) {                                                     \
            std::fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #expr,   \
                         sift_hip_strerror(st_));                                 \
            return st_;                                                           \
        }                                                                         \
    } while (0)

// detect this rank's images (one job each, two in flight), records to HBM
int detect_local(Rank& r, int w, int h) {
    using clk = std::chrono::steady_clock;
    if (hipSetDevice(r.device) != hipSuccess) return SIFT_ERR_HIP;
    sift_ctx* ctx = nullptr;
    CHECK(sift_hip_create(r.device, &ctx));
    std::vector<std::vector<double>> imgs(r.ids.size());
    for (size_t j = 0; j < r.ids.size(); ++j) {
        imgs[j].resize((size_t)w * h);
        CHECK(sift_synth_image(w, h, 1, (int64_t)w * h / 52, 6.0, 42 + (uint64_t)r.ids[j],
                               imgs[j].data()));
    }
    sift_params p;
    sift_params_default(&p);
    const auto t0 = clk::now();
    std::vector<int> tickets(r.ids.size());
    size_t cap = 0;
    std::vector<sift_kp*> parts;
    for (size_t j = 0; j < r.ids.size(); ++j) {
        const void* img = imgs[j].data();
        CHECK(sift_hip_submit(ctx, &img, 1, SIFT_INPUT_F64_HOST, w, h, 1, &p, 0, &tickets[j]));
        if (j == 0) continue;
        // job j-1 finishes while job j runs
        size_t n = 0;
        CHECK(sift_hip_wait(ctx, tickets[j - 1], nullptr, &n));
        r.counts.push_back(n);
        sift_kp* d = nullptr;
        if (hipMalloc(&d, std::max<size_t>(n, 1) * sizeof(sift_kp)) != hipSuccess)
            return SIFT_ERR_NOMEM;
        CHECK(sift_hip_fetch_device(ctx, tickets[j - 1], d, n));
        parts.push_back(d);
    }
    if (!r.ids.empty()) {
        size_t n = 0;
        CHECK(sift_hip_wait(ctx, tickets.back(), nullptr, &n));
        r.counts.push_back(n);
        sift_kp* d = nullptr;
        if (hipMalloc(&d, std::max<size_t>(n, 1) * sizeof(sift_kp)) != hipSuccess)
            return SIFT_ERR_NOMEM;
        CHECK(sift_hip_fetch_device(ctx, tickets.back(), d, n));
        parts.push_back(d);
    }
    for (size_t n : r.counts) cap += n;
    if (hipMalloc(&r.d_recs, std::max<size_t>(cap, 1) * sizeof(sift_kp)) != hipSuccess)
        return SIFT_ERR_NOMEM;
    size_t off = 0;
    for (size_t j = 0; j < parts.size(); ++j) {
        if (r.counts[j] &&
            hipMemcpy(r.d_recs + off, parts[j], r.counts[j] * sizeof(sift_kp),
                      hipMemcpyDeviceToDevice) != hipSuccess)
            return SIFT_ERR_HIP;
        off += r.counts[j];
        (void)hipFree(parts[j]);
    }
    r.ms_detect = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
    CHECK(sift_hip_destroy(ctx));
    return SIFT_OK;
}

int exchange(Rank& r, sift_comm* comm, int max_local, int n_ranks) {
    using clk = std::chrono::steady_clock;
    if (hipSetDevice(r.device) != hipSuccess) return SIFT_ERR_HIP;
    r.all_ids.resize((size_t)n_ranks * max_local);
    r.all_counts.resize((size_t)n_ranks * max_local);
    const auto t0 = clk::now();
    // capacity: first call with cap 0 learns the total (the collective runs
    // on every rank either way), then the real exchange
    int st = sift_hip_allgather_records(comm, r.d_recs, r.ids.data(), r.counts.data(),
                                        (int)r.ids.size(), max_local, nullptr, 0,
                                        r.all_ids.data(), r.all_counts.data(), &r.n_all,
                                        nullptr);
    if (st != SIFT_OK && st != SIFT_ERR_ARG) return st;
    r.cap_all = r.n_all;
    // an allocation failure still joins the second exchange (with no output
    // room: it returns SIFT_ERR_ARG once the collectives are done), so no
    // peer is left waiting in it
    int alloc = SIFT_OK;
    if (hipMalloc(&r.d_all, std::max<size_t>(r.cap_all, 1) * sizeof(sift_kp)) != hipSuccess) {
        r.d_all = nullptr;
        r.cap_all = 0;
        alloc = SIFT_ERR_NOMEM;
    }
    st = sift_hip_allgather_records(comm, r.d_recs, r.ids.data(), r.counts.data(),
                                    (int)r.ids.size(), max_local, r.d_all, r.cap_all,
                                    r.all_ids.data(), r.all_counts.data(), &r.n_all, nullptr);
    if (alloc != SIFT_OK) return alloc;
    CHECK(st);
    r.ms_exchange = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
    return SIFT_OK;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s <n_images> [width height] [n_gpus]\n", argv[0]);
        return 2;
    }
    const int n_images = std::atoi(argv[1]);
    const int w = argc > 3 ? std::atoi(argv[2]) : 1920, h = argc > 3 ? std::atoi(argv[3]) : 1080;
    int n_dev = 0;
    if (hipGetDeviceCount(&n_dev) != hipSuccess || n_dev < 1) {
        std::fprintf(stderr, "no HIP device\n");
        return 1;
    }
    const int n_gpus = argc > 4 ? std::min(std::atoi(argv[4]), n_dev) : n_dev;
    std::vector<Rank> ranks(n_gpus);
    int max_local = 1;
    for (int g = 0; g < n_gpus; ++g) {
        ranks[g].device = g;
        for (int i = g; i < n_images; i += n_gpus) ranks[g].ids.push_back(i);
        max_local = std::max(max_local, (int)ranks[g].ids.size());
    }
    std::vector<int> devs(n_gpus);
    for (int g = 0; g < n_gpus; ++g) devs[g] = g;
    std::vector<sift_comm*> comms(n_gpus, nullptr);
    int st = sift_hip_comm_init_all(n_gpus, devs.data(), comms.data());
    if (st != SIFT_OK) {
        std::fprintf(stderr, "sift_hip_comm_init_all: %s\n", sift_hip_strerror(st));
        return 1;
    }
    // one host thread per GPU: detect, then the collective (every rank must
    // enter it concurrently)
    std::vector<std::thread> th;
    for (int g = 0; g < n_gpus; ++g)
        th.emplace_back([&, g] {
            Rank& r = ranks[g];
            r.status = detect_local(r, w, h);
            // a rank that failed still joins the exchange with no images,
            // so the others are not left waiting
            if (r.status != SIFT_OK) {
                r.ids.clear();
                r.counts.clear();
            }
            const int e = exchange(r, comms[g], max_local, n_gpus);
            if (r.status == SIFT_OK) r.status = e;
        });
    for (auto& t : th) t.join();
    int rc = 0;
    for (int g = 0; g < n_gpus; ++g)
        if (ranks[g].status != SIFT_OK) {
            std::fprintf(stderr, "rank %d: %s\n", g, sift_hip_strerror(ranks[g].status));
            rc = 1;
        }
    // rank 0's view: counts in global image order, checksum of its buffer
    Rank& r0 = ranks[0];
    std::vector<long long> per_image(n_images, -1);
    for (size_t k = 0; k < r0.all_ids.size(); ++k)
        if (r0.all_ids[k] >= 0 && r0.all_ids[k] < n_images)
            per_image[r0.all_ids[k]] = (long long)r0.all_counts[k];
    std::vector<uint64_t> words(r0.n_all * sizeof(sift_kp) / 8);
    if (rc == 0 && r0.n_all) {
        (void)hipSetDevice(r0.device);
        if (hipMemcpy(words.data(), r0.d_all, r0.n_all * sizeof(sift_kp),
                      hipMemcpyDeviceToHost) != hipSuccess)
            rc = 1;
    }
    uint64_t sum = 0;
    for (uint64_t v : words) sum += v;
    // every rank received the same bytes
    for (int g = 1; g < n_gpus && rc == 0; ++g) {
        std::vector<uint64_t> other(ranks[g].n_all * sizeof(sift_kp) / 8);
        (void)hipSetDevice(ranks[g].device);
        if (ranks[g].n_all != r0.n_all ||
            hipMemcpy(other.data(), ranks[g].d_all, ranks[g].n_all * sizeof(sift_kp),
                      hipMemcpyDeviceToHost) != hipSuccess ||
            other != words)
            rc = 1;
    }
    std::printf("{\"images\": %d, \"gpus\": %d, \"total\": %zu, \"checksum\": %llu, "
                "\"ranks_agree\": %s, \"counts\": [",
                n_images, n_gpus, r0.n_all, (unsigned long long)sum, rc == 0 ? "true" : "false");
    for (int i = 0; i < n_images; ++i) std::printf("%s%lld", i ? ", " : "", per_image[i]);
    double md = 0, mx = 0;
    for (auto& r : ranks) {
        md = std::max(md, r.ms_detect);
        mx = std::max(mx, r.ms_exchange);
    }
    std::printf("], \"ms_detect_max_rank\": %.3f, \"ms_exchange_max_rank\": %.3f}\n", md, mx);
    for (int g = 0; g < n_gpus; ++g) {
        (void)hipSetDevice(ranks[g].device);
        if (ranks[g].d_recs) (void)hipFree(ranks[g].d_recs);
        if (ranks[g].d_all) (void)hipFree(ranks[g].d_all);
        sift_hip_comm_destroy(comms[g]);
    }
    return rc;
}
