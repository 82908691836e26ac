// sift_comm.hip — native RCCL record exchange for C++ batch drivers
// (include/sift_hip.h "multi-GPU"; SURVEY §8e, BASELINE config 4).
//
// detect_keypoints_and_descriptors is a pure function of one image
// (reference src/sift.cpp:712-776), so a batch shards by image: rank r
// detects images i % nranks == r with no data-path collective. The one
// exchange gives every rank every image's final records, as
// sift_dist.allgather_records does over torch.distributed, here without
// torch: RCCL has no all-gather-v, so
//   phase 1  all-gather of each rank's (image id, record count) table
//            (max_local entries, -1 = absent),
//   phase 2  all-gather of the records padded to the largest rank's count,
//            then the padding is dropped by device-to-device copies into the
//            caller's buffer, rank-major (rank 0's images in their order,
//            then rank 1's, ...).
// Communicators come from ncclCommInitAll (one process driving every GPU,
// one host thread per GPU) or ncclCommInitRank (one process per
// GPU, the id shared out of band). RCCL is opened with dlopen on first use,
// so libsift_hip.so carries no link dependency on it (a process that already
// loaded RCCL — torch — shares its copy).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <new>
#include <vector>

#include "../../include/sift_hip.h"

namespace {

struct RcclApi {
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) init_rank = nullptr;
    decltype(&ncclCommInitAll) init_all = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclAllGather) all_gather = nullptr;
    bool ok = false;
};

const RcclApi& rccl() {
    static const RcclApi api = [] {
        RcclApi a;
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
        if (!h) return a;
        a.get_unique_id = reinterpret_cast<decltype(a.get_unique_id)>(dlsym(h, "ncclGetUniqueId"));
        a.init_rank = reinterpret_cast<decltype(a.init_rank)>(dlsym(h, "ncclCommInitRank"));
        a.init_all = reinterpret_cast<decltype(a.init_all)>(dlsym(h, "ncclCommInitAll"));
        a.destroy = reinterpret_cast<decltype(a.destroy)>(dlsym(h, "ncclCommDestroy"));
        a.all_gather = reinterpret_cast<decltype(a.all_gather)>(dlsym(h, "ncclAllGather"));
        a.ok = a.get_unique_id && a.init_rank && a.init_all && a.destroy && a.all_gather;
        return a;
    }();
    return api;
}

constexpr size_t kRec = sizeof(sift_kp);  // 168 B, the reference Keypoint

}  // namespace

struct sift_comm {
    ncclComm_t comm = nullptr;
    int rank = 0, nranks = 1, device = 0;
    hipStream_t own = nullptr;  // used when the caller passes no stream
    // device scratch: meta tables (send, gathered) and padded payloads
    int64_t* d_meta = nullptr;
    size_t meta_cap = 0;  // int64 words of the gathered table
    unsigned char* d_send = nullptr;
    unsigned char* d_recv = nullptr;
    size_t rows_cap = 0;  // padded rows per rank the scratch holds
    int64_t* h_meta = nullptr;  // pinned: send table + gathered table
    size_t h_meta_cap = 0;
};

namespace {

int comm_create(int device, sift_comm** out) {
    sift_comm* c = new (std::nothrow) sift_comm();
    if (!c) return SIFT_ERR_NOMEM;
    c->device = device;
    if (hipSetDevice(device) != hipSuccess ||
        hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return SIFT_ERR_HIP;
    }
    *out = c;
    return SIFT_OK;
}

// grow-only scratch of one exchange: 2 * max_local (id, count) words per rank
// and max_rows padded records per rank
int ensure_scratch(sift_comm* c, int max_local, size_t max_rows) {
    const size_t meta = (size_t)2 * max_local * (c->nranks + 1);
    if (meta > c->meta_cap) {
        if (c->d_meta) (void)hipFree(c->d_meta);
        if (c->h_meta) (void)hipHostFree(c->h_meta);
        c->d_meta = nullptr;
        c->h_meta = nullptr;
        c->meta_cap = 0;
        if (hipMalloc(&c->d_meta, meta * sizeof(int64_t)) != hipSuccess ||
            hipHostMalloc(&c->h_meta, meta * sizeof(int64_t)) != hipSuccess)
            return SIFT_ERR_NOMEM;
        c->meta_cap = meta;
    }
    if (max_rows > c->rows_cap) {
        if (c->d_send) (void)hipFree(c->d_send);
        if (c->d_recv) (void)hipFree(c->d_recv);
        c->d_send = c->d_recv = nullptr;
        c->rows_cap = 0;
        const size_t want = max_rows + max_rows / 4;
        if (hipMalloc(&c->d_send, want * kRec) != hipSuccess ||
            hipMalloc(&c->d_recv, want * kRec * c->nranks) != hipSuccess)
            return SIFT_ERR_NOMEM;
        c->rows_cap = want;
    }
    return SIFT_OK;
}

}  // namespace

extern "C" {

int sift_hip_comm_unique_id(unsigned char id[SIFT_COMM_ID_BYTES]) {
    if (!id) return SIFT_ERR_ARG;
    if (!rccl().ok) return SIFT_ERR_NO_COMM;
    ncclUniqueId u;
    if (rccl().get_unique_id(&u) != ncclSuccess) return SIFT_ERR_NO_COMM;
    static_assert(sizeof u == SIFT_COMM_ID_BYTES, "RCCL unique id size");
    std::memcpy(id, &u, sizeof u);
    return SIFT_OK;
}

int sift_hip_comm_init_rank(const unsigned char id[SIFT_COMM_ID_BYTES], int nranks, int rank,
                            int device, sift_comm** out) {
    if (!id || !out || nranks < 1 || rank < 0 || rank >= nranks) return SIFT_ERR_ARG;
    *out = nullptr;
    if (!rccl().ok) return SIFT_ERR_NO_COMM;
    sift_comm* c = nullptr;
    int st = comm_create(device, &c);
    if (st != SIFT_OK) return st;
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof u);
    if (rccl().init_rank(&c->comm, nranks, u, rank) != ncclSuccess) {
        c->comm = nullptr;
        sift_hip_comm_destroy(c);
        return SIFT_ERR_NO_COMM;
    }
    c->rank = rank;
    c->nranks = nranks;
    *out = c;
    return SIFT_OK;
}

int sift_hip_comm_init_all(int n_devices, const int* devices, sift_comm** comms) {
    if (n_devices < 1 || !devices || !comms) return SIFT_ERR_ARG;
    for (int i = 0; i < n_devices; ++i) comms[i] = nullptr;
    if (!rccl().ok) return SIFT_ERR_NO_COMM;
    std::vector<ncclComm_t> nc(n_devices, nullptr);
    if (rccl().init_all(nc.data(), n_devices, devices) != ncclSuccess) return SIFT_ERR_NO_COMM;
    int st = SIFT_OK;
    for (int i = 0; i < n_devices; ++i) {
        if (st == SIFT_OK) st = comm_create(devices[i], &comms[i]);
        if (st != SIFT_OK) {
            (void)rccl().destroy(nc[i]);
            continue;
        }
        comms[i]->comm = nc[i];
        comms[i]->rank = i;
        comms[i]->nranks = n_devices;
    }
    if (st != SIFT_OK)
        for (int i = 0; i < n_devices; ++i) {
            if (comms[i]) sift_hip_comm_destroy(comms[i]);
            comms[i] = nullptr;
        }
    return st;
}

int sift_hip_comm_destroy(sift_comm* c) {
    if (!c) return SIFT_ERR_ARG;
    (void)hipSetDevice(c->device);
    if (c->own) (void)hipStreamSynchronize(c->own);
    if (c->comm && rccl().ok) (void)rccl().destroy(c->comm);
    if (c->d_meta) (void)hipFree(c->d_meta);
    if (c->h_meta) (void)hipHostFree(c->h_meta);
    if (c->d_send) (void)hipFree(c->d_send);
    if (c->d_recv) (void)hipFree(c->d_recv);
    if (c->own) (void)hipStreamDestroy(c->own);
    delete c;
    return SIFT_OK;
}

int sift_hip_comm_rank(const sift_comm* c, int* rank, int* nranks) {
    if (!c) return SIFT_ERR_ARG;
    if (rank) *rank = c->rank;
    if (nranks) *nranks = c->nranks;
    return SIFT_OK;
}

int sift_hip_allgather_records(sift_comm* c, const sift_kp* d_recs, const int64_t* ids,
                               const size_t* counts, int n_local, int max_local, sift_kp* d_out,
                               size_t cap_out, int64_t* out_ids, size_t* out_counts,
                               size_t* n_out, void* stream) {
    if (!c || n_local < 0 || max_local < 1 || n_local > max_local || !out_ids || !out_counts ||
        !n_out || (n_local > 0 && (!ids || !counts)))
        return SIFT_ERR_ARG;
    size_t local_rows = 0;
    for (int j = 0; j < n_local; ++j) {
        if (ids[j] < 0) return SIFT_ERR_ARG;
        local_rows += counts[j];
    }
    if (local_rows > 0 && !d_recs) return SIFT_ERR_ARG;
    if (hipSetDevice(c->device) != hipSuccess) return SIFT_ERR_HIP;
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : c->own;
    const RcclApi& R = rccl();
    const int R_ = c->nranks;
    const size_t m = (size_t)2 * max_local;  // words of one rank's table
    int e = ensure_scratch(c, max_local, 0);
    if (e != SIFT_OK) return e;
    // ---- phase 1: (image id, count) tables
    int64_t* h_send = c->h_meta;
    int64_t* h_all = c->h_meta + m;
    for (size_t w = 0; w < m; ++w) h_send[w] = -1;
    for (int j = 0; j < n_local; ++j) {
        h_send[2 * j] = ids[j];
        h_send[2 * j + 1] = (int64_t)counts[j];
    }
    int64_t* d_send_meta = c->d_meta;
    int64_t* d_all_meta = c->d_meta + m;
    if (hipMemcpyAsync(d_send_meta, h_send, m * sizeof(int64_t), hipMemcpyHostToDevice, st) !=
        hipSuccess)
        return SIFT_ERR_HIP;
    if (R.all_gather(d_send_meta, d_all_meta, m, ncclInt64, c->comm, st) != ncclSuccess)
        return SIFT_ERR_NO_COMM;
    if (hipMemcpyAsync(h_all, d_all_meta, m * R_ * sizeof(int64_t), hipMemcpyDeviceToHost, st) !=
            hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        return SIFT_ERR_HIP;
    std::vector<size_t> rows(R_, 0);
    size_t max_rows = 1, total = 0;
    for (int r = 0; r < R_; ++r) {
        for (int j = 0; j < max_local; ++j) {
            const int64_t id = h_all[r * m + 2 * j], n = h_all[r * m + 2 * j + 1];
            out_ids[(size_t)r * max_local + j] = id;
            out_counts[(size_t)r * max_local + j] = id >= 0 ? (size_t)n : 0;
            if (id >= 0) rows[r] += (size_t)n;
        }
        max_rows = std::max(max_rows, rows[r]);
        total += rows[r];
    }
    *n_out = total;
    // ---- phase 2: payloads padded to the largest rank (every rank takes
    // part whatever its capacity, so no rank can leave the others waiting)
    if ((e = ensure_scratch(c, max_local, max_rows)) != SIFT_OK) return e;
    if (local_rows > 0 &&
        hipMemcpyAsync(c->d_send, d_recs, local_rows * kRec, hipMemcpyDeviceToDevice, st) !=
            hipSuccess)
        return SIFT_ERR_HIP;
    if (R.all_gather(c->d_send, c->d_recv, max_rows * kRec, ncclUint8, c->comm, st) !=
        ncclSuccess)
        return SIFT_ERR_NO_COMM;
    if (total > cap_out || (total > 0 && !d_out)) {
        (void)hipStreamSynchronize(st);
        return SIFT_ERR_ARG;  // exchange completed; nothing written to d_out
    }
    unsigned char* dst = reinterpret_cast<unsigned char*>(d_out);
    for (int r = 0; r < R_; ++r) {
        if (rows[r] > 0 &&
            hipMemcpyAsync(dst, c->d_recv + (size_t)r * max_rows * kRec, rows[r] * kRec,
                           hipMemcpyDeviceToDevice, st) != hipSuccess)
            return SIFT_ERR_HIP;
        dst += rows[r] * kRec;
    }
    return hipStreamSynchronize(st) == hipSuccess ? SIFT_OK : SIFT_ERR_HIP;
}

}  // extern "C"
