// sift_comm.hip — native RCCL record exchange for C++ batch drivers
// (include/sift_hip.h "multi-GPU"; SURVEY §8e, BASELINE config 4).
//
// detect_keypoints_and_descriptors is a pure function of one image
// (reference src/sift.cpp:712-776), so a batch shards by image: rank r
// detects images i % nranks == r with no data-path collective. The one
// exchange gives every rank every image's final records, as
// sift_dist.allgather_records does over torch.distributed, here without
// torch. The protocol (header all-gather, agreement on every rank's
// readiness, then the padded payload all-gather and a rank-major compaction;
// no local failure leaves a peer inside a collective) is sift_exchange.h,
// written against a transport; this file is its RCCL transport.
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
#include "sift_exchange.h"

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

}  // namespace

struct sift_comm {
    ncclComm_t comm = nullptr;
    int rank = 0, nranks = 1, device = 0;
    hipStream_t own = nullptr;  // used when the caller passes no stream
    // fixed word buffers of the header / ready collectives (allocated with
    // the communicator, so those collectives never fail for lack of memory):
    // device send (kWordCap) + gathered (kWordCap * nranks), pinned host same
    int64_t* d_words = nullptr;
    int64_t* h_words = nullptr;
    int64_t seq = 0;  // exchange calls so far (sift_exchange.h tags)
    // grow-only payload scratch: one send slot + nranks receive slots
    unsigned char* d_send = nullptr;
    unsigned char* d_recv = nullptr;
    size_t slot_cap = 0;
};

namespace {

constexpr size_t kWordCap = sift_amd::kExchHdrWords;

int comm_create(int device, int nranks, sift_comm** out) {
    sift_comm* c = new (std::nothrow) sift_comm();
    if (!c) return SIFT_ERR_NOMEM;
    c->device = device;
    c->nranks = nranks;
    const size_t words = kWordCap * (nranks + 1);
    if (hipSetDevice(device) != hipSuccess ||
        hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return SIFT_ERR_HIP;
    }
    if (hipMalloc(&c->d_words, words * sizeof(int64_t)) != hipSuccess ||
        hipHostMalloc(&c->h_words, words * sizeof(int64_t)) != hipSuccess) {
        sift_hip_comm_destroy(c);
        return SIFT_ERR_NOMEM;
    }
    // no valid tag in the send words before the first call (a staging
    // failure in that call then shows as tag 0 to the peers)
    if (hipMemset(c->d_words, 0, words * sizeof(int64_t)) != hipSuccess ||
        hipDeviceSynchronize() != hipSuccess) {
        sift_hip_comm_destroy(c);
        return SIFT_ERR_HIP;
    }
    *out = c;
    return SIFT_OK;
}

// sift_exchange.h's transport over RCCL on one stream
struct RcclTransport {
    sift_comm* c;
    hipStream_t st;
    int rank() const { return c->rank; }
    int nranks() const { return c->nranks; }
    int64_t next_seq() { return ++c->seq; }
    int gather_words(const int64_t* mine, int64_t* all, size_t words, bool* sent) {
        if (words > kWordCap) return SIFT_ERR_NO_COMM;  // equal on every rank: no collective
        std::memcpy(c->h_words, mine, words * sizeof(int64_t));
        // a failed staging copy still joins the collective (the peers are
        // in it): they receive the send buffer's previous words, whose tag
        // is not this call's, and count this rank as failed
        *sent = hipMemcpyAsync(c->d_words, c->h_words, words * sizeof(int64_t),
                               hipMemcpyHostToDevice, st) == hipSuccess;
        if (rccl().all_gather(c->d_words, c->d_words + kWordCap, words, ncclInt64, c->comm,
                              st) != ncclSuccess)
            return SIFT_ERR_NO_COMM;
        if (hipMemcpyAsync(c->h_words + kWordCap, c->d_words + kWordCap,
                           words * c->nranks * sizeof(int64_t), hipMemcpyDeviceToHost,
                           st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            return SIFT_ERR_HIP;
        std::memcpy(all, c->h_words + kWordCap, words * c->nranks * sizeof(int64_t));
        return *sent ? SIFT_OK : SIFT_ERR_HIP;
    }
    int reserve(size_t slot, unsigned char** d_send, unsigned char** d_recv) {
        if (slot > c->slot_cap) {
            if (c->d_send) (void)hipFree(c->d_send);
            if (c->d_recv) (void)hipFree(c->d_recv);
            c->d_send = c->d_recv = nullptr;
            c->slot_cap = 0;
            const size_t want = (slot + slot / 4 + 15) & ~(size_t)15;
            if (hipMalloc(&c->d_send, want) != hipSuccess ||
                hipMalloc(&c->d_recv, want * c->nranks) != hipSuccess)
                return SIFT_ERR_NOMEM;
            c->slot_cap = want;
        }
        *d_send = c->d_send;
        *d_recv = c->d_recv;
        return SIFT_OK;
    }
    int gather_slots(const unsigned char* d_send, unsigned char* d_recv, size_t slot) {
        return rccl().all_gather(d_send, d_recv, slot, ncclUint8, c->comm, st) == ncclSuccess
                   ? SIFT_OK
                   : SIFT_ERR_NO_COMM;
    }
    int copy(void* d, const void* s, size_t n, hipMemcpyKind k) {
        return hipMemcpyAsync(d, s, n, k, st) == hipSuccess ? SIFT_OK : SIFT_ERR_HIP;
    }
    int h2d(void* d, const void* h, size_t n) { return copy(d, h, n, hipMemcpyHostToDevice); }
    int d2d(void* d, const void* s, size_t n) { return copy(d, s, n, hipMemcpyDeviceToDevice); }
    int d2h(void* h, const void* d, size_t n) { return copy(h, d, n, hipMemcpyDeviceToHost); }
    int sync() { return hipStreamSynchronize(st) == hipSuccess ? SIFT_OK : SIFT_ERR_HIP; }
};

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
    int st = comm_create(device, nranks, &c);
    if (st != SIFT_OK) return st;
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof u);
    if (rccl().init_rank(&c->comm, nranks, u, rank) != ncclSuccess) {
        c->comm = nullptr;
        sift_hip_comm_destroy(c);
        return SIFT_ERR_NO_COMM;
    }
    c->rank = rank;
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
        if (st == SIFT_OK) st = comm_create(devices[i], n_devices, &comms[i]);
        if (st != SIFT_OK) {
            (void)rccl().destroy(nc[i]);
            continue;
        }
        comms[i]->comm = nc[i];
        comms[i]->rank = i;
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
    if (c->d_words) (void)hipFree(c->d_words);
    if (c->h_words) (void)hipHostFree(c->h_words);
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
    if (!c) return SIFT_ERR_ARG;  // no communicator: no collective to join
    if (hipSetDevice(c->device) != hipSuccess) return SIFT_ERR_HIP;
    RcclTransport t{c, stream ? static_cast<hipStream_t>(stream) : c->own};
    return sift_amd::exchange_records(t, d_recs, ids, counts, n_local, max_local, d_out, cap_out,
                                      out_ids, out_counts, n_out);
}

}  // extern "C"
