// sift_exchange.h — the record exchange's protocol, independent of the
// transport (include/sift_hip.h sift_hip_allgather_records).
//
// detect_keypoints_and_descriptors is a pure function of one image
// (reference src/sift.cpp:712-776), so a batch shards by image and the only
// collective is this exchange: every rank receives every image's final
// records. RCCL has no all-gather-v, so the records travel padded to the
// largest rank's count. The protocol is written so that NO local failure can
// leave a peer blocked inside a collective: every rank enters every
// collective of a call, and failures are agreed on before the data moves.
//
//   A  header    all-gather of 4 words per rank (fixed size, buffers
//                allocated with the communicator): {status, max_local,
//                n_local, local_rows}. A bad argument is a status, not an
//                early return. Every rank sees every header, so all ranks
//                take the same decision: any status != OK -> every rank
//                returns (its own error, or SIFT_ERR_PEER); differing
//                max_local -> SIFT_ERR_ARG on every rank.
//   B  ready     each rank grows its scratch to the agreed slot size
//                (16 * max_local table bytes + max_rows * 168 record bytes)
//                and stages its table + records into its send slot; then an
//                all-gather of one status word per rank; any failure ->
//                every rank returns before the payload collective.
//   C  payload   all-gather of the slots; the receiver drops the padding by
//                copies into the caller's buffer, rank-major, and reads the
//                tables back for out_ids / out_counts (local work only: a
//                failure here, or cap_out too small, is this rank's error and
//                nobody waits for it).
//
// A collective that itself fails (transport error) is reported as
// SIFT_ERR_NO_COMM; a broken device cannot be recovered by any protocol.
//
// Transport interface (T): rank(), nranks(),
//   int gather_words(const int64_t* mine, int64_t* all, size_t words)
//       — collective on small host arrays (staged through buffers the
//         transport owns, so it cannot fail for lack of memory),
//   int reserve(size_t slot_bytes, unsigned char** d_send, unsigned char** d_recv)
//       — grow-only device scratch: send slot + nranks receive slots,
//   int gather_slots(const unsigned char* d_send, unsigned char* d_recv, size_t slot_bytes),
//   int h2d(void* d, const void* h, size_t n), d2d(...), d2h(...), sync().
// Every call returns SIFT_OK or a SIFT_ERR_* code.
#pragma once

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/sift_hip.h"

namespace sift_amd {

constexpr size_t kExchRec = sizeof(sift_kp);  // 168 B, the reference Keypoint
constexpr int kExchHdrWords = 4;

// per-rank figures every rank derives identically from the gathered headers
struct ExchangePlan {
    size_t max_rows = 0, total = 0, slot_bytes = 0, table_bytes = 0;
    std::vector<size_t> rows;  // records per rank
};

inline ExchangePlan exchange_plan(const int64_t* hdr_all, int nranks, int max_local) {
    ExchangePlan p;
    p.rows.assign(nranks, 0);
    for (int r = 0; r < nranks; ++r) {
        p.rows[r] = (size_t)hdr_all[r * kExchHdrWords + 3];
        p.max_rows = std::max(p.max_rows, p.rows[r]);
        p.total += p.rows[r];
    }
    p.table_bytes = (size_t)16 * max_local;
    // 16-B aligned slots (the records follow the table)
    p.slot_bytes = (p.table_bytes + p.max_rows * kExchRec + 15) & ~(size_t)15;
    return p;
}

template <class T>
int exchange_records(T& t, const sift_kp* d_recs, const int64_t* ids, const size_t* counts,
                     int n_local, int max_local, sift_kp* d_out, size_t cap_out,
                     int64_t* out_ids, size_t* out_counts, size_t* n_out) {
    const int R = t.nranks();
    // ---- local validation: a status in the header, never an early return
    int st = SIFT_OK;
    size_t local_rows = 0;
    if (n_local < 0 || max_local < 1 || n_local > max_local || !out_ids || !out_counts ||
        !n_out || (n_local > 0 && (!ids || !counts)))
        st = SIFT_ERR_ARG;
    for (int j = 0; st == SIFT_OK && j < n_local; ++j) {
        if (ids[j] < 0) st = SIFT_ERR_ARG;
        local_rows += counts[j];
    }
    if (st == SIFT_OK && local_rows > 0 && !d_recs) st = SIFT_ERR_ARG;
    if (st != SIFT_OK) local_rows = 0;
    // ---- A: headers
    const int64_t hdr[kExchHdrWords] = {st, max_local, st == SIFT_OK ? n_local : 0,
                                        (int64_t)local_rows};
    std::vector<int64_t> all((size_t)R * kExchHdrWords);
    int e = t.gather_words(hdr, all.data(), kExchHdrWords);
    if (e != SIFT_OK) return e;
    bool peer_bad = false, mismatch = false;
    for (int r = 0; r < R; ++r) {
        peer_bad |= all[r * kExchHdrWords] != SIFT_OK;
        mismatch |= all[r * kExchHdrWords + 1] != max_local;
    }
    if (st != SIFT_OK) return st;
    if (mismatch) return SIFT_ERR_ARG;  // every rank sees the same headers
    if (peer_bad) return SIFT_ERR_PEER;
    const ExchangePlan p = exchange_plan(all.data(), R, max_local);
    // ---- B: scratch + staging, then agree
    unsigned char *d_send = nullptr, *d_recv = nullptr;
    st = t.reserve(p.slot_bytes, &d_send, &d_recv);
    if (st == SIFT_OK) {
        std::vector<int64_t> table((size_t)2 * max_local, -1);
        for (int j = 0; j < n_local; ++j) {
            table[2 * j] = ids[j];
            table[2 * j + 1] = (int64_t)counts[j];
        }
        st = t.h2d(d_send, table.data(), p.table_bytes);
        // the host table must outlive the copy
        if (st == SIFT_OK) st = t.sync();
    }
    if (st == SIFT_OK && local_rows > 0)
        st = t.d2d(d_send + p.table_bytes, d_recs, local_rows * kExchRec);
    const int64_t ready = st;
    std::vector<int64_t> ready_all(R);
    e = t.gather_words(&ready, ready_all.data(), 1);
    if (e != SIFT_OK) return e;
    if (st != SIFT_OK) return st;
    for (int r = 0; r < R; ++r)
        if (ready_all[r] != SIFT_OK) return SIFT_ERR_PEER;
    // ---- C: payload, then local compaction
    if ((e = t.gather_slots(d_send, d_recv, p.slot_bytes)) != SIFT_OK) return e;
    *n_out = p.total;
    std::vector<int64_t> tables((size_t)R * 2 * max_local);
    for (int r = 0; r < R; ++r)
        if ((e = t.d2h(tables.data() + (size_t)r * 2 * max_local, d_recv + r * p.slot_bytes,
                       p.table_bytes)) != SIFT_OK)
            return e;
    const bool fits = p.total <= cap_out && (p.total == 0 || d_out);
    if (fits) {
        unsigned char* dst = reinterpret_cast<unsigned char*>(d_out);
        for (int r = 0; r < R; ++r) {
            if (p.rows[r] > 0 &&
                (e = t.d2d(dst, d_recv + r * p.slot_bytes + p.table_bytes,
                           p.rows[r] * kExchRec)) != SIFT_OK)
                return e;
            dst += p.rows[r] * kExchRec;
        }
    }
    if ((e = t.sync()) != SIFT_OK) return e;
    for (int r = 0; r < R; ++r)
        for (int j = 0; j < max_local; ++j) {
            const int64_t id = tables[((size_t)r * max_local + j) * 2];
            const int64_t n = tables[((size_t)r * max_local + j) * 2 + 1];
            out_ids[(size_t)r * max_local + j] = id;
            out_counts[(size_t)r * max_local + j] = id >= 0 ? (size_t)n : 0;
        }
    return fits ? SIFT_OK : SIFT_ERR_ARG;  // too small: exchange done, d_out untouched
}

}  // namespace sift_amd
