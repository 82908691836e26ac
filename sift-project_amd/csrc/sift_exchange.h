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
//   A  header    all-gather of 5 words per rank (fixed size, buffers
//                allocated with the communicator): {tag A, status,
//                max_local, n_local, local_rows}. A bad argument is a status,
//                not an early return.
//   B  ready     ALWAYS joined by every rank, whatever phase A showed: a rank
//                that phase A left healthy grows its scratch to the agreed
//                slot size (16 * max_local table bytes + max_rows * 168
//                record bytes) and stages its table + records into its send
//                slot; then an all-gather of 2 words per rank {tag B, ready}.
//                The payload collective runs only when every rank's ready
//                word is OK and carries this call's tag B.
//   C  payload   all-gather of the slots; the receiver drops the padding by
//                copies into the caller's buffer, rank-major, and reads the
//                tables back for out_ids / out_counts (local work only: a
//                failure here, or cap_out too small, is this rank's error and
//                nobody waits for it).
//
// Tags: every word block starts with a per-call tag (call sequence number *
// 4 + phase; all ranks count calls alike). A rank whose host->device staging
// of its words failed still joins the collective, and its peers receive the
// send buffer's previous contents, whose tag is another call's or another
// phase's: they read that as a failed peer. So a staging failure is agreed
// like any other local failure (the failing rank returns its own error, the
// peers SIFT_ERR_PEER after phase B), and a failure to read phase A's result
// back only makes that rank report "not ready" in phase B.
//
// Statuses, identical on every healthy rank: a local failure -> that rank's
// own error; max_local differing between ranks -> SIFT_ERR_ARG; any other
// rank failed -> SIFT_ERR_PEER. A collective that itself fails (transport
// error) is reported as SIFT_ERR_NO_COMM, and so is the one case no further
// collective can settle: a rank that sent "ready" and then cannot read phase
// B's words back (the device itself is lost; the peers may be in phase C).
//
// Transport interface (T): rank(), nranks(),
//   int64_t next_seq()  — this rank's call counter (1, 2, ...),
//   int gather_words(const int64_t* mine, int64_t* all, size_t words, bool* sent)
//       — collective on small host arrays through buffers the transport
//         owns. The collective is always joined; SIFT_ERR_NO_COMM when it
//         failed; SIFT_ERR_HIP when a local copy failed (*sent: whether this
//         rank's words reached the collective; `all` is valid only on SIFT_OK),
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
constexpr int kExchHdrWords = 5;
constexpr int kExchReadyWords = 2;

// per-rank figures every rank derives identically from the gathered headers
struct ExchangePlan {
    size_t max_rows = 0, total = 0, slot_bytes = 0, table_bytes = 0;
    std::vector<size_t> rows;  // records per rank
};

inline ExchangePlan exchange_plan(const int64_t* hdr_all, int nranks, int max_local) {
    ExchangePlan p;
    p.rows.assign(nranks, 0);
    for (int r = 0; r < nranks; ++r) {
        p.rows[r] = (size_t)hdr_all[r * kExchHdrWords + 4];
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
    const int64_t seq = t.next_seq();
    const int64_t tag_a = seq * 4 + 1, tag_b = seq * 4 + 2;
    // ---- A: headers
    const int64_t hdr[kExchHdrWords] = {tag_a, st, max_local, st == SIFT_OK ? n_local : 0,
                                        (int64_t)local_rows};
    std::vector<int64_t> all((size_t)R * kExchHdrWords);
    bool sent = false;
    int e = t.gather_words(hdr, all.data(), kExchHdrWords, &sent);
    if (e == SIFT_ERR_NO_COMM) return e;
    if (e != SIFT_OK && st == SIFT_OK) st = e;  // staging or read-back: local
    int agreed = SIFT_OK;                       // phase A's verdict (healthy ranks)
    ExchangePlan p;
    if (st == SIFT_OK) {
        bool peer_bad = false, mismatch = false;
        for (int r = 0; r < R; ++r) {
            const int64_t* h = &all[(size_t)r * kExchHdrWords];
            if (h[0] != tag_a || h[1] != SIFT_OK)
                peer_bad = true;  // failed, or its words never arrived (stale tag)
            else
                mismatch |= h[2] != max_local;
        }
        agreed = mismatch ? SIFT_ERR_ARG : peer_bad ? SIFT_ERR_PEER : SIFT_OK;
        if (agreed == SIFT_OK) p = exchange_plan(all.data(), R, max_local);
    }
    // ---- B: scratch + staging (healthy ranks only), then agree (everyone)
    unsigned char *d_send = nullptr, *d_recv = nullptr;
    int st_b = SIFT_OK;
    if (st == SIFT_OK && agreed == SIFT_OK) {
        st_b = t.reserve(p.slot_bytes, &d_send, &d_recv);
        if (st_b == SIFT_OK) {
            std::vector<int64_t> table((size_t)2 * max_local, -1);
            for (int j = 0; j < n_local; ++j) {
                table[2 * j] = ids[j];
                table[2 * j + 1] = (int64_t)counts[j];
            }
            st_b = t.h2d(d_send, table.data(), p.table_bytes);
            // the host table must outlive the copy
            if (st_b == SIFT_OK) st_b = t.sync();
        }
        if (st_b == SIFT_OK && local_rows > 0)
            st_b = t.d2d(d_send + p.table_bytes, d_recs, local_rows * kExchRec);
    }
    const int64_t my_ready = st != SIFT_OK ? st : agreed != SIFT_OK ? agreed : st_b;
    const int64_t ready[kExchReadyWords] = {tag_b, my_ready};
    std::vector<int64_t> ready_all((size_t)R * kExchReadyWords);
    e = t.gather_words(ready, ready_all.data(), kExchReadyWords, &sent);
    if (e == SIFT_ERR_NO_COMM) return e;
    if (st != SIFT_OK) return st;  // not ready: no peer goes on to phase C
    if (agreed != SIFT_OK) return agreed;
    if (st_b != SIFT_OK) return st_b;
    // ready was sent as OK but the verdict cannot be read back: the peers
    // may be in phase C already (see the header)
    if (e != SIFT_OK) return sent ? SIFT_ERR_NO_COMM : e;
    for (int r = 0; r < R; ++r)
        if (ready_all[(size_t)r * kExchReadyWords] != tag_b ||
            ready_all[(size_t)r * kExchReadyWords + 1] != SIFT_OK)
            return SIFT_ERR_PEER;
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
