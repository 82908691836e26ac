// exchange_selftest.cpp — CPU test of the record exchange's protocol
// (sift-project_amd/csrc/sift_exchange.h, the code sift_hip_allgather_records
// runs over RCCL) at world sizes 1-4 with one host thread per rank and a
// host-memory transport: the same padding, slot offsets and rank-major
// compaction, plus injected local failures (bad arguments, max_local
// mismatch, allocation and staging failures, a too-small output) that must
// end every rank's call — none may be left inside a collective — with the
// agreed statuses. A watchdog turns a hang into exit code 3.
//
//   exchange_selftest      prints one line per scenario, exit 0 when all pass
// Built with g++ by __graft_entry__.build(); run by tests/test_dist.py.
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../sift-project_amd/csrc/sift_exchange.h"

namespace {

// all-gather of equal-size byte blocks between threads (a generation barrier)
struct Bus {
    explicit Bus(int n) : R(n), blocks(n) {}
    int R;
    std::mutex m;
    std::condition_variable cv;
    int arrived = 0, gen = 0;
    std::vector<std::vector<unsigned char>> blocks;
    void barrier() {
        std::unique_lock<std::mutex> g(m);
        const int my = gen;
        if (++arrived == R) {
            arrived = 0;
            ++gen;
            cv.notify_all();
        } else {
            cv.wait(g, [&] { return gen != my; });
        }
    }
    void gather(int rank, const void* mine, void* all, size_t bytes) {
        {
            std::lock_guard<std::mutex> g(m);
            blocks[rank].assign((const unsigned char*)mine, (const unsigned char*)mine + bytes);
        }
        barrier();
        for (int r = 0; r < R; ++r) {
            if (blocks[r].size() != bytes) {  // unequal counts: RCCL would be undefined
                std::fprintf(stderr, "collective size mismatch\n");
                std::_Exit(4);
            }
            std::memcpy((unsigned char*)all + r * bytes, blocks[r].data(), bytes);
        }
        barrier();
    }
};

struct Faults {
    bool fail_reserve = false, fail_h2d = false;
    // word collective number k (0-based over the rank's whole life) fails:
    // its staging copy (the peers receive the previous words) / its read-back
    int fail_stage_at = -1, fail_read_at = -1;
};

struct HostTransport {
    Bus* bus;
    int r;
    Faults f;
    std::vector<unsigned char> send, recv;
    int collectives = 0, word_calls = 0;
    int64_t seq = 0;
    int64_t send_words[8] = {};  // the "device" send buffer of the word collectives
    int rank() const { return r; }
    int nranks() const { return bus->R; }
    int64_t next_seq() { return ++seq; }
    int gather_words(const int64_t* mine, int64_t* all, size_t words, bool* sent) {
        ++collectives;
        const int k = word_calls++;
        *sent = k != f.fail_stage_at;
        if (*sent) std::memcpy(send_words, mine, words * sizeof(int64_t));
        std::vector<int64_t> got(words * bus->R);
        bus->gather(r, send_words, got.data(), words * sizeof(int64_t));
        if (k == f.fail_read_at) return SIFT_ERR_HIP;
        std::memcpy(all, got.data(), got.size() * sizeof(int64_t));
        return *sent ? SIFT_OK : SIFT_ERR_HIP;
    }
    int reserve(size_t slot, unsigned char** ds, unsigned char** dr) {
        if (f.fail_reserve) return SIFT_ERR_NOMEM;
        send.assign(slot, 0xAB);  // poisoned padding
        recv.assign(slot * bus->R, 0xCD);
        *ds = send.data();
        *dr = recv.data();
        return SIFT_OK;
    }
    int gather_slots(const unsigned char* ds, unsigned char* dr, size_t slot) {
        ++collectives;
        bus->gather(r, ds, dr, slot);
        return SIFT_OK;
    }
    int h2d(void* d, const void* h, size_t n) {
        if (f.fail_h2d) return SIFT_ERR_HIP;
        std::memcpy(d, h, n);
        return SIFT_OK;
    }
    int d2d(void* d, const void* s, size_t n) {
        std::memcpy(d, s, n);
        return SIFT_OK;
    }
    int d2h(void* h, const void* d, size_t n) {
        std::memcpy(h, d, n);
        return SIFT_OK;
    }
    int sync() { return SIFT_OK; }
};

struct RankIn {
    std::vector<int64_t> ids;
    std::vector<size_t> counts;
    int max_local = 1;
    size_t cap_out = (size_t)-1;
    bool bad_arg = false;
    Faults f;
};

sift_kp make_rec(int64_t id, size_t k) {
    sift_kp p;
    std::memset(&p, 0, sizeof p);
    p.x = (double)id + 0.25;
    p.y = (double)k;
    p.octave = (int)id;
    p.layer = (int)(k % 7);
    for (int b = 0; b < 128; ++b) p.desc[b] = (uint8_t)(id * 31 + k * 7 + b);
    return p;
}

bool rec_eq(const sift_kp& a, const sift_kp& b) { return std::memcmp(&a, &b, sizeof a) == 0; }

// run one scenario; expect[r] = status rank r must return
// (calls > 1: the same transports run the exchange `calls` times, the
// earlier calls must succeed; statuses and outputs are the last call's)
bool scenario(const char* name, const std::vector<RankIn>& in, const std::vector<int>& expect,
              int calls = 1) {
    const int R = (int)in.size();
    Bus bus(R);
    std::vector<int> st(R, 99);
    std::vector<std::vector<sift_kp>> out(R);
    std::vector<std::vector<int64_t>> oid(R);
    std::vector<std::vector<size_t>> ocnt(R);
    std::vector<size_t> nout(R, 0);
    std::vector<int> ncoll(R, 0);
    std::atomic<int> finished{0};
    std::vector<std::thread> th;
    for (int r = 0; r < R; ++r)
        th.emplace_back([&, r] {
            const RankIn& a = in[r];
            std::vector<sift_kp> recs;
            for (size_t j = 0; j < a.ids.size(); ++j)
                for (size_t k = 0; k < a.counts[j]; ++k) recs.push_back(make_rec(a.ids[j], k));
            size_t total_in = 0;
            for (const RankIn& b : in)
                for (size_t c : b.counts) total_in += c;
            out[r].assign(total_in + 1, sift_kp{});
            oid[r].assign((size_t)R * std::max(1, a.max_local), -7);
            ocnt[r].assign((size_t)R * std::max(1, a.max_local), 7);
            HostTransport t{&bus, r, a.f, {}, {}};
            for (int call = 0; call < calls; ++call) {
                const bool last = call + 1 == calls;
                const int n_local = a.bad_arg && last ? a.max_local + 1 : (int)a.ids.size();
                t.collectives = 0;
                st[r] = sift_amd::exchange_records(
                    t, recs.empty() ? nullptr : recs.data(), a.ids.data(), a.counts.data(),
                    n_local, a.max_local, out[r].data(), std::min(a.cap_out, out[r].size()),
                    oid[r].data(), ocnt[r].data(), &nout[r]);
                if (!last && st[r] != SIFT_OK) st[r] = 1000 + st[r];  // an earlier call failed
            }
            ncoll[r] = t.collectives;
            finished.fetch_add(1);
        });
    const auto t0 = std::chrono::steady_clock::now();
    while (finished.load() < R) {
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(10)) {
            std::printf("HANG %s: %d of %d ranks returned\n", name, finished.load(), R);
            std::fflush(stdout);
            std::_Exit(3);
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    for (auto& x : th) x.join();
    bool ok = true;
    std::string why;
    for (int r = 0; r < R; ++r) {
        if (st[r] != expect[r]) {
            ok = false;
            why += " rank" + std::to_string(r) + " status " + std::to_string(st[r]) +
                   " want " + std::to_string(expect[r]);
        }
        // every rank took part in the same number of collectives
        if (ncoll[r] != ncoll[0]) {
            ok = false;
            why += " rank" + std::to_string(r) + " collectives " + std::to_string(ncoll[r]);
        }
    }
    // successful ranks: rank-major records, tables, total
    for (int r = 0; r < R && ok; ++r) {
        // (SIFT_ERR_ARG from a too-small output still has the tables and n_out)
        const bool cap_short = st[r] == SIFT_ERR_ARG && in[r].cap_out != (size_t)-1;
        if (st[r] != SIFT_OK && !cap_short) continue;
        size_t k = 0, total = 0;
        for (int q = 0; q < R; ++q) {
            const int ml = in[r].max_local;
            for (int j = 0; j < ml; ++j) {
                const bool has = j < (int)in[q].ids.size();
                const int64_t want_id = has ? in[q].ids[j] : -1;
                const size_t want_n = has ? in[q].counts[j] : 0;
                if (oid[r][(size_t)q * ml + j] != want_id || ocnt[r][(size_t)q * ml + j] != want_n) {
                    ok = false;
                    why += " table";
                }
            }
            for (size_t j = 0; j < in[q].ids.size(); ++j)
                for (size_t c = 0; c < in[q].counts[j]; ++c, ++k)
                    if (st[r] == SIFT_OK && !rec_eq(out[r][k], make_rec(in[q].ids[j], c))) {
                        ok = false;
                        why += " record";
                    }
            for (size_t c : in[q].counts) total += c;
        }
        if (nout[r] != total) {
            ok = false;
            why += " n_out";
        }
        if (st[r] == SIFT_ERR_ARG) {  // d_out untouched
            for (const sift_kp& p : out[r])
                if (!rec_eq(p, sift_kp{})) {
                    ok = false;
                    why += " wrote";
                    break;
                }
        }
    }
    std::printf("%s %s (world %d, %d collectives)%s\n", ok ? "ok" : "FAIL", name, R, ncoll[0],
                why.c_str());
    return ok;
}

RankIn rank_of(std::vector<int64_t> ids, std::vector<size_t> counts, int max_local) {
    RankIn a;
    a.ids = std::move(ids);
    a.counts = std::move(counts);
    a.max_local = max_local;
    return a;
}

}  // namespace

int main() {
    bool ok = true;
    // BASELINE config 4 layout at small scale: image i on rank i % R
    ok &= scenario("world1", {rank_of({0, 1}, {5, 0}, 2)}, {SIFT_OK});
    ok &= scenario("world2-uneven", {rank_of({0, 2, 4}, {3, 7, 1}, 3), rank_of({1, 3}, {9, 2}, 3)},
                   {SIFT_OK, SIFT_OK});
    ok &= scenario("world3-empty-rank",
                   {rank_of({0, 3}, {4, 0}, 2), rank_of({}, {}, 2), rank_of({2}, {11}, 2)},
                   {SIFT_OK, SIFT_OK, SIFT_OK});
    ok &= scenario("world3-all-empty", {rank_of({}, {}, 1), rank_of({}, {}, 1), rank_of({}, {}, 1)},
                   {SIFT_OK, SIFT_OK, SIFT_OK});
    ok &= scenario("world2-three-calls",
                   {rank_of({0, 2}, {3, 7}, 2), rank_of({1}, {9}, 2)}, {SIFT_OK, SIFT_OK}, 3);
    ok &= scenario("world4-large",
                   {rank_of({0, 4}, {3000, 10}, 2), rank_of({1, 5}, {1, 2}, 2),
                    rank_of({2}, {777}, 2), rank_of({3, 7}, {0, 5000}, 2)},
                   {SIFT_OK, SIFT_OK, SIFT_OK, SIFT_OK});
    {  // a rank's allocation fails after the headers: everyone returns before the payload
        std::vector<RankIn> in = {rank_of({0}, {4}, 1), rank_of({1}, {6}, 1), rank_of({2}, {2}, 1)};
        in[1].f.fail_reserve = true;
        ok &= scenario("world3-nomem-rank1", in, {SIFT_ERR_PEER, SIFT_ERR_NOMEM, SIFT_ERR_PEER});
    }
    {  // a rank's staging copy fails
        std::vector<RankIn> in = {rank_of({0}, {4}, 1), rank_of({1}, {6}, 1)};
        in[0].f.fail_h2d = true;
        ok &= scenario("world2-staging-rank0", in, {SIFT_ERR_HIP, SIFT_ERR_PEER});
    }
    {  // a bad argument on one rank: agreed in the headers
        std::vector<RankIn> in = {rank_of({0}, {4}, 1), rank_of({1}, {6}, 1)};
        in[1].bad_arg = true;
        ok &= scenario("world2-badarg-rank1", in, {SIFT_ERR_PEER, SIFT_ERR_ARG});
    }
    {  // a rank's header staging fails: the peers see the send buffer's old
       // words (no valid tag) and count it as failed
        std::vector<RankIn> in = {rank_of({0}, {4}, 1), rank_of({1}, {6}, 1), rank_of({2}, {2}, 1)};
        in[1].f.fail_stage_at = 0;
        ok &= scenario("world3-header-stage-rank1", in,
                       {SIFT_ERR_PEER, SIFT_ERR_HIP, SIFT_ERR_PEER});
    }
    {  // the same in a second call: the stale words are the first call's
        std::vector<RankIn> in = {rank_of({0}, {4}, 1), rank_of({1}, {6}, 1), rank_of({2}, {2}, 1)};
        in[2].f.fail_stage_at = 2;
        ok &= scenario("world3-header-stage-2nd-call", in,
                       {SIFT_ERR_PEER, SIFT_ERR_PEER, SIFT_ERR_HIP}, 2);
    }
    {  // a rank's ready staging fails: the peers see its header words (phase-A tag)
        std::vector<RankIn> in = {rank_of({0}, {4}, 1), rank_of({1}, {6}, 1)};
        in[0].f.fail_stage_at = 1;
        ok &= scenario("world2-ready-stage-rank0", in, {SIFT_ERR_HIP, SIFT_ERR_PEER});
    }
    {  // a rank cannot read the headers back: its peers went on to phase B,
       // where it reports "not ready"
        std::vector<RankIn> in = {rank_of({0}, {4}, 1), rank_of({1}, {6}, 1), rank_of({2}, {2}, 1)};
        in[0].f.fail_read_at = 0;
        ok &= scenario("world3-header-read-rank0", in,
                       {SIFT_ERR_HIP, SIFT_ERR_PEER, SIFT_ERR_PEER});
    }
    // max_local differs: every rank reports the argument error
    ok &= scenario("world2-maxlocal-mismatch", {rank_of({0}, {4}, 1), rank_of({1}, {6}, 2)},
                   {SIFT_ERR_ARG, SIFT_ERR_ARG});
    {  // one rank's output too small: only it fails, after the collectives
        std::vector<RankIn> in = {rank_of({0}, {4}, 1), rank_of({1}, {6}, 1)};
        in[0].cap_out = 3;
        ok &= scenario("world2-cap-rank0", in, {SIFT_ERR_ARG, SIFT_OK});
    }
    std::printf("%s\n", ok ? "ALL OK" : "FAILURES");
    return ok ? 0 : 1;
}
