// share_tsan.cpp — CPU stress, under ThreadSanitizer, of the process-wide engine sharing
// (sdfs_amd/csrc/engine_share.h) and of the coalescing queue's shutdown while callers are in
// progress (sdfs_amd/csrc/host_queue.h), with a stand-in device engine (no GPU).
//
// What SDFS does to the engine and must be safe: many engine instances (static singletons,
// HashFunctionPool.borrowObject's pool, HashStore's one-shot instance — SparseDedupFile.java:100,
// HashFunctionPool.java:73-86, HashStore.java:68) used from many flush threads, and
// HashFunctionPool.destroyObject (:98-100) destroying an instance another thread may still be
// using.  Checks:
//   1. handles with equal keys share one set (reference counts), other keys get their own;
//   2. destroy while calls are in progress waits for them; calls on a destroyed handle fail;
//      the last destroy tears the set down exactly once, with no call in progress on it;
//   3. keyed calls always reach the same device (key -> device is a function), unkeyed calls
//      spread over the set, contiguous shares partition a batch;
//   4. queue shutdown with callers in flight: every caller gets its own correct result or
//      kQueueStopped, nobody hangs;
//   5. a call releasing its handle while destroy runs: destroy waits for the release to finish;
//      handle tokens are never reused;
//   6. the batch split of sdfs_cdc_get_chunks_batch at 2 and 8 devices processes every buffer
//      exactly once, and stream-key routing is stable.
// Test infrastructure only.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <string>
#include <random>
#include <thread>
#include <vector>

#include "../../sdfs_amd/csrc/engine_share.h"
#include "../../sdfs_amd/csrc/host_queue.h"

using namespace sdfs;

static uint64_t digest_of(const uint8_t* p, uint64_t n) {
    uint64_t h = 1469598103934665603ull;
    for (uint64_t i = 0; i < n; i++) h = (h ^ p[i]) * 1099511628211ull;
    return h ^ n;
}

struct CpuBackend {
    uint64_t slot_bytes = 1 << 20;
    int prepare(QSlot& s) {
        s.in = static_cast<uint8_t*>(malloc(slot_bytes));
        s.cap = slot_bytes;
        s.dev = new std::vector<uint64_t>();
        return s.in ? 0 : -4;
    }
    void release(QSlot& s) {
        free(s.in);
        s.in = nullptr;
        delete static_cast<std::vector<uint64_t>*>(s.dev);
        s.dev = nullptr;
    }
    bool admits(const QSlot&, const QReq&) { return true; }
    int launch(QSlot&, int) {
        std::this_thread::sleep_for(std::chrono::microseconds(30));
        return 0;
    }
    int wait(QSlot& s) {
        auto* r = static_cast<std::vector<uint64_t>*>(s.dev);
        r->assign(s.chunks.size(), 0);
        for (size_t i = 0; i < s.chunks.size(); i++) (*r)[i] = digest_of(s.in + s.chunks[i]->off, s.chunks[i]->len);
        return 0;
    }
};

static std::atomic<int> g_alive{0}, g_built{0}, g_torn{0};

struct FakeDev {
    int ord;
    CpuBackend b;
    CoalescingQueue<CpuBackend> q;
    std::atomic<int> calls{0}, busy{0};
    explicit FakeDev(int o) : ord(o), q(b, cfg()) {
        q.start();
        g_alive++;
        g_built++;
    }
    ~FakeDev() {
        if (busy.load() != 0) abort();  // torn down under a call in progress
        q.shutdown();
        g_alive--;
        g_torn++;
    }
    static CoalescingQueue<CpuBackend>::Config cfg() {
        CoalescingQueue<CpuBackend>::Config c;
        c.nslots = 4;
        c.lanes = 2;
        c.max_reqs = 64;
        c.linger_us = 50;
        return c;
    }
    // one getChunks-like call: returns 0 and the right digest, or the queue's refusal
    int call(const std::vector<uint8_t>& buf, uint64_t* got) {
        busy++;
        calls++;
        QReq r;
        r.kind = QReq::kChunks;
        r.len = buf.size();
        const int rc = q.run_fill(
            r,
            [&](uint8_t* dst) {
                memcpy(dst, buf.data(), buf.size());
                return 0;
            },
            [&](const QSlot& s, const QReq& rq, int status) -> int {
                if (status) return status;
                *got = (*static_cast<std::vector<uint64_t>*>(s.dev))[rq.idx];
                return 0;
            });
        busy--;
        return rc;
    }
};

typedef Registry<FakeDev> Reg;

static int make(int ord, std::unique_ptr<FakeDev>* d) {
    d->reset(new FakeDev(ord));
    return 0;
}

static int sharing_and_lifecycle() {
    if (g_alive != 0) return 9;
    g_built = 0;
    g_torn = 0;
    Reg reg;
    void *a, *b, *c;
    if (reg.create("K1", {0, 1, 2}, make, &a) || reg.create("K1", {0, 1, 2}, make, &b) ||
        reg.create("K2", {0}, make, &c))
        return 10;
    if (reg.set_of(a) != reg.set_of(b) || reg.set_of(a) == reg.set_of(c) || reg.sets() != 2 || reg.handles() != 3)
        return 11;
    if (reg.refs_of(*reg.set_of(a)) != 2 || g_built != 4) return 12;
    // many callers on a and b while other threads create/destroy more handles of K1 and finally
    // destroy a mid-flight
    std::atomic<bool> stop{false};
    std::atomic<int> bad{0}, refused{0}, ok{0};
    std::vector<std::thread> th;
    for (int t = 0; t < 24; t++)
        th.emplace_back([&, t] {
            std::mt19937_64 rng(77 + t);
            std::vector<uint8_t> buf;
            while (!stop) {
                void* h = (t & 1) ? a : b;
                Reg::Use u(reg, h);
                if (!u.ok()) {
                    refused++;
                    std::this_thread::yield();
                    continue;
                }
                const bool keyed = rng() % 2;
                const uint64_t key = rng() % 16;
                const size_t i = Reg::pick(u.set(), keyed, key);
                if (keyed && i != (size_t)(share_mix64(key) % u.set().ndev())) bad++;
                Reg::Load ld(u.set(), i);
                buf.resize(64 + rng() % 4000);
                for (auto& x : buf) x = (uint8_t)rng();
                uint64_t got = 0;
                const int rc = u.set().devs[i]->call(buf, &got);
                if (rc != 0 || got != digest_of(buf.data(), buf.size()))
                    bad++;
                else
                    ok++;
            }
        });
    for (int t = 0; t < 4; t++)
        th.emplace_back([&] {
            for (int k = 0; k < 30; k++) {
                void* h;
                if (reg.create("K1", {0, 1, 2}, make, &h)) {
                    bad++;
                    return;
                }
                std::this_thread::sleep_for(std::chrono::microseconds(200));
                if (!reg.destroy(h)) bad++;
            }
        });
    std::this_thread::sleep_for(std::chrono::milliseconds(300));
    if (!reg.destroy(a)) return 13;  // waits for a's calls in progress
    std::this_thread::sleep_for(std::chrono::milliseconds(200));
    stop = true;
    for (auto& x : th) x.join();
    if (reg.destroy(a)) return 14;  // a second destroy is refused
    {
        Reg::Use u(reg, a);
        if (u.ok()) return 15;  // calls on a destroyed handle are refused
    }
    if (reg.refs_of(*reg.set_of(b)) != 1 || g_alive != 4) return 16;
    if (!reg.destroy(b)) return 17;  // the last K1 handle: its three devices go
    if (g_alive != 1 || reg.sets() != 1) return 18;
    if (!reg.destroy(c) || g_alive != 0 || reg.sets() != 0 || reg.handles() != 0) return 19;
    printf("sharing: ok=%d refused=%d bad=%d built=%d torn=%d\n", ok.load(), refused.load(), bad.load(), g_built.load(),
           g_torn.load());
    if (bad || ok < 100 || refused == 0) return 20;
    return 0;
}

static int assignment() {
    Reg reg;
    void* h;
    if (reg.create("K3", {0, 1, 2, 3}, make, &h)) return 30;
    SharedSet<FakeDev>& s = *reg.set_of(h);
    std::map<uint64_t, size_t> seen;
    std::vector<int> per(4, 0);
    for (uint64_t key = 0; key < 4000; key++) {
        const size_t i = Reg::pick(s, true, key);
        per[i]++;
        if (Reg::pick(s, true, key) != i) return 31;  // a stream stays on its device
    }
    for (int c : per)
        if (c < 800 || c > 1200) return 32;  // keys spread evenly over the set
    // unkeyed: the least loaded device wins
    {
        Reg::Load l0(s, 0), l1(s, 1), l2(s, 2), l1b(s, 1), l0b(s, 0);
        for (int k = 0; k < 8; k++)
            if (Reg::pick(s, false, 0) != 3) return 33;
    }
    std::vector<int> hits(4, 0);
    for (int k = 0; k < 400; k++) hits[Reg::pick(s, false, 0)]++;
    for (int c : hits)
        if (c != 100) return 34;  // idle set: round robin
    for (uint32_t n : {0u, 1u, 7u, 64u, 1000u, 16384u})
        for (uint32_t k : {1u, 2u, 3u, 8u}) {
            if (share_begin(n, k, 0) != 0 || share_begin(n, k, k) != n) return 35;
            for (uint32_t i = 0; i < k; i++) {
                const uint32_t sz = share_begin(n, k, i + 1) - share_begin(n, k, i);
                if (sz != n / k && sz != n / k + 1) return 36;
            }
        }
    if (!reg.destroy(h)) return 37;
    return 0;
}

static int shutdown_in_flight() {
    for (int rep = 0; rep < 20; rep++) {
        FakeDev d(0);
        std::atomic<int> good{0}, stopped{0}, bad{0};
        std::vector<std::thread> th;
        for (int t = 0; t < 32; t++)
            th.emplace_back([&, t] {
                std::mt19937_64 rng(1000 * rep + t);
                std::vector<uint8_t> buf(100 + rng() % 20000);
                for (int k = 0; k < 50; k++) {
                    for (auto& x : buf) x = (uint8_t)rng();
                    uint64_t got = 0;
                    const int rc = d.call(buf, &got);
                    if (rc == kQueueStopped) {
                        stopped++;
                        return;
                    }
                    if (rc || got != digest_of(buf.data(), buf.size())) bad++;
                    good++;
                }
            });
        std::this_thread::sleep_for(std::chrono::microseconds(200 + 300 * (rep % 5)));
        d.q.shutdown();  // callers are mid-flight: placed requests complete, the rest are refused
        for (auto& x : th) x.join();
        if (bad) return 40;
        if (rep == 0) printf("shutdown: good=%d stopped=%d\n", good.load(), stopped.load());
    }
    return 0;
}

// A call's release racing destroy: the call's Use decrements its handle's count and,
// through the test hook, lingers before unlocking; destroy issued in that window must wait for
// it rather than free the handle under it.
static std::atomic<int> g_hook_phase{0};
static void linger_hook() {
    if (g_hook_phase.load() != 1) return;
    g_hook_phase = 2;  // decremented, handle lock still held
    std::this_thread::sleep_for(std::chrono::milliseconds(100));
    g_hook_phase = 3;
}

static int release_vs_destroy() {
    Reg reg;
    void* h;
    if (reg.create("K4", {0}, make, &h)) return 50;
    Reg::after_release_hook = linger_hook;
    g_hook_phase = 0;
    std::thread caller([&] {
        Reg::Use u(reg, h);
        if (!u.ok()) return;
        g_hook_phase = 1;
    });
    while (g_hook_phase.load() < 2) std::this_thread::yield();
    const bool destroyed = reg.destroy(h);
    const int phase_at_return = g_hook_phase.load();
    caller.join();
    Reg::after_release_hook = nullptr;
    if (!destroyed) return 51;
    if (phase_at_return != 3) return 52;  // destroy returned while the call still held the handle
    if (reg.destroy(h)) return 53;        // the token stays dead
    // tokens are never reused: a new handle never takes a destroyed one's value
    void* h2;
    if (reg.create("K4", {0}, make, &h2)) return 54;
    if (h2 == h || reg.set_of(h) != nullptr) return 55;
    {
        Reg::Use u(reg, h);
        if (u.ok()) return 56;
    }
    if (!reg.destroy(h2) || reg.handles() != 0 || reg.sets() != 0) return 57;
    return 0;
}

// sdfs_cdc_get_chunks_batch's split (Registry::run_shares) at 2 and 8 devices: every buffer is
// processed exactly once, shares are contiguous and balanced, each share runs on its own device
// and thread, and keyed routing (the write stream -> device map) is a stable function of the key.
static int shares_and_routing() {
    for (int n : {2, 8}) {
        Reg reg;
        std::vector<int> ords;
        for (int i = 0; i < n; i++) ords.push_back(i);
        void* h;
        if (reg.create("K5/" + std::to_string(n), ords, make, &h)) return 60;
        SharedSet<FakeDev>& s = *reg.set_of(h);
        for (uint32_t nbuf : {0u, 1u, 63u, 64u, 127u, 128u, 129u, 1000u, 4096u, 16385u}) {
            std::vector<std::atomic<int>> seen(nbuf);
            for (auto& x : seen) x = 0;
            std::vector<std::atomic<int>> per_dev(n);
            for (auto& x : per_dev) x = 0;
            std::mutex tm;
            std::map<std::thread::id, int> threads;
            size_t failed = 99;
            const int rc = Reg::run_shares(
                s, nbuf, 64,
                [&](size_t d, uint32_t b0, uint32_t b1) {
                    {
                        std::lock_guard<std::mutex> lk(tm);
                        threads[std::this_thread::get_id()]++;
                    }
                    if (s.load[d].load() < 1) return 1;  // the share is counted against its device
                    per_dev[d] += (int)(b1 - b0);
                    for (uint32_t b = b0; b < b1; b++) seen[b]++;
                    return 0;
                },
                &failed);
            if (rc) return 61;
            for (uint32_t b = 0; b < nbuf; b++)
                if (seen[b] != 1) return 62;
            const uint32_t k = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(n, nbuf / 64));
            int used = 0;
            for (int d = 0; d < n; d++)
                if (per_dev[d] > 0) used++;
            if (nbuf && used != (int)k) return 63;
            if (k > 1) {
                if (threads.size() != k) return 64;  // one thread per share
                for (uint32_t d = 0; d < k; d++)
                    if (per_dev[d] != (int)(share_begin(nbuf, k, d + 1) - share_begin(nbuf, k, d))) return 65;
            }
            for (int d = 0; d < n; d++)
                if (s.load[d].load() != 0) return 66;  // loads released
        }
        // a failing share is reported with its device
        size_t failed = 99;
        const int rc = Reg::run_shares(
            s, 64u * n, 64, [&](size_t d, uint32_t, uint32_t) { return d == (size_t)n - 1 ? -3 : 0; }, &failed);
        if (rc != -3 || failed != (size_t)n - 1) return 67;
        // keyed routing: stable per key, spread over the set
        std::vector<int> per(n, 0);
        for (uint64_t key = 0; key < 8000; key++) {
            const size_t i = Reg::pick(s, true, key);
            if (i != (size_t)(share_mix64(key) % n) || Reg::pick(s, true, key) != i) return 68;
            per[i]++;
        }
        for (int c : per)
            if (c < 8000 / n * 8 / 10 || c > 8000 / n * 12 / 10) return 69;
        if (!reg.destroy(h)) return 70;
    }
    return 0;
}

int main() {
    int rc = assignment();
    if (!rc) rc = shutdown_in_flight();
    if (!rc) rc = sharing_and_lifecycle();
    if (!rc) rc = release_vs_destroy();
    if (!rc) rc = shares_and_routing();
    printf(rc ? "FAIL %d\n" : "OK\n", rc);
    return rc;
}
