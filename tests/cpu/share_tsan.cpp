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
//      kQueueStopped, nobody hangs.
// Test infrastructure only.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <map>
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
    Handle<FakeDev>*a, *b, *c;
    if (reg.create("K1", {0, 1, 2}, make, &a) || reg.create("K1", {0, 1, 2}, make, &b) ||
        reg.create("K2", {0}, make, &c))
        return 10;
    if (a->set != b->set || a->set == c->set || reg.sets() != 2 || reg.handles() != 3) return 11;
    if (reg.refs_of(*a->set) != 2 || g_built != 4) return 12;
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
                Handle<FakeDev>* h = (t & 1) ? a : b;
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
                Handle<FakeDev>* h;
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
    if (reg.refs_of(*b->set) != 1 || g_alive != 4) return 16;
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
    Handle<FakeDev>* h;
    if (reg.create("K3", {0, 1, 2, 3}, make, &h)) return 30;
    SharedSet<FakeDev>& s = *h->set;
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

int main() {
    int rc = assignment();
    if (!rc) rc = shutdown_in_flight();
    if (!rc) rc = sharing_and_lifecycle();
    printf(rc ? "FAIL %d\n" : "OK\n", rc);
    return rc;
}
