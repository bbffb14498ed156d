// queue_tsan.cpp — CPU stress of the engine's host-side concurrency (sdfs_amd/csrc/host_queue.h)
// under ThreadSanitizer: the coalescing queue that serves concurrent getChunks/getHash callers
// (SparseDedupFile.java:100,432 — one engine shared by every flush thread), driven by a CPU
// backend that stands in for the GPU (launch = nothing, wait = compute every request's result
// into the slot's result image), and the CopyPool used by the batched host path.
//
// Checks: every caller gets exactly its own result (a per-request function of its bytes), the
// queue really coalesces (fewer batches than requests), slots are reused, and a backend failure
// reaches every request of the failing batch.  The backend completes getChunks requests early
// (Backend::poll), so callers leave while their batch is still running, and a slot is reused only
// once its batch is done and its last caller has left.  Test infrastructure only.
#include <algorithm>
#include <atomic>
#include <cassert>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <thread>
#include <vector>

#include "../../sdfs_amd/csrc/host_queue.h"

using namespace sdfs;

static uint64_t digest_of(const uint8_t* p, uint64_t n, uint64_t salt) {
    uint64_t h = 1469598103934665603ull ^ salt;
    for (uint64_t i = 0; i < n; i++) h = (h ^ p[i]) * 1099511628211ull;
    return h ^ n;
}

struct CpuSlot {
    std::vector<uint64_t> chunk_res, hash_res;
    size_t next = 0;  // early completion: chunk requests computed so far
    bool fail_next = false;
};

struct CpuBackend {
    uint64_t slot_bytes;
    std::atomic<int> fail_batches{0};  // number of upcoming batches to fail
    std::atomic<int> launches{0};
    std::atomic<int> early{0};  // chunk requests completed before their batch

    int prepare(QSlot& s) {
        s.in = static_cast<uint8_t*>(malloc(slot_bytes));
        s.cap = slot_bytes;
        s.dev = new CpuSlot();
        return s.in ? 0 : -4;
    }
    void release(QSlot& s) {
        free(s.in);
        s.in = nullptr;
        delete static_cast<CpuSlot*>(s.dev);
        s.dev = nullptr;
    }
    bool admits(const QSlot& s, const QReq& r) {
        (void)r;
        return s.chunks.size() < 200;  // a result-image limit below max_reqs (exercises the hook)
    }
    int launch(QSlot& s, int lane) {
        (void)lane;
        launches++;
        auto* d = static_cast<CpuSlot*>(s.dev);
        int f = fail_batches.load();
        d->fail_next = false;
        while (f > 0 && !fail_batches.compare_exchange_weak(f, f - 1)) {
        }
        if (f > 0) d->fail_next = true;
        // result arrays sized once per batch: early-completed callers read them while the rest
        // of the batch is still being computed
        d->chunk_res.assign(s.chunks.size(), 0);
        d->hash_res.assign(s.hashes.size(), 0);
        d->next = 0;
        // a "device" that takes a moment, so batches overlap the callers' copies
        std::this_thread::sleep_for(std::chrono::microseconds(50));
        return 0;
    }
    void chunk_result(QSlot& s, CpuSlot* d, size_t i) {
        const QReq* q = s.chunks[i];
        assert(q->off % 64 == 0 && q->off + q->len <= s.lo);
        d->chunk_res[i] = digest_of(s.in + q->off, q->len, 1);
    }
    // early completion (host_queue.h Backend::poll): one more chunk request per call, in a
    // scrambled order; a batch that is going to fail completes nothing early (as on the GPU,
    // where a failed launch sets no ready word)
    int poll(QSlot& s, uint8_t* ready, bool* finished) {
        auto* d = static_cast<CpuSlot*>(s.dev);
        const size_t n = s.chunks.size();
        if (d->fail_next || d->next >= n) {
            *finished = true;
            return wait(s);
        }
        const size_t i = (d->next * 7 + 3) % n;  // a permutation whenever gcd(7, n) == 1
        d->next++;
        if (!ready[i] && std::__gcd<size_t>(7, n) == 1) {
            chunk_result(s, d, i);
            ready[i] = 1;
            early++;
        }
        *finished = false;
        return 0;
    }
    int wait(QSlot& s) {
        auto* d = static_cast<CpuSlot*>(s.dev);
        if (d->fail_next) return -3;
        for (size_t i = 0; i < s.chunks.size(); i++)
            if (d->chunk_res[i] == 0) chunk_result(s, d, i);  // those not completed early
        for (size_t j = 0; j < s.hashes.size(); j++) {
            const QReq* q = s.hashes[j];
            assert(q->off % 16 == 0 && q->off >= s.hi && q->off + q->len <= s.cap);
            d->hash_res[j] = digest_of(s.in + q->off, q->len, 2);
        }
        return 0;
    }
};

static int stress(int nthreads, int per_thread, uint64_t slot_bytes, int fail_batches) {
    CpuBackend b;
    b.slot_bytes = slot_bytes;
    CoalescingQueue<CpuBackend>::Config c;
    c.nslots = 5;
    c.lanes = 3;
    c.max_reqs = 256;
    c.linger_us = 100;
    CoalescingQueue<CpuBackend> q(b, c);
    if (q.start() != 0) return 1;
    b.fail_batches = fail_batches;
    std::atomic<int> bad{0}, failed{0};
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; t++)
        th.emplace_back([&, t] {
            std::mt19937_64 rng(1234 + t);
            std::vector<uint8_t> buf(slot_bytes / 2);
            for (int k = 0; k < per_thread; k++) {
                const bool hash = (rng() % 5) == 0;
                uint64_t n = rng() % 3 == 0 ? rng() % (slot_bytes / 2 + 1) : 262144 - (rng() % 2) * 64;
                n = std::min<uint64_t>(n, slot_bytes / 2);
                for (uint64_t i = 0; i < n; i += 64) buf[i] = (uint8_t)rng();
                QReq r;
                r.kind = hash ? QReq::kHash : QReq::kChunks;
                r.src = buf.data();
                r.len = n;
                const uint64_t want = digest_of(buf.data(), n, hash ? 2 : 1);
                uint64_t got = 0;
                const int rc = q.run(r, [&](const QSlot& s, const QReq& rq, int status) -> int {
                    if (status) return status;
                    const auto* d = static_cast<const CpuSlot*>(s.dev);
                    got = hash ? d->hash_res[rq.idx] : d->chunk_res[rq.idx];
                    return 0;
                });
                if (rc == -3)
                    failed++;
                else if (rc != 0 || got != want)
                    bad++;
            }
        });
    for (auto& x : th) x.join();
    const uint64_t batches = q.batches(), reqs = q.requests();
    q.shutdown();
    printf("threads=%d reqs=%llu batches=%llu failed=%d bad=%d early=%d\n", nthreads, (unsigned long long)reqs,
           (unsigned long long)batches, failed.load(), bad.load(), b.early.load());
    if (bad) return 2;
    if (reqs != (uint64_t)nthreads * per_thread) return 3;
    if (fail_batches == 0 && failed) return 4;
    if (fail_batches > 0 && failed == 0) return 5;
    if (nthreads >= 8 && batches >= reqs) return 6;  // concurrent callers must share batches
    if (nthreads >= 8 && b.early == 0) return 8;      // early completion must have happened
    return 0;
}

static int copy_pool() {
    CopyPool pool(5);
    std::vector<uint8_t> src(8 << 20), dst(8 << 20);
    for (size_t i = 0; i < src.size(); i++) src[i] = (uint8_t)(i * 131 + 7);
    for (int rep = 0; rep < 20; rep++) {
        std::fill(dst.begin(), dst.end(), 0);
        std::vector<CopyPiece> pieces;
        for (size_t o = 0; o < src.size(); o += 300000)
            pieces.push_back({dst.data() + o, src.data() + o, std::min<size_t>(300000, src.size() - o)});
        pool.run(pieces);
        if (dst != src) return 7;
    }
    return 0;
}

int main() {
    int rc = copy_pool();
    if (!rc) rc = stress(1, 40, 1 << 20, 0);
    if (!rc) rc = stress(64, 12, 1 << 20, 0);
    if (!rc) rc = stress(128, 6, 4 << 20, 0);
    if (!rc) rc = stress(32, 10, 1 << 20, 3);
    printf(rc ? "FAIL %d\n" : "OK\n", rc);
    return rc;
}
