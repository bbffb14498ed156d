// engine_share.h — one process-wide engine per (parameters, device set), shared by every handle
// the C-ABI gives out; free of HIP so that the CPU sanitizer test (tests/cpu/share_tsan.cpp)
// drives exactly this code with a stand-in device engine.
//
// Why: SDFS creates many hash engines, not one.  Static singletons (SparseDedupFile.java:100,
// HashBlobArchive.java:140, FileIOServiceImpl.java:152), a throwaway one for the blank hash
// (HashStore.java:68), and a pool that grows to the number of concurrent write-accelerator
// callers (HashFunctionPool.borrowObject, HashFunctionPool.java:73-86, WritableCacheBuffer.java:640,
// 779).  If each `new HipVariableSha256HashEngine` owned a native engine, every instance would pin
// its own staging and run its own coalescing queue, and calls made on different instances would
// never share a GPU pass.  So sdfs_cdc_create returns a small HANDLE; handles with equal
// parameters and device sets share one SharedSet holding one device engine (one coalescing queue,
// one set of lanes) per GPU of the set.
//
// Lifecycle: a handle counts its calls in progress.  Destroying a handle first makes it unusable
// for new calls (they fail with EINVAL), then waits for its calls in progress, then drops its
// reference; the last reference tears the device engines down (no call can be in progress on any
// of them then).  The reference's destroy() is a no-op (VariableSha256HashEngine.java:96-99);
// HashFunctionPool.destroyObject (:98-100) may call it while another thread still uses the
// engine — here that call simply finishes first.
//
// Devices: host-buffer calls go to one device of the set.  A call that names a write stream
// (getChunks(buf, uuid): a key derived from the uuid) goes to device key mod N, so one stream's
// buffers stay on one GPU ("whole streams round-robin"); a call without a key goes
// to the device with the fewest calls in progress (ties: round robin).
#pragma once

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

namespace sdfs {

template <class Dev>
struct SharedSet {
    std::string key;
    std::vector<std::unique_ptr<Dev>> devs;  // one per device of the set, in set order
    std::vector<int> ordinals;               // HIP ordinal of devs[i]
    std::unique_ptr<std::atomic<int>[]> load;  // host calls in progress per device
    std::atomic<uint64_t> rr{0};
    int refs = 0;  // live handles (registry lock)
    // set-wide extras of the device side (the RCCL communicators of the record exchange); declared
    // after devs, so they are released before the device engines
    std::mutex coll_mu;
    std::shared_ptr<void> coll;
    size_t ndev() const { return devs.size(); }
};

template <class Dev>
struct Handle {
    SharedSet<Dev>* set = nullptr;
    int inflight = 0;  // calls in progress (guarded by mu)
    std::mutex mu;
    std::condition_variable cv;  // inflight reached 0
};

inline uint64_t share_mix64(uint64_t x) {  // splitmix64 finaliser: spreads stream keys over devices
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// Contiguous shares of n buffers over k devices (first n % k devices take one more):
// device i gets [begin(i), begin(i+1)).
inline uint32_t share_begin(uint32_t n, uint32_t k, uint32_t i) {
    const uint32_t q = n / k, r = n % k;
    return i * q + (i < r ? i : r);
}

template <class Dev>
class Registry {
  public:
    using H = Handle<Dev>;
    using S = SharedSet<Dev>;

    // A handle for (key, ordinals): shares the set of that key, or builds it with
    // make(ordinal, std::unique_ptr<Dev>*) -> status (0 = ok) for every ordinal.  Creation and
    // teardown are serialised among themselves, not against calls.
    template <class Make>
    int create(const std::string& key, const std::vector<int>& ordinals, Make&& make, void** out) {
        *out = nullptr;
        std::lock_guard<std::mutex> life(life_mu_);
        {
            std::lock_guard<std::mutex> lk(mu_);
            auto it = sets_.find(key);
            if (it != sets_.end()) {
                it->second->refs++;
                *out = new_handle(it->second);
                return 0;
            }
        }
        auto* s = new S();
        s->key = key;
        s->ordinals = ordinals;
        s->load.reset(new std::atomic<int>[ordinals.size()]);
        for (size_t i = 0; i < ordinals.size(); i++) s->load[i] = 0;
        for (int ord : ordinals) {
            std::unique_ptr<Dev> d;
            const int rc = make(ord, &d);
            if (rc) {
                s->devs.clear();  // engines already built are torn down here
                delete s;
                return rc;
            }
            s->devs.push_back(std::move(d));
        }
        std::lock_guard<std::mutex> lk(mu_);
        s->refs = 1;
        sets_[key] = s;
        *out = new_handle(s);
        return 0;
    }

    // Ends a handle: no new calls, wait for the ones in progress, drop the reference (the last
    // one tears the set down).  false: not a live handle (never issued, or already destroyed).
    bool destroy(const void* tok) {
        H* h = nullptr;
        {
            std::lock_guard<std::mutex> lk(mu_);
            auto it = live_.find(reinterpret_cast<uintptr_t>(tok));
            if (it == live_.end()) return false;
            h = it->second;
            live_.erase(it);  // no Use can start on h from here on
        }
        {
            // Use::~Use decrements under h->mu and touches h no more after unlocking it, so once
            // this wait returns nothing else can reach h
            std::unique_lock<std::mutex> lk(h->mu);
            h->cv.wait(lk, [&] { return h->inflight == 0; });
        }
        std::lock_guard<std::mutex> life(life_mu_);
        S* dead = nullptr;
        {
            std::lock_guard<std::mutex> lk(mu_);
            if (--h->set->refs == 0) {
                dead = h->set;
                sets_.erase(dead->key);
            }
        }
        delete h;
        delete dead;  // device engines torn down outside the call path's lock
        return true;
    }

    // A call in progress on a handle (RAII): ok() false when the token is not a live handle.
    class Use {
      public:
        Use(Registry& r, const void* tok) {
            std::lock_guard<std::mutex> lk(r.mu_);
            auto it = r.live_.find(reinterpret_cast<uintptr_t>(tok));
            if (it == r.live_.end()) return;
            h_ = it->second;
            std::lock_guard<std::mutex> hl(h_->mu);
            h_->inflight++;
        }
        ~Use() {
            if (!h_) return;
            std::lock_guard<std::mutex> lk(h_->mu);
            if (--h_->inflight == 0) h_->cv.notify_all();
            if (after_release_hook) after_release_hook();  // tests: widen the window before unlock
        }
        Use(const Use&) = delete;
        Use& operator=(const Use&) = delete;
        bool ok() const { return h_ != nullptr; }
        S& set() const { return *h_->set; }

      private:
        H* h_ = nullptr;
    };

    // Test hook run by ~Use after its decrement, still holding the handle's lock (null in the
    // product).
    static inline void (*after_release_hook)() = nullptr;

    // Device for a host call: key mod N for keyed calls, else the least-loaded device.
    static size_t pick(S& s, bool keyed, uint64_t key) {
        const size_t n = s.ndev();
        if (n <= 1) return 0;
        if (keyed) return (size_t)(share_mix64(key) % n);
        const size_t start = (size_t)(s.rr.fetch_add(1) % n);
        size_t best = start;
        for (size_t k = 1; k < n; k++) {
            const size_t i = (start + k) % n;
            if (s.load[i].load() < s.load[best].load()) best = i;
        }
        return best;
    }

    // Counts a host call against a device while it runs (RAII).
    class Load {
      public:
        Load(S& s, size_t i) : c_(s.load[i]) { c_++; }
        ~Load() { c_--; }
        Load(const Load&) = delete;
        Load& operator=(const Load&) = delete;

      private:
        std::atomic<int>& c_;
      };

    // One batch of nbuf independent buffers over the set: contiguous shares, one per device, at
    // least min_share buffers each, run concurrently (the calling thread takes share 0) as
    // run(device index, first buffer, end buffer) -> status.  A batch too small to split goes
    // whole to the least-loaded device.  Returns 0, or the first failing share's status with
    // *failed set to its device index.
    template <class Run>
    static int run_shares(S& s, uint32_t nbuf, uint32_t min_share, Run&& run, size_t* failed) {
        *failed = 0;
        const uint64_t want = min_share ? nbuf / min_share : nbuf;
        const uint32_t k = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(s.ndev(), want));
        if (k == 1) {
            const size_t i = pick(s, false, 0);
            Load ld(s, i);
            *failed = i;
            return run(i, 0u, nbuf);
        }
        std::vector<int> rcs(k, 0);
        auto share = [&](uint32_t d) {
            Load ld(s, d);
            rcs[d] = run((size_t)d, share_begin(nbuf, k, d), share_begin(nbuf, k, d + 1));
        };
        std::vector<std::thread> th;
        for (uint32_t d = 1; d < k; d++) th.emplace_back(share, d);
        share(0);
        for (auto& t : th) t.join();
        for (uint32_t d = 0; d < k; d++)
            if (rcs[d]) {
                *failed = d;
                return rcs[d];
            }
        return 0;
    }

    // The set behind a live token (tests); null when the token is not live.
    S* set_of(const void* tok) {
        std::lock_guard<std::mutex> lk(mu_);
        auto it = live_.find(reinterpret_cast<uintptr_t>(tok));
        return it == live_.end() ? nullptr : it->second->set;
    }

    // handles sharing a set (statistics, tests)
    int refs_of(const S& s) {
        std::lock_guard<std::mutex> lk(mu_);
        return s.refs;
    }
    size_t sets() {
        std::lock_guard<std::mutex> lk(mu_);
        return sets_.size();
    }
    size_t handles() {
        std::lock_guard<std::mutex> lk(mu_);
        return live_.size();
    }

  private:
    // Tokens are never reused (a 64-bit counter), so a stale token from a destroyed handle can
    // never name a later handle: every call on it fails with EINVAL, a second destroy too.
    void* new_handle(S* s) {  // registry lock held
        H* h = new H();
        h->set = s;
        const uintptr_t tok = (++next_tok_) << 4;  // nonzero, 16-byte "aligned" like a pointer
        live_.emplace(tok, h);
        return reinterpret_cast<void*>(tok);
    }

    std::mutex life_mu_;  // create / teardown
    std::mutex mu_;       // live handles, sets, reference counts
    uintptr_t next_tok_ = 0;
    std::map<uintptr_t, H*> live_;
    std::map<std::string, S*> sets_;
};

}  // namespace sdfs
