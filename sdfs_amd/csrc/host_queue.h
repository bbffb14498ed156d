// host_queue.h — host-side concurrency of the drop-in boundary, free of HIP so that the CPU
// sanitizer test (tests/cpu/queue_tsan.cpp, run under -fsanitize=thread) exercises exactly this
// code with a CPU backend.
//
// SDFS calls the hash engine synchronously, one write buffer per call, from many flush threads
// that share ONE static engine (SparseDedupFile.java:100,432; the flush pools are
// Main.writeThreads wide, WritableCacheBuffer.java:100-104; the write-accelerator path calls
// getChunks from the same pool, WritableCacheBuffer.java:640-643).  A GPU round trip per
// 256 KiB buffer would leave the device idle, so concurrent calls are coalesced:
//
//   caller thread                          dispatcher thread          completer thread
//   reserve space in the OPEN slot  ──┐
//   copy its bytes into pinned staging │    OPEN slot has requests
//   (in parallel with other callers)   └─►  and < max_inflight in
//   wait for its request's `done`           flight: CLOSE it, wait
//                                           for the copies, launch ─► wait for the device,
//   copy its results out of the slot ◄───────────────────────────────  mark every request done
//   last reader frees the slot
//
// The batch size adapts to the load: an idle engine launches a request at once; under load the
// OPEN slot fills while `max_inflight` batches are on the device.  Requests that do not fit a
// slot bypass the queue (the caller handles them directly).
//
// CopyPool: a small persistent thread pool for host memcpy into pinned staging
// (sdfs_cdc_get_chunks_batch from pageable memory).
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

namespace sdfs {

// ---------------------------------------------------------------------------------------------
// CopyPool
// ---------------------------------------------------------------------------------------------
struct CopyPiece {
    uint8_t* dst;
    const uint8_t* src;
    size_t n;
};

class CopyPool {
  public:
    explicit CopyPool(int workers) {
        for (int i = 0; i < workers; i++) th_.emplace_back([this] { loop(); });
    }
    ~CopyPool() {
        {
            std::lock_guard<std::mutex> l(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    CopyPool(const CopyPool&) = delete;
    CopyPool& operator=(const CopyPool&) = delete;

    // Copies every piece; the calling thread works too.  One job at a time per pool (callers
    // serialise on the engine mutex).
    void run(const std::vector<CopyPiece>& p) {
        if (th_.empty() || p.size() < 2) {
            for (const auto& x : p) memcpy(x.dst, x.src, x.n);
            return;
        }
        {
            std::lock_guard<std::mutex> l(m_);
            job_ = &p;
            next_.store(0);
            active_ = th_.size();
            gen_++;
        }
        cv_.notify_all();
        drain(p);
        std::unique_lock<std::mutex> l(m_);
        done_.wait(l, [&] { return active_ == 0; });
        job_ = nullptr;
    }

  private:
    void drain(const std::vector<CopyPiece>& p) {
        for (size_t i; (i = next_.fetch_add(1)) < p.size();) memcpy(p[i].dst, p[i].src, p[i].n);
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            const std::vector<CopyPiece>* job;
            {
                std::unique_lock<std::mutex> l(m_);
                cv_.wait(l, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
                job = job_;
            }
            drain(*job);
            std::lock_guard<std::mutex> l(m_);
            if (--active_ == 0) done_.notify_all();
        }
    }
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, done_;
    const std::vector<CopyPiece>* job_ = nullptr;
    std::atomic<size_t> next_{0};
    size_t active_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

// ---------------------------------------------------------------------------------------------
// Coalescing request queue
// ---------------------------------------------------------------------------------------------
// One caller's request.  kChunks = getChunks(buf) (the bytes go to the slot's chunk region, in
// request order, at 64-byte aligned offsets); kHash = getHash(data) (the hash region, filled
// from the top of the slot down, 16-byte aligned).
struct QReq {
    enum Kind : uint8_t { kChunks = 0, kHash = 1 };
    Kind kind = kChunks;
    const uint8_t* src = nullptr;
    uint64_t len = 0;
    // placement, set when the request joins a slot
    int slot = -1;
    uint32_t idx = 0;   // index among the slot's requests of its kind
    uint64_t off = 0;   // staging offset of its bytes
    // completion
    int status = 0;
    bool done = false;
};

struct QSlot {
    enum State { kFree, kOpen, kClosed, kFlight, kDone };
    State state = kFree;
    uint8_t* in = nullptr;  // staging (the backend allocates it: pinned host memory on the GPU)
    uint64_t cap = 0;       // staging bytes
    uint64_t lo = 0;        // chunk region [0, lo)
    uint64_t hi = 0;        // hash region [hi, cap)
    std::vector<QReq*> chunks, hashes;
    uint32_t uniform_len = 0;  // every chunk request has this length (0 = mixed)
    uint64_t max_chunk_len = 0;
    int copying = 0;  // callers still copying their bytes in
    int readers = 0;  // callers yet to copy their results out
    int status = 0;
    uint64_t seq = 0;
    void* dev = nullptr;  // backend state of this slot
    size_t nreq() const { return chunks.size() + hashes.size(); }
};

inline uint64_t qalign(uint64_t x, uint64_t a) { return (x + a - 1) & ~(a - 1); }

// queue-level statuses (outside the backend's status range)
constexpr int kQueueStopped = -1000;  // the queue is not running
constexpr int kQueueTooBig = -1001;   // the request exceeds the per-request limit (accepts() is false)

// Backend concept:
//   int  prepare(QSlot&)   allocate s.in / s.cap and s.dev (called once per slot, queue lock held;
//                          on failure the queue calls release on every slot)
//   int  launch(QSlot&)    enqueue transfer + compute of a CLOSED slot (dispatcher thread)
//   int  wait(QSlot&)      block until that work completed (completer thread)
//   void release(QSlot&)   free what prepare allocated
// launch and wait run without the queue lock.
template <class Backend>
class CoalescingQueue {
  public:
    struct Config {
        int nslots = 4;           // staging slots (one open, up to max_inflight in flight, readers)
        int max_inflight = 2;     // batches on the device at once
        uint32_t max_reqs = 1024; // requests per slot (the backend sizes its result image for this)
        uint64_t max_req_bytes = 0;  // larger requests bypass the queue (0 = cap / 2)
    };

    CoalescingQueue(Backend& b, Config c) : b_(b), c_(c), slots_(c.nslots) {}
    ~CoalescingQueue() { shutdown(); }
    CoalescingQueue(const CoalescingQueue&) = delete;
    CoalescingQueue& operator=(const CoalescingQueue&) = delete;

    // true when a request of `len` bytes is served by the queue (else the caller goes direct)
    bool accepts(uint64_t len) {
        std::lock_guard<std::mutex> lk(m_);
        return prepared_ && len <= max_req_;
    }

    // Prepare the slots (idempotent); returns the backend's status.
    int start() {
        std::lock_guard<std::mutex> lk(m_);
        if (prepared_) return 0;
        for (auto& s : slots_) {
            const int rc = b_.prepare(s);
            if (rc) {
                for (auto& t : slots_)
                    if (t.in || t.dev) b_.release(t);
                return rc;
            }
        }
        max_req_ = c_.max_req_bytes ? c_.max_req_bytes : slots_[0].cap / 2;
        prepared_ = true;
        stop_ = false;
        disp_ = std::thread([this] { dispatcher(); });
        comp_ = std::thread([this] { completer(); });
        return 0;
    }

    // Stops the threads (after the in-flight batches completed) and releases the slots.  No
    // request may be in progress.
    void shutdown() {
        {
            std::lock_guard<std::mutex> lk(m_);
            if (!prepared_) return;
            stop_ = true;
        }
        cv_disp_.notify_all();
        cv_comp_.notify_all();
        if (disp_.joinable()) disp_.join();
        if (comp_.joinable()) comp_.join();
        std::lock_guard<std::mutex> lk(m_);
        for (auto& s : slots_) b_.release(s);
        prepared_ = false;
    }

    // Runs one request to completion.  `read(slot, req, status)` runs on the calling thread after
    // the batch completed (the slot stays allocated to it until `read` returns): it copies the
    // caller's results out, or reports the batch's failure `status`; its return value is run's.
    template <class ReadFn>
    int run(QReq& r, ReadFn&& read) {
        std::unique_lock<std::mutex> lk(m_);
        if (!prepared_ || stop_) return kQueueStopped;
        const uint64_t need = r.kind == QReq::kChunks ? qalign(r.len, 64) : qalign(r.len, 16);
        if (r.len > max_req_) return kQueueTooBig;  // callers check accepts() first
        QSlot* s = nullptr;
        for (;;) {
            if (open_ >= 0) {
                QSlot& o = slots_[open_];
                if (o.nreq() < c_.max_reqs && o.lo + need <= o.hi) {
                    s = &o;
                    break;
                }
            }
            if (open_ < 0) {  // open a free slot
                for (size_t i = 0; i < slots_.size(); i++)
                    if (slots_[i].state == QSlot::kFree) {
                        QSlot& f = slots_[i];
                        f.state = QSlot::kOpen;
                        f.lo = 0;
                        f.hi = f.cap;
                        f.chunks.clear();
                        f.hashes.clear();
                        f.uniform_len = 0;
                        f.max_chunk_len = 0;
                        f.copying = f.readers = 0;
                        f.status = 0;
                        f.seq = ++seq_;
                        open_ = (int)i;
                        break;
                    }
                if (open_ >= 0) continue;
            }
            // the open slot is full (the dispatcher launches it as soon as it may) or every slot
            // is busy: wait for space
            cv_disp_.notify_one();
            cv_space_.wait(lk);
            if (stop_) return kQueueStopped;
        }
        r.slot = open_;
        r.done = false;
        r.status = 0;
        if (r.kind == QReq::kChunks) {
            r.off = s->lo;
            s->lo += need;
            r.idx = (uint32_t)s->chunks.size();
            if (s->chunks.empty())
                s->uniform_len = (uint32_t)r.len;
            else if (s->uniform_len != r.len)
                s->uniform_len = 0;
            if (r.len > s->max_chunk_len) s->max_chunk_len = r.len;
            s->chunks.push_back(&r);
        } else {
            s->hi -= need;
            r.off = s->hi;
            r.idx = (uint32_t)s->hashes.size();
            s->hashes.push_back(&r);
        }
        s->copying++;
        cv_disp_.notify_one();
        lk.unlock();
        if (r.len) memcpy(s->in + r.off, r.src, r.len);
        lk.lock();
        if (--s->copying == 0) cv_disp_.notify_all();
        cv_done_.wait(lk, [&] { return r.done; });
        lk.unlock();
        const int rc = read(*s, r, r.status);
        lk.lock();
        if (--s->readers == 0) {
            s->state = QSlot::kFree;
            cv_space_.notify_all();
        }
        return rc;
    }

    // statistics (tests, bench)
    uint64_t batches() {
        std::lock_guard<std::mutex> lk(m_);
        return launched_;
    }
    uint64_t requests() {
        std::lock_guard<std::mutex> lk(m_);
        return served_;
    }

  private:
    void dispatcher() {
        std::unique_lock<std::mutex> lk(m_);
        for (;;) {
            cv_disp_.wait(lk, [&] {
                return stop_ || (open_ >= 0 && slots_[open_].nreq() > 0 && inflight_ < c_.max_inflight);
            });
            if (stop_) break;
            QSlot& s = slots_[open_];
            s.state = QSlot::kClosed;
            open_ = -1;
            inflight_++;
            cv_space_.notify_all();  // waiting callers may open the next slot now
            cv_disp_.wait(lk, [&] { return s.copying == 0; });
            s.readers = (int)s.nreq();
            launched_++;
            served_ += s.nreq();
            lk.unlock();
            const int rc = b_.launch(s);
            lk.lock();
            s.status = rc;
            s.state = QSlot::kFlight;
            flight_.push_back(&s);
            cv_comp_.notify_one();
        }
    }

    void completer() {
        std::unique_lock<std::mutex> lk(m_);
        for (;;) {
            cv_comp_.wait(lk, [&] { return !flight_.empty() || (stop_ && inflight_ == 0); });
            if (flight_.empty()) break;  // stop_ and nothing in flight
            QSlot* s = flight_.front();
            flight_.pop_front();
            const int launched_rc = s->status;
            lk.unlock();
            const int rc = b_.wait(*s);  // always: drains whatever a failed launch enqueued
            lk.lock();
            s->status = launched_rc ? launched_rc : rc;
            s->state = QSlot::kDone;
            inflight_--;
            for (QReq* q : s->chunks) {
                q->status = s->status;
                q->done = true;
            }
            for (QReq* q : s->hashes) {
                q->status = s->status;
                q->done = true;
            }
            cv_done_.notify_all();
            cv_disp_.notify_all();
        }
    }

    Backend& b_;
    Config c_;
    std::vector<QSlot> slots_;
    std::mutex m_;
    std::condition_variable cv_disp_, cv_comp_, cv_done_, cv_space_;
    std::deque<QSlot*> flight_;
    std::thread disp_, comp_;
    int open_ = -1;
    int inflight_ = 0;
    bool prepared_ = false;
    bool stop_ = false;
    uint64_t max_req_ = 0;
    uint64_t seq_ = 0;
    uint64_t launched_ = 0, served_ = 0;
};

}  // namespace sdfs
