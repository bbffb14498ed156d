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
//   caller thread                          dispatcher thread          completer thread (per lane)
//   reserve space in the OPEN slot  ──┐
//   copy its bytes into pinned staging │    OPEN slot ready and a
//   (in parallel with other callers)   └─►  device lane idle: CLOSE
//   wait for its request's `done`           it, wait for the copies,
//                                           launch on that lane ────► wait for the device,
//   copy its results out of the slot ◄───────────────────────────────  mark every request done
//   last reader frees the slot
//
// The batch size adapts to the load: an idle engine launches a request at once; under load the
// OPEN slot fills while the lanes are busy (policy below).  Requests that do not fit a slot
// bypass the queue (the caller handles them directly).
//
// CopyPool: a small persistent thread pool for host memcpy into pinned staging
// (sdfs_cdc_get_chunks_batch from pageable memory).
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>
#include <type_traits>
#include <utility>
#include <vector>
#ifdef __linux__
#include <sys/prctl.h>
#endif

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
    // admission (set by the queue for a caller that waited for room: 1 = placed, < 0 = refused)
    int admit = 0;
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
    bool full = false;  // cannot take another request of the largest admitted size
    int copying = 0;  // callers still copying their bytes in
    int readers = 0;  // callers yet to copy their results out
    int status = 0;
    uint64_t seq = 0;
    std::chrono::steady_clock::time_point t_open, t_close, t_launch, t_done;  // batch timeline
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
//   bool admits(const QSlot&, const QReq&)  whether the slot's result image has room for one more
//                          request (queue lock held; must be true for an empty slot)
//   int  launch(QSlot&, int lane)  enqueue transfer + compute of a CLOSED slot on device lane
//                          `lane` (one stream per lane; dispatcher thread)
//   int  wait(QSlot&)      block until that work completed (the lane's completer thread)
//   void release(QSlot&)   free what prepare allocated
//   int  poll(QSlot&, uint8_t* ready, bool* finished)   OPTIONAL, non-blocking progress of a
//                          launched slot: sets ready[i] = 1 for each getChunks request i (the
//                          slot's chunks[i]) whose results are final before the whole batch is
//                          (its buffer's last chunk was fingerprinted); *finished = true once the
//                          batch completed, and then the return value is its status as wait's.
//                          A backend with poll lets each caller go as soon as its own buffer is
//                          done instead of when the batch's longest chunk is.
// launch, wait and poll run without the queue lock.
//
// Dispatch policy.  A batch costs the device about the same time whatever its size (its
// longest chunk's serial SHA-256 chain sets it), so batches should be as large as the callers
// allow, but no caller should wait long: the dispatcher launches the OPEN slot onto an idle lane
// when nothing is in flight, or when it holds its share of the callers (active callers /
// lanes), or when it is full, or when its first request has waited `linger_us`.
template <class B, class = void>
struct has_poll : std::false_type {};
template <class B>
struct has_poll<B, std::void_t<decltype(std::declval<B&>().poll(std::declval<QSlot&>(), (uint8_t*)nullptr, (bool*)nullptr))>>
    : std::true_type {};

template <class Backend>
class CoalescingQueue {
  public:
    struct Config {
        int nslots = 8;            // staging slots (one open, up to `lanes` in flight, readers)
        int lanes = 4;             // batches on the device at once, one stream each
        uint32_t max_reqs = 1024;  // requests per slot (the backend sizes its result image for this)
        uint64_t max_req_bytes = 0;  // larger requests bypass the queue (0 = cap / 2)
        uint32_t linger_us = 250;  // longest a request waits for company while a batch is in flight
        uint32_t poll_us = 10;     // early completion (Backend::poll): the completer's poll period
        uint32_t share_div = 1;    // a slot goes once it holds active callers / (lanes x share_div)
    };

    CoalescingQueue(Backend& b, Config c)
        : b_(b), c_(c), slots_(c.nslots), flight_(c.lanes), comp_cv_(c.lanes),
          lane_busy_(c.lanes, 0), early_(c.lanes), wake_(c.lanes) {}
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
        disp_done_ = false;
        disp_ = std::thread([this] { dispatcher(); });
        for (int l = 0; l < c_.lanes; l++) comp_.emplace_back([this, l] { completer(l); });
        return 0;
    }

    // Stops the queue: callers that arrive from now on, and callers still waiting for room, get
    // kQueueStopped; every request already placed in a slot is launched and completed (the open
    // slot included), its caller reads its result; then the threads end and, once the last
    // caller has left run(), the slots are released.
    void shutdown() {
        {
            std::lock_guard<std::mutex> lk(m_);
            if (!prepared_) return;
            stop_ = true;
        }
        cv_disp_.notify_all();
        for (auto& cv : comp_cv_) cv.notify_all();
        for (auto& cv : cv_admit_) cv.notify_all();
        if (disp_.joinable()) disp_.join();
        for (auto& t : comp_)
            if (t.joinable()) t.join();
        comp_.clear();
        std::unique_lock<std::mutex> lk(m_);
        idle_cv_.wait(lk, [&] { return active_ == 0; });
        for (auto& s : slots_) b_.release(s);
        prepared_ = false;
    }

    // Runs one request to completion.  `read(slot, req, status)` runs on the calling thread after
    // the batch completed (the slot stays allocated to it until `read` returns): it copies the
    // caller's results out, or reports the batch's failure `status`; its return value is run's.
    template <class ReadFn>
    int run(QReq& r, ReadFn&& read) {
        return run_fill(
            r,
            [&r](uint8_t* dst) {
                if (r.len) memcpy(dst, r.src, r.len);
                return 0;
            },
            read);
    }

    // The same, with the caller's bytes written into the slot's staging by `fill(dst)` (r.len
    // bytes; a non-zero return is this call's result, its bytes still travel with the batch): a
    // caller whose bytes are not in plain memory (a JNI byte[]) copies them once, straight into
    // the pinned staging.
    template <class FillFn, class ReadFn>
    int run_fill(QReq& r, FillFn&& fill, ReadFn&& read) {
        std::unique_lock<std::mutex> lk(m_);
        if (!prepared_ || stop_) return kQueueStopped;
        if (r.len > max_req_) return kQueueTooBig;  // callers check accepts() first
        active_++;
        // Admission is first come, first served: a caller that finds no room joins the waiting
        // line, and whoever makes room (a slot launched or freed) places the waiting requests in
        // arrival order while they fit, then wakes their callers.  (Waking every waiter to race
        // for the room let an unlucky caller lose for several passes: 8-10 ms tails.)
        int rc = waitq_.empty() ? place(r) : 0;
        if (rc == 0) {
            r.admit = 0;
            waitq_.push_back(&r);
            cv_disp_.notify_one();  // the open slot is full: have it launched
            admit_cv(&r).wait(lk, [&] { return r.admit != 0 || stop_; });
            if (r.admit == 0) {  // stopped while waiting
                for (auto it = waitq_.begin(); it != waitq_.end(); ++it)
                    if (*it == &r) {
                        waitq_.erase(it);
                        break;
                    }
                leave();
                return kQueueStopped;
            }
            rc = r.admit;
        }
        if (rc != 1) {  // not even an empty slot takes it
            leave();
            return kQueueTooBig;
        }
        QSlot* s = &slots_[r.slot];
        lk.unlock();
        cv_disp_.notify_one();  // after the unlock: the dispatcher does not wake into a held lock
        const int frc = fill(s->in + r.off);
        lk.lock();
        if (--s->copying == 0) {  // the last copy: the dispatcher may launch (woken unlocked)
            lk.unlock();
            cv_disp_.notify_all();
            lk.lock();
        }
        done_cv(&r).wait(lk, [&] { return r.done; });  // woken with its own request (about) only
        lk.unlock();
        const int ret = frc ? frc : read(*s, r, r.status);
        lk.lock();
        // an early-completed caller may leave while its batch is still on the device: the slot
        // is free once its last reader has left AND the batch has completed
        if (--s->readers == 0 && s->state == QSlot::kDone) {
            s->state = QSlot::kFree;
            admit_waiting();
        }
        leave();
        flush_admits(lk, false);
        return ret;
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
    // getChunks requests completed before their batch (Backend::poll)
    uint64_t early() {
        std::lock_guard<std::mutex> lk(m_);
        return early_done_;
    }
    // mean microseconds per completed batch: open -> closed (filling), closed -> launched (the
    // callers' copies), launched -> completion observed (transfers + kernels)
    void timing(double* fill_us, double* copy_us, double* device_us) {
        std::lock_guard<std::mutex> lk(m_);
        const double n = timed_ ? (double)timed_ : 1.0;
        if (fill_us) *fill_us = t_fill_ / n;
        if (copy_us) *copy_us = t_copy_ / n;
        if (device_us) *device_us = t_dev_ / n;
    }

  private:
    // a caller leaves run() (queue lock held)
    void leave() {
        if (--active_ == 0 && stop_) idle_cv_.notify_all();
    }

    // Condition variables picked by a request's address (Fibonacci hashing: requests live on their
    // callers' stacks, which sit at the same offset in equally sized stacks, so low address bits
    // alone would put every caller on one variable)
    static size_t cv_index(const QReq* q, size_t n) {
        return (size_t)((reinterpret_cast<uintptr_t>(q) * 0x9E3779B97F4A7C15ull) >> 40) % n;
    }
    std::condition_variable& admit_cv(const QReq* q) { return cv_admit_[cv_index(q, kAdmitCvs)]; }
    std::condition_variable& done_cv(const QReq* q) { return cv_done_[cv_index(q, kDoneCvs)]; }

    // Places `r` in the open slot, opening a free slot when there is none (queue lock held).
    // 1 = placed (the caller copies its bytes to s.in + r.off next), 0 = no room now (the open
    // slot is marked full so that it launches), kQueueTooBig = not even an empty slot takes it.
    int place(QReq& r) {
        const uint64_t need = r.kind == QReq::kChunks ? qalign(r.len, 64) : qalign(r.len, 16);
        if (open_ < 0) {
            for (size_t i = 0; i < slots_.size() && open_ < 0; i++)
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
                    f.full = false;
                    f.seq = ++seq_;
                    f.t_open = std::chrono::steady_clock::now();
                    open_ = (int)i;
                }
            if (open_ < 0) return 0;  // every slot is busy
        }
        QSlot& o = slots_[open_];
        if (!(o.nreq() < c_.max_reqs && o.lo + need <= o.hi && b_.admits(o, r))) {
            if (o.nreq() == 0) return kQueueTooBig;
            o.full = true;  // launch it without lingering
            return 0;
        }
        r.slot = open_;
        r.done = false;
        r.status = 0;
        if (r.kind == QReq::kChunks) {
            r.off = o.lo;
            o.lo += need;
            r.idx = (uint32_t)o.chunks.size();
            if (o.chunks.empty())
                o.uniform_len = (uint32_t)r.len;
            else if (o.uniform_len != r.len)
                o.uniform_len = 0;
            if (r.len > o.max_chunk_len) o.max_chunk_len = r.len;
            o.chunks.push_back(&r);
        } else {
            o.hi -= need;
            r.off = o.hi;
            r.idx = (uint32_t)o.hashes.size();
            o.hashes.push_back(&r);
        }
        if (o.nreq() >= c_.max_reqs || o.hi - o.lo < max_req_) o.full = true;
        o.copying++;
        return 1;
    }

    // Wakes the callers admit_waiting placed, after releasing the queue lock (relock: take it
    // again before returning).  Every admit_waiting() is followed by one of these.
    void flush_admits(std::unique_lock<std::mutex>& lk, bool relock) {
        if (admit_wake_.empty()) return;
        std::vector<std::condition_variable*> adm;
        adm.swap(admit_wake_);
        lk.unlock();
        for (auto* cv : adm) cv->notify_all();
        if (relock) lk.lock();
    }

    // Room may have appeared (a slot launched or freed): place waiting requests in arrival order
    // while they fit and mark their callers to wake (queue lock held; flush_admits wakes them).
    void admit_waiting() {
        if (stop_) return;  // the waiting callers see stop_ and leave
        bool any = false;
        while (!waitq_.empty()) {
            QReq* q = waitq_.front();
            const int rc = place(*q);
            if (rc == 0) break;
            waitq_.pop_front();
            q->admit = rc;
            admit_wake_.push_back(&admit_cv(q));  // notified by flush_admits, after the unlock
            any = true;
        }
        if (any) cv_disp_.notify_one();
    }

    // Whether the open slot should go now (queue lock held); else *deadline = when it will.
    bool ready(std::chrono::steady_clock::time_point* deadline) {
        if (open_ < 0 || inflight_ >= c_.lanes) return false;
        const QSlot& o = slots_[open_];
        const size_t n = o.nreq();
        if (n == 0) return false;
        if (stop_) return true;  // draining: launch what was placed
        const size_t lanes = (size_t)c_.lanes * (c_.share_div ? c_.share_div : 1);
        const size_t share = ((size_t)active_ + lanes - 1) / lanes;
        if (inflight_ == 0 || o.full || n >= share) return true;
        *deadline = o.t_open + std::chrono::microseconds(c_.linger_us);
        return std::chrono::steady_clock::now() >= *deadline;
    }

    void dispatcher() {
#ifdef __linux__
        prctl(PR_SET_NAME, "sdfs-qdisp", 0, 0, 0);  // per-thread CPU accounting (scripts/queue_probe.py)
#endif
        std::unique_lock<std::mutex> lk(m_);
        for (;;) {
            std::chrono::steady_clock::time_point deadline{};
            while (!ready(&deadline)) {
                if (stop_ && (open_ < 0 || slots_[open_].nreq() == 0)) break;  // nothing left to launch
                if (deadline != std::chrono::steady_clock::time_point{}) {
                    // a timed wait on the system clock (pthread_cond_timedwait): the steady-clock
                    // form (pthread_cond_clockwait) is invisible to the GCC 11 ThreadSanitizer;
                    // the deadline itself is re-checked on the steady clock above
                    const auto left = deadline - std::chrono::steady_clock::now();
                    cv_disp_.wait_until(lk, std::chrono::system_clock::now() +
                                                std::chrono::duration_cast<std::chrono::system_clock::duration>(left));
                } else {
                    cv_disp_.wait(lk);
                }
                deadline = {};
            }
            if (!ready(&deadline)) break;  // stopped with nothing placed
            QSlot& s = slots_[open_];
            s.state = QSlot::kClosed;
            s.t_close = std::chrono::steady_clock::now();
            open_ = -1;
            inflight_++;
            int lane = 0;  // an idle lane exists: inflight_ <= lanes
            for (int l = 1; l < c_.lanes; l++)
                if (lane_busy_[l] < lane_busy_[lane]) lane = l;
            lane_busy_[lane]++;
            admit_waiting();  // waiting callers may open the next slot now
            flush_admits(lk, true);
            cv_disp_.wait(lk, [&] { return s.copying == 0; });
            s.readers = (int)s.nreq();
            launched_++;
            served_ += s.nreq();
            s.t_launch = std::chrono::steady_clock::now();
            lk.unlock();
            const int rc = b_.launch(s, lane);
            lk.lock();
            s.status = rc;
            s.state = QSlot::kFlight;
            flight_[lane].push_back(&s);
            lk.unlock();
            comp_cv_[lane].notify_one();
            lk.lock();
        }
        disp_done_ = true;  // completers may end once nothing is in flight
        for (auto& cv : comp_cv_) cv.notify_all();
    }

    // Waits for a launched slot's batch like Backend::wait, completing each getChunks request as
    // soon as the backend reports it final (called and returns without the queue lock).
    int wait_early(QSlot& s, int lane, std::unique_lock<std::mutex>& lk) {
        std::vector<uint8_t>& rdy = early_[lane];
        rdy.assign(s.chunks.size(), 0);  // the slot is closed: its request list does not change
        size_t left = s.chunks.size();
        std::vector<std::condition_variable*>& wake = wake_[lane];
        wake.clear();
        for (;;) {
            bool fin = false;
            const int rc = b_.poll(s, rdy.data(), &fin);
            if (fin) return rc;
            bool any = false;
            for (size_t i = 0; i < rdy.size(); i++)
                if (rdy[i] == 1) {
                    if (!any) lk.lock();
                    any = true;
                    rdy[i] = 2;  // completed early: the request may be gone once its caller wakes
                    s.chunks[i]->status = 0;
                    s.chunks[i]->done = true;
                    wake.push_back(&done_cv(s.chunks[i]));
                    early_done_++;
                    left--;
                }
            if (any) {
                // notified after the unlock (the variables are the queue's, the requests may
                // already be gone): a woken caller does not block again on the queue lock
                lk.unlock();
                for (auto* cv : wake) cv->notify_all();
                wake.clear();
            }
            if (left == 0) return b_.wait(s);  // nothing else can complete early
            std::this_thread::sleep_for(std::chrono::microseconds(c_.poll_us));
        }
    }

    // One per lane: a lane's batches complete in launch order (one stream).
    void completer(int lane) {
#ifdef __linux__
        prctl(PR_SET_TIMERSLACK, 1000UL, 0, 0, 0);  // 1 us: the poll period's sleeps stay short
        prctl(PR_SET_NAME, "sdfs-qcomp", 0, 0, 0);
#endif
        std::unique_lock<std::mutex> lk(m_);
        for (;;) {
            comp_cv_[lane].wait(lk, [&] { return !flight_[lane].empty() || (disp_done_ && inflight_ == 0); });
            if (flight_[lane].empty()) break;  // dispatcher gone and nothing in flight
            QSlot* s = flight_[lane].front();
            flight_[lane].pop_front();
            const int launched_rc = s->status;
            lk.unlock();
            bool polled = false;
            int rc;
            if constexpr (has_poll<Backend>::value) {
                polled = launched_rc == 0;
                rc = polled ? wait_early(*s, lane, lk) : b_.wait(*s);
            } else {
                rc = b_.wait(*s);  // always: drains whatever a failed launch enqueued
            }
            lk.lock();
            s->status = launched_rc ? launched_rc : rc;
            s->state = QSlot::kDone;
            s->t_done = std::chrono::steady_clock::now();
            t_fill_ += std::chrono::duration<double, std::micro>(s->t_close - s->t_open).count();
            t_copy_ += std::chrono::duration<double, std::micro>(s->t_launch - s->t_close).count();
            t_dev_ += std::chrono::duration<double, std::micro>(s->t_done - s->t_launch).count();
            timed_++;
            inflight_--;
            lane_busy_[lane]--;
            for (size_t i = 0; i < s->chunks.size(); i++) {
                if (polled && early_[lane][i] == 2) continue;  // completed (and maybe gone) already
                s->chunks[i]->status = s->status;
                s->chunks[i]->done = true;
                wake_[lane].push_back(&done_cv(s->chunks[i]));
            }
            for (QReq* q : s->hashes) {
                q->status = s->status;
                q->done = true;
                wake_[lane].push_back(&done_cv(q));
            }
            if (s->readers == 0) {  // every caller completed early and has left
                s->state = QSlot::kFree;
                admit_waiting();
            }
            cv_disp_.notify_all();
            if (disp_done_ && inflight_ == 0)
                for (auto& cv : comp_cv_) cv.notify_all();
            if (!wake_[lane].empty() || !admit_wake_.empty()) {
                // the pass's remaining callers and newly admitted ones, woken outside the lock
                std::vector<std::condition_variable*> adm;
                adm.swap(admit_wake_);
                lk.unlock();
                for (auto* cv : wake_[lane]) cv->notify_all();
                for (auto* cv : adm) cv->notify_all();
                wake_[lane].clear();
                lk.lock();
            }
        }
    }

    Backend& b_;
    Config c_;
    std::vector<QSlot> slots_;
    std::mutex m_;
    // callers waiting for room, in arrival order; each waits on a condition variable picked by
    // its request's address, so an admission wakes (about) one thread, not every waiting caller
    static constexpr uintptr_t kAdmitCvs = 64;
    std::deque<QReq*> waitq_;
    std::condition_variable cv_admit_[kAdmitCvs];
    std::condition_variable cv_disp_;
    // a caller waits for its request's completion on one of these (done_cv): completing a request
    // wakes about one thread, not every caller of the pass (round 6: with early completion a pass
    // of 30 callers woke all 30 up to ~10 times, ~200 us of CPU per call at 128 callers)
    static constexpr size_t kDoneCvs = 256;
    std::condition_variable cv_done_[kDoneCvs];
    std::vector<std::deque<QSlot*>> flight_;        // per lane, in launch order
    std::vector<std::condition_variable> comp_cv_;  // per lane
    std::vector<int> lane_busy_;
    std::vector<std::vector<uint8_t>> early_;  // per lane: its slot's requests completed early (2)
    std::vector<std::vector<std::condition_variable*>> wake_;  // per lane: completions to notify
    std::vector<std::condition_variable*> admit_wake_;  // admissions to notify (queue lock)
    std::thread disp_;
    std::vector<std::thread> comp_;
    int open_ = -1;
    int inflight_ = 0;
    int active_ = 0;  // callers inside run()
    std::condition_variable idle_cv_;  // active_ reached 0 while stopping
    bool prepared_ = false;
    bool stop_ = false;
    bool disp_done_ = false;  // the dispatcher has ended (stopping)
    uint64_t max_req_ = 0;
    uint64_t seq_ = 0;
    uint64_t launched_ = 0, served_ = 0, timed_ = 0, early_done_ = 0;
    double t_fill_ = 0, t_copy_ = 0, t_dev_ = 0;
};

}  // namespace sdfs
