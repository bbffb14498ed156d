// cdc_engine.hip — host side of the C-ABI (include/sdfs_cdc.h): engine lifecycle, device
// workspaces, the device-resident pipeline, and the host-buffer paths (getChunks / getHash /
// batched getChunks) with pinned staging and the coalescing queue for concurrent callers.
// Drop-in for org.opendedup.hashing.AbstractHashEngine (AbstractHashEngine.java:24-39) as
// implemented by VariableSha256HashEngine / VariableMD5HashEngine
// (VariableSha256HashEngine.java:41-121, VariableMD5HashEngine.java:37-108).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/sdfs_cdc.h"
#include "cdc_internal.h"
#include "engine_share.h"
#include "host_queue.h"

using namespace sdfs;

namespace {

thread_local std::string g_last_error;

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

}  // namespace

// shared with the other C-ABI translation units (dedup_index.hip, lz4, aes, map)
int sdfs::fail_status(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

namespace {

#define HIP_TRY(expr)                                                                             \
    do {                                                                                          \
        hipError_t _e = (expr);                                                                   \
        if (_e != hipSuccess)                                                                     \
            return fail(SDFS_CDC_EHIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e),     \
                        __FILE__, __LINE__);                                                      \
    } while (0)

int poly_degree(uint64_t p) { return p ? 63 - __builtin_clzll(p) : -1; }

uint64_t mulx_mod(uint64_t v, uint64_t poly, int d) {
    v <<= 1;
    if ((v >> d) & 1) v ^= poly;
    return v;
}

uint64_t bitrev64_host(uint64_t v) {
    uint64_t r = 0;
    for (int i = 0; i < 64; i++) r |= ((v >> i) & 1) << (63 - i);
    return r;
}
uint32_t bitrev32_host(uint32_t v) { return (uint32_t)(bitrev64_host(v) >> 32); }
uint32_t rev8_host(uint32_t v) { return (uint32_t)(bitrev64_host(v) >> 56); }

// Rolling-hash tables (same definition as the jar's precompute), laid out as the
// scan kernel's LDS image with `copies` lane-private copies (cdc_internal.h).  `mirror`: the
// tables of the bit-reversed state (cdc_device.h roll_step): entry x = bitrev64(table[rev8(x)]).
std::vector<uint8_t> build_table_image(uint64_t poly, uint32_t window, int copies, bool mirror, bool pop_swap) {
    const int d = poly_degree(poly);
    std::vector<uint64_t> push(256), pop(256);
    for (uint64_t i = 0; i < 256; i++) {
        uint64_t r = i;  // i mod P (deg P > 8)
        for (int k = 0; k < d; k++) r = mulx_mod(r, poly, d);
        push[i] = (i << d) ^ r;
        uint64_t q = i;
        for (uint32_t k = 0; k < 8 * window; k++) q = mulx_mod(q, poly, d);
        pop[i] = q;
    }
    if (mirror) {
        std::vector<uint64_t> mpush(256), mpop(256);
        for (uint32_t x = 0; x < 256; x++) {
            mpush[x] = bitrev64_host(push[rev8_host(x)]);
            mpop[x] = bitrev64_host(pop[rev8_host(x)]);
        }
        push.swap(mpush);
        pop.swap(mpop);
        if (pop_swap)  // high word first (the scan's kAblPopSwap forms)
            for (uint64_t& v : pop) v = (v << 32) | (v >> 32);
    }
    std::vector<uint8_t> img(scan_lds_bytes(copies));
    const uint32_t push_off = copies == 32 ? 0x10000u : 0x80u;
    for (uint32_t e = 0; e < 256; e++)
        for (uint32_t c = 0; c < (uint32_t)copies; c++) {
            memcpy(&img[(e << 8) | (c << 3)], &pop[e], 8);
            memcpy(&img[push_off | (e << 8) | (c << 3)], &push[e], 8);
        }
    return img;
}

template <typename T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;  // elements
    bool fits(size_t want) const { return p && want <= n; }
    hipError_t ensure(size_t want) {
        if (fits(want)) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
        size_t alloc = std::max<size_t>(want, 1);
        hipError_t e = hipMalloc(reinterpret_cast<void**>(&p), alloc * sizeof(T));
        if (e == hipSuccess) n = alloc;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
};

int pinned_ensure(uint8_t** p, size_t* n, size_t want) {
    if (*p && *n >= want) return SDFS_CDC_OK;
    if (*p) (void)hipHostFree(*p);
    *p = nullptr;
    *n = 0;
    if (hipHostMalloc(reinterpret_cast<void**>(p), std::max<size_t>(want, 64), hipHostMallocDefault) != hipSuccess)
        return fail(SDFS_CDC_ENOMEM, "hipHostMalloc(%zu) failed", want);
    *n = std::max<size_t>(want, 64);
    return SDFS_CDC_OK;
}

// timed stages (kernel_times order); "pipeline" = device time from the first enqueue to the last
// kernel of the run on its stream
constexpr int kNumTimed = 7;
const char* kKernelNames[kNumTimed] = {"prep", "cdc_scan", "cdc_resolve", "cdc_prefix", "cdc_scatter",
                                       "chunk_hash", "pipeline"};
enum { K_PREP = 0, K_SCAN, K_RESOLVE, K_PREFIX, K_SCATTER, K_HASH, K_PIPE };
constexpr int kEvPerRun = 2 * 8;

// Device scratch of one pipeline run.  The engine keeps a ring of them so that runs enqueued on
// different streams (two batches in flight: the coalescing queue, or a caller alternating
// streams) proceed concurrently on one engine; a workspace is reused only behind the event
// recorded after its previous run (cross-stream wait, no host sync).
constexpr uint32_t kSmall = 2 * kMaxBins + 8;  // hist | cursor | overflow, total, wave_ctr ..
constexpr int kRing = 3;
constexpr int kQueueInflight = 8;  // coalescing-queue lane streams (the most lanes a queue can run)
constexpr int kQueueLanes = 6;     // lanes: batches on the device at once, one stream each.  Since
                                   // callers leave as their own buffer is done (early completion), a
                                   // pass's tail holds its lane with few callers left: 6 lanes at 48
                                   // callers 12.5 -> 13.1 GiB/s (4 KiB mix), 9.3 -> 9.8 (default);
                                   // 8 no better (profiles/r06/queue_early/)
constexpr uint32_t kSplitSpreadPad = 96 * 1024;  // + the kernel's 32 KiB: one per CU (160 KiB of LDS)
constexpr int kQueueSpareSlots = 4;  // slots beyond one per lane: the open one and the ones being read
struct Workspace {
    DevBuf<uint32_t> bitmap;
    DevBuf<uint64_t> seg_prefix;
    DevBuf<uint32_t> small;
    DevBuf<uint32_t> rec_base;
    DevBuf<uint32_t> tasks;
    DevBuf<uint32_t> spec_starts, spec_cnt, spec_next;  // sectioned cut walk of very long buffers
    DevBuf<uint32_t> join;  // its parallel stitch: kJoinWords per section, then one flag per buffer
    DevBuf<uint32_t> seg_sum;  // piece mode: the scan's segment summaries (kSegSumWords per segment)
    DevBuf<uint32_t> x_scratch;  // extent ordering (getHash in bulk): hist | cursor | total, starts | tasks
    hipEvent_t free_ev = nullptr;
    bool pending = false;  // free_ev recorded and possibly not reached yet
    uint32_t* overflow() const { return small.p + 2 * kMaxBins; }
    void release_all() {
        for (auto* b : {&bitmap, &small, &rec_base, &tasks, &spec_starts, &spec_cnt, &spec_next, &join, &seg_sum,
                        &x_scratch})
            b->release();
        seg_prefix.release();
    }
};

// One slot of the double-buffered batch path (sdfs_cdc_get_chunks_batch): pinned staging in and
// out, the device copy of the packed batch and its output slots.  While the GPU chunks the batch
// in one slot, the host packs the next batch into the other and unpacks the previous one's
// results.
struct HostSlot {
    uint8_t* pin_in = nullptr;
    size_t pin_in_n = 0;
    uint8_t* pin_out = nullptr;
    size_t pin_out_n = 0;
    DevBuf<uint8_t> data;
    DevBuf<uint64_t> offs;
    DevBuf<uint32_t> lens;
    DevBuf<uint32_t> counts, starts, clens, total;
    DevBuf<uint8_t> digests;
    hipEvent_t h2d = nullptr;   // staging -> device copy done (copy stream)
    hipEvent_t done = nullptr;  // pipeline + device -> pinned results done (engine stream)
    bool busy = false;
    uint32_t b0 = 0, n = 0, dcap = 0;
};

// Device state of one coalescing-queue slot (host_queue.h): the batch's device copy, and its
// result image, written by the kernels in place on the device (dimg) and copied to pinned host
// memory (pin_out) in ONE pass by the last kernel of the batch (copy_out_kernel):
//   counts[n] | starts[n*dcap] | lens[n*dcap] | flags[16] | digests[n*dcap*32] | hash digests[nh*32]
// The GPU writes the pinned image itself, in stream order behind the fingerprint: no DMA-engine
// copy (copies of every stream share the DMA queues in order, so a device->host copy waiting on
// one batch's kernels would hold up the next batch's host->device copy) and no host round trip
// between the kernels and the copy (the completer used to issue it after waking on the kernels:
// 27 us at 8 caller threads, 350 us at 48, profiles/r05/queue/).
struct QSlotDev {
    uint8_t* pin_meta = nullptr;  // chunk offs u64[max_reqs] | lens u32 | hash offs u64 | lens u32
    size_t pin_meta_n = 0;
    uint8_t* pin_out = nullptr;
    size_t pin_out_n = 0;
    DevBuf<uint8_t> data;
    DevBuf<uint64_t> meta64;  // chunk offs | hash offs
    DevBuf<uint32_t> meta32;  // chunk lens | hash lens
    DevBuf<uint32_t> total;
    DevBuf<uint8_t> dimg;     // device result image (pin_out's layout)
    Workspace ws;  // the slot's own pipeline scratch (a slot is reused only after its batch completed)
    hipEvent_t kdone = nullptr;  // kernels of the batch done (result image in pin_out)
    hipStream_t st = nullptr;    // the lane stream it runs on
    // layout of the batch in flight (read by the callers)
    uint32_t n = 0, nh = 0, dcap = 0;
    uint64_t digests_at = 0, hdig_at = 0, img_bytes = 0;
    uint64_t ready_at = 0;  // pinned ready words (early completion), one per request, past the largest image
    bool early = false;     // the batch in flight completes its getChunks requests early
    std::string err;  // message of a failed launch/wait (set on the queue's threads)
};

}  // namespace

struct QueueBackend;

struct DevEngine {
    ~DevEngine();  // full teardown (the last handle of its set is gone)
    sdfs_cdc_params prm{};
    int degree = 0;
    int num_cus = 256;
    uint32_t seg_len = 4096;  // bytes of one buffer per scan lane (multiple of the block)
    int scan_variant = 0;     // 0 = production; others exist only in the tuning build
    int hash_variant = 0;
    int hash_wg_per_cu = 2;
    uint32_t scan_max_block = kScanThreads;  // widest scan workgroup (tuning build: SDFS_SCAN_MAX_BLOCK)
    bool hash_split = true;                  // latency form of the fingerprint for small batches (tuning: SDFS_HASH_SPLIT)
    bool small_seg = true;                   // short scan segments for small batches (tuning: SDFS_SMALL_SEG)
    uint32_t small_seg_len = kSmallBatchSeg;  // their length (tuning: SDFS_SMALL_SEG_LEN, a multiple of 256)
    uint32_t tiny_seg_len = kTinyBatchSeg;    // below 32 MiB (tuning: SDFS_TINY_SEG_LEN, a multiple of 64)
    bool q_early = true;  // queue passes complete each getChunks request when its buffer is done (tuning: SDFS_Q_EARLY=0 = off)
    bool tiny_scan = true;  // passes < 32 MiB: 64/128-byte segments with ScanTiny (tuning: SDFS_TINY_SCAN=0 = off)
    bool long_split = true;                  // latency form for chunks > 32 KiB (tuning: SDFS_LONG_SPLIT)
    bool par_stitch = true;                  // parallel join/place of long buffers' sections (tuning: SDFS_PAR_STITCH)
    uint32_t sec_log2 = 18;                  // section length of long buffers' cut walk (tuning: SDFS_SEC_LOG2)
    uint32_t skip_walk = 0;                  // measurement only (tuning: SDFS_SKIP_WALK 1..3): no chunks
    bool list_walk = true;                   // fused walk: LDS list form (tuning: SDFS_LIST_WALK=0 = queue walk)
    // Scan work handed out per wave from a counter instead of a static workgroup stride (tuning:
    // SDFS_SCAN_DYN=0 = static): the same rate alone (interleaved A/B within 0.5 %), and a scan
    // workgroup that starts late -- its CU held by another kernel, e.g. the exchange's RCCL
    // all-gather at N > 1 -- no longer holds up the whole scan (one-GPU projection of the 8-rank
    // exchange: +21 % per step with the static stride, +6-11 % with this; profiles/r06/exchange_proxy/)
    bool scan_dyn = true;
    bool piece_walk = true;                  // sections walked in the scan's epilogue when they fit (tuning: SDFS_PIECE_WALK)
    bool scan_prio = false;                  // pre-fingerprint stages on a high-priority stream (tuning: SDFS_SCAN_PRIO)
    hipStream_t s_scan = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    // Front-end order across streams (SDFS_FRONT_SERIAL): a batch's scan waits for the previous
    // batch's prefix/scatter (whatever stream it ran on), so those one-workgroup kernels never
    // queue behind a full-chip scan of the other stream; the fingerprint kernels still overlap.
    bool front_serial = false;
    bool front_recorded = false;
    // Measurement probe (tuning: SDFS_FUSED_PROBE): the batch's fingerprint kernel is replaced by
    // the fused scan + fingerprint kernel over the batch's own scan (again) and its tasks.
    int fused_probe = 0;  // form (cdc_sweep_r3.hip launch_fused_probe)
    // latency form of the fingerprint: two lanes per chunk (tuning: SDFS_SPLIT_PACKED=0 = one lane)
    bool split_packed = true;
    bool split_spread = false;  // one latency-form workgroup per CU for small passes (tuning: SDFS_SPLIT_SPREAD)
    bool split_masked = false;  // tuning: SDFS_SPLIT_MASKED (latency form, finished lanes masked off)
    bool split_bybuf = true;    // latency-form groups per buffer, not per 32 longest (tuning: SDFS_SPLIT_BYBUF;
                                // DESIGN.md §14)
    // small-batch cut walk: candidate list + successors (tuning: SDFS_SMALL_BALLOT=1 = ballots only)
    bool small_ballot = false;
    hipEvent_t ev_front = nullptr;
    ScanVariantInfo scan_info{};
    bool pred_div = false;  // divisor detector evaluated as such (scan predicate kind 3)
    uint32_t first_off = 0;
    uint32_t bin_shift = 0, nbins = 1;
    uint32_t digest_len = 32;
    hipStream_t stream = nullptr;  // direct host paths
    std::mutex mu;                 // enqueue order of every device operation of the engine

    DevBuf<uint8_t> tab_image;
    DevBuf<uint8_t> zero_page;
    Workspace ws[kRing];
    uint32_t ws_next = 0;
    // direct getHash device buffers and pinned staging
    DevBuf<uint8_t> h_data;
    DevBuf<uint32_t> o_starts;
    DevBuf<uint8_t> o_digests;
    DevBuf<uint8_t> x_data;  // host-batch staging of getHash in bulk
    DevBuf<uint64_t> x_offs;
    DevBuf<uint32_t> x_lens;
    DevBuf<uint8_t> x_digests;
    uint8_t* pin_data = nullptr;
    size_t pin_data_n = 0;
    // batched host path: two slots, H2D on its own stream, packing on copy_threads threads
    HostSlot hs[2];
    hipStream_t s_h2d = nullptr;
    int copy_threads = 8;
    std::unique_ptr<CopyPool> pool;
    // coalescing queue for concurrent single-buffer callers
    hipStream_t qs[kQueueInflight] = {};
    std::unique_ptr<QueueBackend> qb;
    std::unique_ptr<CoalescingQueue<QueueBackend>> q;
    std::mutex q_init;
    int q_state = 0;  // 0 = not started, 1 = running, -1 = disabled (flag or start failure)
    uint32_t timing_mask = 0xFFFFFFFFu;  // stages timed when timing is on (bit = kKernelNames index)

    // per-kernel HIP events for the last `timing_slots` runs (ring); averaged by kernel_times
    struct TimedRun {
        std::vector<hipEvent_t> ev;  // kEvPerRun events
        std::vector<int> kid;        // stage id of event pair i (ev[2i], ev[2i+1])
    };
    int timing_slots = 0;
    std::vector<TimedRun> ev_runs;
    uint64_t runs_recorded = 0;
    TimedRun* run = nullptr;  // run in flight (nullptr: timing off)
};

namespace {

int validate(const sdfs_cdc_params* p) {
    if (!p) return fail(SDFS_CDC_EINVAL, "null params");
    const int d = poly_degree(p->poly);
    // fp < 2^d lives in two dwords with the push index (bits d-8..d-1) inside the high one
    if (d < 48 || d > 55) return fail(SDFS_CDC_EINVAL, "polynomial degree %d outside [48,55]", d);
    if (!scan_window_supported((int)p->window))
        return fail(SDFS_CDC_EINVAL, "window %u unsupported (16/32/48/64)", p->window);
    if (p->max_len == 0) return fail(SDFS_CDC_EINVAL, "max_len must be > 0");
    if (p->min_cmp > SDFS_CDC_MIN_GE) return fail(SDFS_CDC_EINVAL, "bad min_cmp");
    if (p->hash_algo > SDFS_CDC_MD5) return fail(SDFS_CDC_EINVAL, "bad hash_algo");
    if (p->pred_kind > SDFS_CDC_PRED_DIV) return fail(SDFS_CDC_EINVAL, "bad pred_kind %u", p->pred_kind);
    if (p->pred_kind == SDFS_CDC_PRED_MASK && (p->pred_mask >> d))
        return fail(SDFS_CDC_EINVAL, "pred_mask has bits above the fp degree");
    if (p->pred_kind == SDFS_CDC_PRED_DIV) {
        if (p->pred_div == 0 || (p->pred_div >> 32))
            return fail(SDFS_CDC_EINVAL, "pred_div must be in [1, 2^32)");
        // a divisor other than a power of two is evaluated in f64: the window fp must be exact
        if ((p->pred_div & (p->pred_div - 1)) != 0 && d > 53)
            return fail(SDFS_CDC_EINVAL, "divisor predicate needs a polynomial of degree <= 53 (got %d)", d);
    }
    if (p->flags & ~(uint32_t)SDFS_CDC_FLAG_DIRECT) return fail(SDFS_CDC_EINVAL, "unknown flags 0x%x", p->flags);
    if (p->device < -1 && !p->device_mask) return fail(SDFS_CDC_EINVAL, "device %d (-1 = every gfx950 device)", p->device);
    return SDFS_CDC_OK;
}

uint32_t slot_cap_for(const sdfs_cdc_params& p, uint64_t len) {
    const uint64_t shortest_cut = p.min_cmp == SDFS_CDC_MIN_GT ? (uint64_t)p.min_len + 1 : std::max<uint64_t>(p.min_len, 1);
    const uint64_t shortest = std::min<uint64_t>(shortest_cut, p.max_len);
    return (uint32_t)(len / shortest + 2);
}

// ---- workspace ring ----
struct WsNeed {
    uint64_t bitmap_words = 0, seg_prefix = 0, rec_base = 0, tasks = 0, spec_starts = 0, spec_items = 0, x_scratch = 0,
             seg_sum = 0;
};

// Next workspace of the ring (or `own`, a queue slot's), sized for `nd`, ordered behind its
// previous use on `s`.  Caller holds e->mu and has set the device.
int ws_acquire(DevEngine* e, const WsNeed& nd, hipStream_t s, Workspace** out, Workspace* own = nullptr) {
    Workspace* w = own ? own : &e->ws[e->ws_next++ % kRing];
    const bool fits = w->bitmap.fits(nd.bitmap_words) && w->small.fits(kSmall + 8) &&
                      w->rec_base.fits(nd.rec_base) && w->tasks.fits(nd.tasks) &&
                      (!nd.seg_prefix || w->seg_prefix.fits(nd.seg_prefix)) &&
                      (!nd.spec_items || (w->spec_starts.fits(nd.spec_starts) && w->spec_cnt.fits(nd.spec_items) &&
                                          w->spec_next.fits(nd.spec_items) &&
                                          w->join.fits(nd.spec_items * kJoinWords + nd.rec_base))) &&
                      (!nd.x_scratch || w->x_scratch.fits(nd.x_scratch)) && (!nd.seg_sum || w->seg_sum.fits(nd.seg_sum));
    if (!fits && w->pending) HIP_TRY(hipEventSynchronize(w->free_ev));  // never free memory in use
    HIP_TRY(w->bitmap.ensure(std::max<uint64_t>(nd.bitmap_words, 2)));
    HIP_TRY(w->small.ensure(kSmall + 8));
    HIP_TRY(w->rec_base.ensure(std::max<uint64_t>(nd.rec_base, 1)));
    HIP_TRY(w->tasks.ensure(std::max<uint64_t>(nd.tasks, 1)));
    if (nd.seg_prefix) HIP_TRY(w->seg_prefix.ensure(nd.seg_prefix));
    if (nd.spec_items) {
        HIP_TRY(w->spec_starts.ensure(nd.spec_starts));
        HIP_TRY(w->spec_cnt.ensure(nd.spec_items));
        HIP_TRY(w->spec_next.ensure(nd.spec_items));
        HIP_TRY(w->join.ensure(nd.spec_items * kJoinWords + nd.rec_base));  // + one flag per buffer
    }
    if (nd.x_scratch) HIP_TRY(w->x_scratch.ensure(nd.x_scratch));
    if (nd.seg_sum) HIP_TRY(w->seg_sum.ensure(nd.seg_sum));
    if (w->pending) HIP_TRY(hipStreamWaitEvent(s, w->free_ev, 0));
    *out = w;
    return SDFS_CDC_OK;
}

int ws_release(Workspace* w, hipStream_t s) {
    HIP_TRY(hipEventRecord(w->free_ev, s));
    w->pending = true;
    return SDFS_CDC_OK;
}

// Records a start event for stage `kid` on stream `st` (timing runs only); returns the pair index.
int t_begin(DevEngine* e, int kid, hipStream_t st) {
    if (!e->run || !((e->timing_mask >> kid) & 1u)) return -1;
    const int i = (int)e->run->kid.size();
    if (2 * i + 1 >= kEvPerRun) return -1;
    e->run->kid.push_back(kid);
    (void)hipEventRecord(e->run->ev[2 * i], st);
    return i;
}
void t_end(DevEngine* e, int i, hipStream_t st) {
    if (e->run && i >= 0) (void)hipEventRecord(e->run->ev[2 * i + 1], st);
}

#ifdef SDFS_TUNING
// measurement only: per-wave stamps of fingerprint variant 50 go here (sdfs_cdc_tuning_set_stamps)
uint64_t* g_stamps = nullptr;
#endif

// Early completion of a coalescing-queue pass (HashArgs::done_ctr): the pinned image's header
// (counts | starts | lens | flags) is copied before the fingerprint runs, the digests go straight
// into the pinned image, and each buffer's ready word is set as its last chunk is stored.
struct EarlyDone {
    const void* hdr_src = nullptr;  // device result image
    void* hdr_dst = nullptr;        // pinned result image
    uint64_t hdr_bytes = 0;         // [0, hdr_bytes): its header (a multiple of 16)
    uint32_t* ready = nullptr;      // pinned ready words, one per buffer
    uint32_t seq = 0;               // the pass's number (what a ready word is set to)
};

inline uint32_t early_words(const EarlyDone* early, uint32_t nbuf) { return early ? (nbuf + 3u) & ~3u : 0u; }

// Workspace needs of one pipeline run.
WsNeed pipeline_need(const DevEngine* e, uint64_t data_bytes, uint32_t nbuf, uint32_t uniform_len, uint32_t cap,
                     uint64_t max_buf_len, uint32_t* sec_len_out, uint32_t* nsec_out, uint32_t* spec_cap_out) {
    WsNeed nd;
    nd.bitmap_words = ((data_bytes + 63) / 64) * 2 + 2;
    nd.rec_base = nbuf;
    nd.tasks = (uint64_t)nbuf * cap;
    if (!uniform_len) nd.seg_prefix = (uint64_t)nbuf + 1;
    const uint64_t mbl = uniform_len ? uniform_len : max_buf_len;
    const uint32_t sec = resolve_section_len(mbl, e->prm.max_len, e->sec_log2);
    *sec_len_out = sec;
    *nsec_out = *spec_cap_out = 0;
    if (sec) {
        *nsec_out = (uint32_t)((mbl + sec - 1) / sec);
        *spec_cap_out = sec / (e->first_off + 1) + 2;
        nd.spec_items = (uint64_t)nbuf * *nsec_out;
        nd.spec_starts = nd.spec_items * *spec_cap_out;
        if (uniform_len)  // piece mode's segment summaries (run_pipeline decides; sized for it here)
            nd.seg_sum = (uint64_t)nbuf * ((uniform_len + e->seg_len - 1) / e->seg_len) * kSegSumWords;
    }
    return nd;
}

// The device pipeline (scan [+ fused cut walk] | resolve, prefix, scatter, fingerprint) of one
// batch, enqueued on `s` behind everything already there, on workspace `w` (acquired by the
// caller).  Caller holds e->mu.
int run_pipeline(DevEngine* e, Workspace* w, const uint8_t* d_data, uint64_t data_bytes, const uint64_t* d_offs,
                 const uint32_t* d_lens, uint32_t nbuf, uint32_t uniform_len, uint64_t buffer_id_base,
                 const sdfs_cdc_dev_out* out, hipStream_t s, uint64_t max_buf_len, uint32_t sec_len, uint32_t nsec,
                 uint32_t spec_cap, uint32_t* ovf_to = nullptr, const EarlyDone* early = nullptr) {
    e->run = nullptr;
    if (e->timing_slots > 0) {
        e->run = &e->ev_runs[e->runs_recorded % e->timing_slots];
        e->run->kid.clear();
    }
    const int tpipe = t_begin(e, K_PIPE, s);
    if (nbuf == 0) {
        HIP_TRY(hipMemsetAsync(out->total, 0, 4, s));
        HIP_TRY(hipMemsetAsync(w->small.p, 0, (kSmall + 8) * sizeof(uint32_t), s));
        t_end(e, tpipe, s);
        if (e->run) e->runs_recorded++;
        return SDFS_CDC_OK;
    }
    // Optional (tuning build: SDFS_SCAN_PRIO): the stages before the fingerprint run on a
    // high-priority stream, so that with two batches in flight the dispatcher hands CUs freed by
    // one batch's fingerprint kernel to the next batch's scan first.
    const hipStream_t s_hash = s;
    if (e->scan_prio && e->s_scan && nbuf >= (uint32_t)e->num_cus * 4) {
        HIP_TRY(hipEventRecord(e->ev_fork, s_hash));
        HIP_TRY(hipStreamWaitEvent(e->s_scan, e->ev_fork, 0));
        s = e->s_scan;
    }
    // A batch too small to give every SIMD a wave of full segments (a coalescing-queue pass:
    // fewer 256 KiB buffers than SIMDs) scans in short segments: the fused walk's one wave per
    // buffer would leave most SIMDs idle and put a 4 KiB serial chain on every lane (0.18 ms);
    // 512-byte segments plus the separate walk take ~0.07 ms.  Counted in
    // segments, not buffers: 102 backup buffers of 40 MiB are a million segments.
    const uint64_t full_segs = data_bytes / e->seg_len;
    // Below 32 MiB (a queue pass: its slot is 32 MiB) the segments are shorter again: a lane alone
    // on its SIMD waits out every byte's LDS round trip, so a lone pass's scan time is its lanes'
    // chain length (segment + 48-byte warm-up).  256 bytes: a lone buffer 34 -> 23 us
    // (profiles/r05/small_seg/); then halved while one wave per SIMD still has a segment per
    // lane, down to 64 bytes, scanned by ScanTiny (64-byte blocks): a lone buffer 21.5 -> 10.4 us
    // (profiles/r05/tiny_scan/).  Passes of 16-32 MiB keep 256 (more lanes than one wave per SIMD:
    // the warm-up would only add work).
    // Segments shorter than the scan form's block only go to ScanTiny (its 64-byte blocks);
    // any other form scans whole blocks, so its segments stay multiples of its block.
    const bool tiny_ok = e->tiny_scan && e->scan_variant == 0;
    const uint32_t blk = e->scan_info.blk;
    uint32_t small_len = e->small_seg_len;
    if (full_segs < (uint64_t)e->num_cus * 4 * 8) {
        uint32_t t = e->tiny_seg_len;
        if (tiny_ok) {
            const uint64_t per_lane = data_bytes / ((uint64_t)e->num_cus * 4 * 64);
            while (t > 64 && t % 128 == 0 && t / 2 >= per_lane) t /= 2;
        } else {
            t = (t + blk - 1) / blk * blk;
        }
        if (small_len > t && small_len % t == 0) small_len = t;
    }
    const uint32_t seg_len = (full_segs < (uint64_t)e->num_cus * 4 * 64 && e->seg_len > small_len &&
                              e->seg_len % small_len == 0 && e->small_seg)
                                 ? small_len
                                 : e->seg_len;
    uint32_t* hist = w->small.p;
    uint32_t* cursor = w->small.p + kMaxBins;
    uint32_t* total = w->small.p + 2 * kMaxBins + 1;
    const bool front = e->front_serial && e->ev_front && nbuf >= (uint32_t)e->num_cus * 4;
    if (front && e->front_recorded) HIP_TRY(hipStreamWaitEvent(s, e->ev_front, 0));
    {
        const int t = t_begin(e, K_PREP, s);
        // (+ the per-buffer chunk counters of early completion, behind the fixed words)
        const uint32_t zw = kSmall + 8 + early_words(early, nbuf);
        if (!w->small.fits(zw)) return fail(SDFS_CDC_EHIP, "internal: workspace has no early-completion counters");
        HIP_TRY(launch_prep_zero(w->small.p, zw, ovf_to, s));
        if (!uniform_len) HIP_TRY(launch_seg_prefix(d_lens, nbuf, seg_len, w->seg_prefix.p, s));
        t_end(e, t, s);
    }
    const bool pred64 = (e->prm.pred_mask >> 32) != 0;
    int pk = pred64 ? 1 : 0;
    ScanArgs sa{};
    sa.data = d_data;
    sa.offs = d_offs;
    sa.lens = d_lens;
    sa.bitmap = w->bitmap.p;
    sa.nbuf = nbuf;
    sa.uniform_len = uniform_len;
    sa.seg_len = seg_len;
    if (e->scan_info.mirror) {
        // bit-reversed state: fp bits 0..31 are the reversed hi word (cdc_device.h roll_step)
        const uint64_t m = e->prm.pred_mask, v = e->prm.pred_value;
        sa.jshift = (uint32_t)(64 - e->degree);
        sa.mask_lo = bitrev32_host((uint32_t)m);
        sa.mask_hi = bitrev32_host((uint32_t)(m >> 32));
        sa.val_lo = bitrev32_host((uint32_t)v);
        sa.val_hi = bitrev32_host((uint32_t)(v >> 32));
        if (e->pred_div) {
            // divisor detector: fp % D == R in f64 (cdc_device.h cand_shift<3>); R >= D never
            // matches, which a NaN target expresses (no comparison with NaN holds)
            pk = 3;
            sa.div_d = (double)e->prm.pred_div;
            sa.div_inv = 1.0 / sa.div_d;
            sa.rem_d = e->prm.pred_rem < e->prm.pred_div ? (double)e->prm.pred_rem : __builtin_nan("");
        } else if (!pred64 && m != 0 && (m & (m + 1)) == 0 && v == 0) {  // low k bits zero: one compare
            const int k = __builtin_popcountll(m);
            sa.thr = k == 32 ? 1u : 1u << (32 - k);
            pk = 2;
        }
    } else {
        sa.jshift = (uint32_t)(e->degree - 40);
        sa.mask_lo = (uint32_t)e->prm.pred_mask;
        sa.mask_hi = (uint32_t)(e->prm.pred_mask >> 32);
        sa.val_lo = (uint32_t)e->prm.pred_value;
        sa.val_hi = (uint32_t)(e->prm.pred_value >> 32);
    }
    sa.tab_image = e->tab_image.p;
    sa.zero_page = e->zero_page.p;
    uint64_t seg_bound;
    if (uniform_len) {
        const uint64_t spb = (uniform_len + seg_len - 1) / seg_len;
        sa.total_segs = spb * nbuf;
        seg_bound = sa.total_segs;
    } else {
        sa.seg_prefix = w->seg_prefix.p;
        seg_bound = data_bytes / seg_len + nbuf;
    }
    ResolveArgs ra{};
    ra.bitmap = w->bitmap.p;
    ra.offs = d_offs;
    ra.lens = d_lens;
    ra.nbuf = nbuf;
    ra.uniform_len = uniform_len;
    ra.first_off = e->first_off;
    ra.max_len = e->prm.max_len;
    ra.cap = out->cap;
    ra.bin_shift = e->bin_shift;
    ra.nbins = e->nbins;
    ra.counts = out->counts;
    ra.starts = out->starts;
    ra.clens = out->lens;
    ra.hist = hist;
    ra.overflow = ovf_to ? ovf_to : w->overflow();
    ra.max_buf_len = uniform_len ? uniform_len : max_buf_len;
    ra.small_ballot = e->small_ballot ? 1u : 0u;
    ra.sec_len = sec_len;
    if (sec_len) {
        ra.nsec = nsec;
        ra.spec_cap = spec_cap;
        ra.spec_starts = w->spec_starts.p;
        ra.spec_cnt = w->spec_cnt.p;
        ra.spec_next = w->spec_next.p;
        if (e->par_stitch) {
            ra.join = w->join.p;
            ra.join_bad = w->join.p + (uint64_t)nbuf * nsec * kJoinWords;
        }
    }
    // one wave = one buffer: the scan kernel resolves the cuts in its epilogue
    // (the fused and piece walks read the scan's per-segment state, so a segment is whole blocks:
    // a uniform pass of 4 or 8 KiB buffers at 64- or 128-byte segments takes ScanTiny + the walk)
    const bool fused = e->scan_info.fuse && uniform_len && (e->scan_info.chains == 1 || e->scan_info.fuse == 2) &&
                       (uint64_t)uniform_len == 64ull * seg_len && seg_len < 0xFFFFu && seg_len % blk == 0;
    // long uniform buffers whose sections are exactly one wave's 64 segments: the scan's epilogue
    // walks every section speculatively from the lanes' summaries (no spec kernel)
    const bool piece = !fused && e->piece_walk && e->par_stitch && sec_len && uniform_len && w->seg_sum.p &&
                       e->scan_info.fuse == 2 && e->scan_info.chains == 1 &&
                       sec_len == 64ull * seg_len && uniform_len % sec_len == 0 && seg_len < 0xFFFF &&
                       seg_len % blk == 0;
    if (piece) {
        ra.spec_from_scan = 1;
        ra.seg_sum = w->seg_sum.p;
        ra.seg_len = seg_len;
    }
    sa.fuse_resolve = fused ? 1u : piece ? 2u : 0u;
    sa.skip_walk = e->skip_walk;
    sa.list_walk = e->list_walk ? 1u : 0u;
    sa.wave_ctr = e->scan_dyn ? w->small.p + 2 * kMaxBins + 8 : nullptr;  // zeroed with `small` above
    sa.res = ra;
    // One workgroup per CU (the LDS tables); a batch too small to give every CU 1024 threads
    // (fewer than ~4096 write buffers, e.g. the coalescing queue's) launches narrower
    // workgroups, so its waves run one per SIMD instead of four on a few CUs.
    const uint64_t max_wgs = (uint64_t)e->num_cus * e->scan_info.wg_per_cu;
    const uint64_t lanes = (seg_bound + e->scan_info.chains - 1) / e->scan_info.chains;
    uint64_t block = (lanes + max_wgs - 1) / max_wgs;
    block = std::min<uint64_t>(std::max<uint64_t>((block + 255) / 256 * 256, 256),
                               std::min<uint64_t>(e->scan_max_block, (uint64_t)e->scan_info.threads));
    const uint64_t per_block = block * e->scan_info.chains;
    uint64_t grid = (seg_bound + per_block - 1) / per_block;
    grid = std::min<uint64_t>(grid, max_wgs);
    grid = std::max<uint64_t>(grid, 1);
    {
        const int t = t_begin(e, K_SCAN, s);
        if (seg_len % blk != 0) {
            if (!tiny_ok || sa.fuse_resolve) return fail(SDFS_CDC_EINVAL, "internal: segment %u not whole blocks", seg_len);
            HIP_TRY(launch_scan_tiny(sa, (int)e->prm.window, pk, (int)grid, (int)block, s));
        } else {
            HIP_TRY(launch_scan(sa, (int)e->prm.window, pk, e->scan_variant, (int)grid, (int)block, s));
        }
        t_end(e, t, s);
    }
    if (!fused) {
        const int t = t_begin(e, K_RESOLVE, s);
        HIP_TRY(launch_resolve(ra, s));
        t_end(e, t, s);
    }
    PrefixArgs pa{};
    pa.counts = out->counts;
    pa.nbuf = nbuf;
    pa.hist = hist;
    pa.nbins = e->nbins;
    pa.cursor = cursor;
    pa.rec_base = w->rec_base.p;
    pa.total = total;
    pa.grand_total = out->total;
    ScatterArgs ca{};
    ca.counts = out->counts;
    ca.clens = out->lens;
    ca.nbuf = nbuf;
    ca.cap = out->cap;
    ca.bin_shift = e->bin_shift;
    ca.nbins = e->nbins;
    ca.cursor = cursor;
    ca.tasks = w->tasks.p;
    if ((uint64_t)nbuf * out->cap <= kSmallScatterSlots && e->nbins <= 1024) {
        // a small batch (a queue pass): both in one workgroup, timed as the prefix stage
        const int t = t_begin(e, K_PREFIX, s);
        HIP_TRY(launch_prefix_scatter_small(pa, ca, s));
        t_end(e, t, s);
    } else {
        {
            const int t = t_begin(e, K_PREFIX, s);
            HIP_TRY(launch_prefix(pa, s));
            t_end(e, t, s);
        }
        const int t = t_begin(e, K_SCATTER, s);
        HIP_TRY(launch_scatter(ca, s));
        t_end(e, t, s);
    }
    if (front) {
        HIP_TRY(hipEventRecord(e->ev_front, s));
        e->front_recorded = true;
    }
    if (s != s_hash) {  // join: the fingerprint runs on the caller's stream
        HIP_TRY(hipEventRecord(e->ev_join, s));
        HIP_TRY(hipStreamWaitEvent(s_hash, e->ev_join, 0));
        s = s_hash;
    }
    HashArgs ha{};
    ha.zero_page = e->zero_page.p;
    ha.data = d_data;
    ha.offs = d_offs;
    ha.uniform_len = uniform_len;
    ha.tasks = w->tasks.p;
    ha.total = total;
    ha.starts = out->starts;
    ha.clens = out->lens;
    ha.rec_base = w->rec_base.p;
    ha.cap = out->cap;
    ha.digests = out->digests;
    ha.records = out->records;
    ha.records_cap = out->records_cap;
    ha.buffer_id_base = buffer_id_base;
    ha.algo = e->prm.hash_algo;
    ha.wave_ctr = w->small.p + 2 * kMaxBins + 2;  // zeroed with the rest of `small` above
    ha.persist_grid = (uint32_t)(e->num_cus * e->hash_wg_per_cu);
#ifdef SDFS_TUNING
    ha.stamps = g_stamps;
#endif
    if (early) {
        // the header the callers read is final once the walk and scatter ran: into the pinned
        // image now, in stream order before the fingerprint (whose digests go there directly)
        HIP_TRY(launch_copy_out(early->hdr_src, early->hdr_dst, early->hdr_bytes, s));
        ha.done_ctr = w->small.p + kSmall + 8;  // zeroed by the prep above
        ha.counts = out->counts;
        ha.ready = early->ready;
        ha.seq = early->seq;
    }
    {
        // chunks of more than kLongBlocks SHA blocks (a maxLen above 32 KiB: the backup profile)
        // head the longest-first list; after the scatter, cursor[b] = tasks in bins >= b, so
        // cursor[tb + 1] counts the chunks of bins wholly above kLongBlocks
        const uint32_t tb = kLongBlocks >> e->bin_shift;
        const uint32_t maxblocks = (e->prm.max_len + 8) / 64 + 1;
        if (e->long_split && e->prm.max_len > 32768 && ((tb + 1) << e->bin_shift) <= maxblocks && tb + 1 < e->nbins) {
            ha.nlong = cursor + tb + 1;
            const uint64_t mbl = uniform_len ? uniform_len : max_buf_len;
            const uint64_t per = mbl / ((uint64_t)kLongBlocks * 64 - 72) + 1;
            ha.max_long = (uint32_t)std::min<uint64_t>((uint64_t)nbuf * per, (uint64_t)nbuf * out->cap);
        }
    }
    {
        const int t = t_begin(e, K_HASH, s);
        const uint64_t max_tasks = (uint64_t)nbuf * out->cap;
        // a batch too small to give every SIMD a wave (a coalescing-queue pass) costs its longest
        // chunk's serial chain: the two-wave latency form shortens it
        if (e->hash_split && e->prm.hash_algo != SDFS_CDC_MD5 && e->hash_variant == 0 &&
            max_tasks <= (uint64_t)e->num_cus * 128)
        {
            // A pass small enough for one latency-form workgroup per CU (the coalescing queue's)
            // can pad its workgroups' LDS so that no two land on one CU: with several passes in
            // flight (the queue's lanes) their serial chain waves would otherwise share SIMDs and
            // issue at a fraction of a lone wave's rate (tuning: SDFS_SPLIT_SPREAD)
            const uint64_t groups = (max_tasks + 31) / 32;
            const uint32_t pad = e->split_spread && groups <= (uint64_t)e->num_cus ? kSplitSpreadPad : 0u;
            // groups drawn from one buffer end that buffer with its own longest chunk instead of
            // the group holding the pass's 32 longest (every group of such a pass runs at once):
            // 48 callers +16 % at the reference default, +4 % at the 4 KiB mix
            ha.split_masked = e->split_masked;
            if (e->split_bybuf && e->split_packed) {
                ha.bybuf = (out->cap + 31) / 32;
                ha.counts = out->counts;
            }
            HIP_TRY(launch_hash_split(ha, max_tasks, s, e->split_packed, pad));
        }
#ifdef SDFS_TUNING
        else if (e->fused_probe && fused && nbuf >= (uint32_t)e->num_cus * 4)
            HIP_TRY(launch_fused_probe(sa, ha, w->small.p + 2 * kMaxBins + 4, (int)e->prm.window, pk, e->num_cus,
                                       e->fused_probe, s));
#endif
        else
            HIP_TRY(launch_hash(ha, max_tasks, e->hash_variant, s, e->split_packed));
        t_end(e, t, s);
    }
    t_end(e, tpipe, s);
    if (e->run) e->runs_recorded++;
    return SDFS_CDC_OK;
}

// Validates a device-run request, acquires a workspace and runs the pipeline on `s`.  The
// overflow flag of the run is left at *ovf_dev (device word, valid until the workspace's next
// use) when ovf_dev != NULL.  Caller holds e->mu.
int device_run(DevEngine* e, const uint8_t* d_data, uint64_t data_bytes, const uint64_t* d_offs,
               const uint32_t* d_lens, uint32_t nbuf, uint32_t uniform_len, uint64_t buffer_id_base,
               const sdfs_cdc_dev_out* out, hipStream_t s, uint64_t max_buf_len, const uint32_t** ovf_dev,
               Workspace* own = nullptr, uint32_t* ovf_to = nullptr, const EarlyDone* early = nullptr) {
    if (!out || !out->counts || !out->starts || !out->lens || !out->digests || !out->total)
        return fail(SDFS_CDC_EINVAL, "incomplete sdfs_cdc_dev_out");
    if (uniform_len && (uniform_len & 63)) return fail(SDFS_CDC_EINVAL, "uniform_len must be a multiple of 64");
    if (!uniform_len && nbuf && (!d_offs || !d_lens)) return fail(SDFS_CDC_EINVAL, "offs/lens required without uniform_len");
    if ((reinterpret_cast<uintptr_t>(d_data) & 63) != 0) return fail(SDFS_CDC_EINVAL, "d_data must be 64-byte aligned");
    if (uniform_len) data_bytes = (uint64_t)nbuf * uniform_len;
    if (uniform_len && out->cap < slot_cap_for(e->prm, uniform_len))
        return fail(SDFS_CDC_ECAP, "cap %u < slot_cap %u", out->cap, slot_cap_for(e->prm, uniform_len));
    uint32_t sec_len, nsec, spec_cap;
    const WsNeed nd = pipeline_need(e, data_bytes, nbuf, uniform_len, out->cap, max_buf_len, &sec_len, &nsec, &spec_cap);
    Workspace* w = nullptr;
    int rc = ws_acquire(e, nd, s, &w, own);
    if (rc) return rc;
    rc = run_pipeline(e, w, d_data, data_bytes, d_offs, d_lens, nbuf, uniform_len, buffer_id_base, out, s, max_buf_len,
                      sec_len, nsec, spec_cap, ovf_to, early);
    const int rr = ws_release(w, s);  // even after a failed enqueue: what was enqueued completes first
    if (ovf_dev) *ovf_dev = w->overflow();
    return rc ? rc : rr;
}

// Fingerprints of n extents on workspace scratch (getHash in bulk).  Caller holds e->mu.
int hash_extents(DevEngine* e, const uint8_t* d_data, const uint64_t* d_offs, const uint32_t* d_lens,
                 const uint32_t* d_count, uint64_t n_max, uint8_t* d_digests, hipStream_t s,
                 Workspace* own = nullptr) {
    if (n_max == 0) return SDFS_CDC_OK;
    if (n_max > 0xFFFFFFFFull) return fail(SDFS_CDC_EINVAL, "more than 2^32 extents");
    WsNeed nd;
    nd.x_scratch = kExtentScratchWords + 2 * n_max;
    Workspace* w = nullptr;
    int rc = ws_acquire(e, nd, s, &w, own);
    if (rc) return rc;
    uint32_t* sc = w->x_scratch.p;
    ExtentArgs xa{d_lens, d_count, n_max, sc + kExtentScratchWords, sc + kExtentScratchWords + n_max,
                  sc + 1024, sc, sc + 512};
    hipError_t he = launch_extent_order(xa, s);
    if (he == hipSuccess) {
        HashArgs ha{};
        ha.zero_page = e->zero_page.p;
        ha.data = d_data;
        ha.offs = d_offs;
        ha.uniform_len = 0;
        ha.tasks = xa.tasks;
        ha.total = xa.total;
        ha.starts = xa.starts;
        ha.clens = d_lens;
        ha.cap = 1;
        ha.digests = d_digests;
        ha.algo = e->prm.hash_algo;
        he = launch_hash(ha, n_max, 0, s);
    }
    const int rr = ws_release(w, s);
    if (he != hipSuccess) return fail(SDFS_CDC_EHIP, "extent hashing: %s", hipGetErrorString(he));
    return rr;
}

// ---- host batch path (sdfs_cdc_get_chunks_batch) ----

// True when [p, p+n) lies inside ONE page-locked host allocation (hipHostMalloc or
// hipHostRegister), so the H2D copy may read it in place.
bool host_range_pinned(const uint8_t* p, uint64_t n) {
    if (!n) return false;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess || a.type != hipMemoryTypeHost) {
        (void)hipGetLastError();  // pageable memory reports an error here: clear it
        return false;
    }
    void* start = nullptr;
    size_t size = 0;
    if (hipPointerGetAttribute(&start, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR, (hipDeviceptr_t)p) != hipSuccess ||
        hipPointerGetAttribute(&size, HIP_POINTER_ATTRIBUTE_RANGE_SIZE, (hipDeviceptr_t)p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    const uint8_t* s = static_cast<const uint8_t*>(start);
    return s <= p && p + n <= s + size;
}

// Results of the batch in slot `sl` (synchronises on it) -> the caller's arrays.
int drain_slot(DevEngine* e, HostSlot& sl, uint32_t* counts, uint32_t* starts, uint32_t* lens_out,
               uint8_t* digests, uint32_t cap) {
    sl.busy = false;
    HIP_TRY(hipEventSynchronize(sl.done));
    const uint32_t n = sl.n, dcap = sl.dcap;
    const uint64_t nout = (uint64_t)n * dcap;
    const uint32_t* pc = reinterpret_cast<const uint32_t*>(sl.pin_out);
    const uint32_t* ps = pc + n;
    const uint32_t* pl = ps + nout;
    const uint32_t* povf = pl + nout;
    const uint8_t* pd = reinterpret_cast<const uint8_t*>(povf + 16);
    if (*povf) return fail(SDFS_CDC_EHIP, "internal: chunk slot overflow");
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t c = pc[i];
        if (c > cap) return fail(SDFS_CDC_ECAP, "buffer %u has %u chunks > cap %u", sl.b0 + i, c, cap);
        counts[sl.b0 + i] = c;
        const uint64_t so = (uint64_t)i * dcap, dst = (uint64_t)(sl.b0 + i) * cap;
        memcpy(starts + dst, ps + so, c * 4ull);
        memcpy(lens_out + dst, pl + so, c * 4ull);
        if (digests)
            for (uint32_t k = 0; k < c; k++)
                memcpy(digests + (dst + k) * e->digest_len, pd + (so + k) * 32, e->digest_len);
    }
    return SDFS_CDC_OK;
}

// Host buffers -> device, pipeline, device -> host, double-buffered: batch i is packed into
// pinned slot i%2 (copy_threads threads) while the GPU copies in and chunks batch i-1, and the
// results of batch i-2 are unpacked once its slot is needed again.  H2D runs on its own
// stream; pipeline and D2H on the engine stream.  Caller holds e->mu.
int host_batch_impl(DevEngine* e, const uint8_t* base, const uint64_t* offs, const uint32_t* lens,
                    uint32_t nbuf, uint32_t* counts, uint32_t* starts, uint32_t* lens_out, uint8_t* digests,
                    uint32_t cap) {
    // 256 MiB per slot: smaller batches leave most CUs idle and pay the per-batch fixed costs
    // (64 MiB: 26.5 GiB/s end to end, 256 MiB: 45.9 GiB/s from pinned memory; scripts/h2d_probe.py)
    const uint64_t staging = e->prm.max_batch_bytes ? e->prm.max_batch_bytes : (256ull << 20);
    if (!e->pool && e->copy_threads > 1) e->pool.reset(new CopyPool(e->copy_threads - 1));
    hipStream_t s = e->stream;
    std::vector<CopyPiece> pieces;
    uint32_t b0 = 0, k = 0;
    uint64_t lo = UINT64_MAX, hi = 0;
    for (uint32_t i = 0; i < nbuf; i++) {
        lo = std::min<uint64_t>(lo, offs[i]);
        hi = std::max<uint64_t>(hi, offs[i] + lens[i]);
    }
    const bool host_pinned = hi > lo && host_range_pinned(base + lo, hi - lo);
    while (b0 < nbuf) {
        HostSlot& sl = e->hs[k++ & 1];
        if (sl.busy) {
            const int rc = drain_slot(e, sl, counts, starts, lens_out, digests, cap);
            if (rc) return rc;
        }
        // pack as many buffers as fit (at 64-byte aligned offsets)
        uint64_t bytes = 0, maxlen = 1;
        uint32_t b1 = b0;
        while (b1 < nbuf) {
            const uint64_t need = (lens[b1] + 63ull) & ~63ull;
            if (b1 > b0 && bytes + need > staging) break;
            bytes += need;
            maxlen = std::max<uint64_t>(maxlen, lens[b1]);
            b1++;
        }
        const uint32_t n = b1 - b0;
        const uint32_t dcap = slot_cap_for(e->prm, maxlen);
        // Pinned input whose buffers sit back to back at 64-byte multiples: copy it to the GPU
        // straight from the caller's memory (no staging).
        bool direct = host_pinned;
        for (uint32_t i = 0; direct && i < n; i++)
            direct = (lens[b0 + i] & 63u) == 0 && (i == 0 || offs[b0 + i] == offs[b0 + i - 1] + lens[b0 + i - 1]);
        const uint64_t meta_at = direct ? 0 : ((bytes + 63) & ~63ull);
        int rc = pinned_ensure(&sl.pin_in, &sl.pin_in_n, meta_at + n * 12ull + 64);
        if (rc) return rc;
        uint64_t* hoffs = reinterpret_cast<uint64_t*>(sl.pin_in + meta_at);
        uint32_t* hlens = reinterpret_cast<uint32_t*>(hoffs + n);
        pieces.clear();
        uint64_t o = 0;
        constexpr size_t kPiece = 1u << 20;
        for (uint32_t i = 0; i < n; i++) {
            const uint8_t* src = base + offs[b0 + i];
            if (!direct)
                for (size_t q = 0; q < lens[b0 + i]; q += kPiece)
                    pieces.push_back({sl.pin_in + o + q, src + q, std::min<size_t>(kPiece, lens[b0 + i] - q)});
            hoffs[i] = o;
            hlens[i] = lens[b0 + i];
            o += (lens[b0 + i] + 63ull) & ~63ull;
        }
        if (e->pool && bytes >= (4u << 20))
            e->pool->run(pieces);
        else
            for (const auto& x : pieces) memcpy(x.dst, x.src, x.n);
        HIP_TRY(sl.data.ensure(std::max<uint64_t>(bytes, 64)));
        HIP_TRY(sl.offs.ensure(n));
        HIP_TRY(sl.lens.ensure(n));
        HIP_TRY(sl.counts.ensure(n));
        HIP_TRY(sl.starts.ensure((uint64_t)n * dcap));
        HIP_TRY(sl.clens.ensure((uint64_t)n * dcap));
        HIP_TRY(sl.digests.ensure((uint64_t)n * dcap * 32));
        HIP_TRY(sl.total.ensure(1));
        const uint64_t nout = (uint64_t)n * dcap;
        rc = pinned_ensure(&sl.pin_out, &sl.pin_out_n, n * 4ull + nout * 8 + 64 + nout * 32 + 64);
        if (rc) return rc;
        HIP_TRY(hipMemcpyAsync(sl.data.p, direct ? base + offs[b0] : sl.pin_in, bytes, hipMemcpyHostToDevice,
                               e->s_h2d));
        HIP_TRY(hipMemcpyAsync(sl.offs.p, hoffs, n * 8ull, hipMemcpyHostToDevice, e->s_h2d));
        HIP_TRY(hipMemcpyAsync(sl.lens.p, hlens, n * 4ull, hipMemcpyHostToDevice, e->s_h2d));
        HIP_TRY(hipEventRecord(sl.h2d, e->s_h2d));
        HIP_TRY(hipStreamWaitEvent(s, sl.h2d, 0));
        sdfs_cdc_dev_out out{};
        out.counts = sl.counts.p;
        out.starts = sl.starts.p;
        out.lens = sl.clens.p;
        out.digests = sl.digests.p;
        out.cap = dcap;
        out.total = sl.total.p;
        const uint32_t* ovf = nullptr;
        rc = device_run(e, sl.data.p, bytes, sl.offs.p, sl.lens.p, n, 0, 0, &out, s, maxlen, &ovf);
        if (rc) return rc;
        // results back through pinned memory: counts | starts | lens | overflow flag (64 B) | digests
        uint32_t* pc = reinterpret_cast<uint32_t*>(sl.pin_out);
        uint32_t* ps = pc + n;
        uint32_t* pl = ps + nout;
        uint32_t* povf = pl + nout;
        uint8_t* pd = reinterpret_cast<uint8_t*>(povf + 16);
        HIP_TRY(hipMemcpyAsync(pc, out.counts, n * 4ull, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipMemcpyAsync(ps, out.starts, nout * 4, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipMemcpyAsync(pl, out.lens, nout * 4, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipMemcpyAsync(povf, ovf, 4, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipMemcpyAsync(pd, out.digests, nout * 32, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipEventRecord(sl.done, s));
        sl.busy = true;
        sl.b0 = b0;
        sl.n = n;
        sl.dcap = dcap;
        b0 = b1;
    }
    // the older batch first
    for (int j = 0; j < 2; j++) {
        HostSlot& sl = e->hs[(k + j) & 1];
        if (sl.busy) {
            const int rc = drain_slot(e, sl, counts, starts, lens_out, digests, cap);
            if (rc) return rc;
        }
    }
    return SDFS_CDC_OK;
}

int host_batch(DevEngine* e, const uint8_t* base, const uint64_t* offs, const uint32_t* lens, uint32_t nbuf,
               uint32_t* counts, uint32_t* starts, uint32_t* lens_out, uint8_t* digests, uint32_t cap) {
    if (nbuf == 0) return SDFS_CDC_OK;
    const int rc = host_batch_impl(e, base, offs, lens, nbuf, counts, starts, lens_out, digests, cap);
    if (rc) {  // leave no batch in flight behind a failed call
        (void)hipStreamSynchronize(e->s_h2d);
        (void)hipStreamSynchronize(e->stream);
        e->hs[0].busy = e->hs[1].busy = false;
    }
    return rc;
}

// Direct getHash (inputs larger than a queue slot, or the queue disabled).  Caller holds e->mu.
int get_hash_direct(DevEngine* e, const uint8_t* data, uint64_t len, uint8_t* digest) {
    hipStream_t s = e->stream;
    int rc = pinned_ensure(&e->pin_data, &e->pin_data_n, len + 256);
    if (rc) return rc;
    if (len) memcpy(e->pin_data, data, len);
    uint32_t* ctl = reinterpret_cast<uint32_t*>(e->pin_data + ((len + 63) & ~63ull));
    ctl[0] = 0;                  // starts[0]
    ctl[1] = (uint32_t)len;      // lens[0]
    ctl[2] = 0;                  // tasks[0]
    ctl[3] = 1;                  // total
    HIP_TRY(e->h_data.ensure(std::max<uint64_t>(len, 64) + 64));
    HIP_TRY(e->o_starts.ensure(4));
    HIP_TRY(e->o_digests.ensure(32));
    if (len) HIP_TRY(hipMemcpyAsync(e->h_data.p, e->pin_data, len, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(e->o_starts.p, ctl, 16, hipMemcpyHostToDevice, s));
    HashArgs ha{};
    ha.zero_page = e->zero_page.p;
    ha.data = e->h_data.p;
    ha.uniform_len = 64;  // buffer 0 at offset 0
    ha.starts = e->o_starts.p;
    ha.clens = e->o_starts.p + 1;
    ha.tasks = e->o_starts.p + 2;
    ha.total = e->o_starts.p + 3;
    ha.cap = 1;
    ha.digests = e->o_digests.p;
    ha.algo = e->prm.hash_algo;
    HIP_TRY(launch_hash(ha, 1, 0, s));
    HIP_TRY(hipMemcpyAsync(ctl + 4, e->o_digests.p, 32, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    memcpy(digest, ctl + 4, e->digest_len);
    return SDFS_CDC_OK;
}

}  // namespace

// ---- coalescing-queue backend (host_queue.h) ----
struct QueueBackend {
    DevEngine* e;
    uint64_t slot_bytes;
    uint32_t max_reqs;
    uint64_t max_req;  // largest request the queue takes (CoalescingQueue::Config::max_req_bytes)

    uint64_t out_entries;  // chunk slots of a slot's result image: sum over its requests of dcap

    // Everything a slot needs is allocated here, once: growing a device buffer later would free
    // the old one, and hipFree waits for the whole device (every batch in flight).  (The pipeline
    // still checks every need, ws_acquire.)
    int prepare(QSlot& s) {
        HIP_TRY(hipSetDevice(e->prm.device));
        auto* d = new QSlotDev();
        s.dev = d;
        int rc = pinned_ensure(&s.in, &s.cap, slot_bytes);
        if (!rc) rc = pinned_ensure(&d->pin_meta, &d->pin_meta_n, (size_t)max_reqs * 24 + 64);
        d->ready_at = image_bytes(max_reqs, out_entries, max_reqs);
        if (!rc) rc = pinned_ensure(&d->pin_out, &d->pin_out_n, d->ready_at + 4ull * max_reqs);
        if (rc) return rc;
        s.cap = slot_bytes;
        HIP_TRY(d->data.ensure(slot_bytes));
        HIP_TRY(d->meta64.ensure(2ull * max_reqs));
        HIP_TRY(d->meta32.ensure(2ull * max_reqs));
        HIP_TRY(d->total.ensure(1));
        HIP_TRY(d->dimg.ensure(image_bytes(max_reqs, out_entries, max_reqs)));
        Workspace& w = d->ws;
        HIP_TRY(w.bitmap.ensure(slot_bytes / 32 + 2));
        HIP_TRY(w.small.ensure(kSmall + 8 + ((max_reqs + 3) & ~3u)));  // + early-completion counters
        HIP_TRY(w.rec_base.ensure(max_reqs));
        HIP_TRY(w.tasks.ensure(out_entries));
        HIP_TRY(w.seg_prefix.ensure(max_reqs + 1ull));
        HIP_TRY(w.x_scratch.ensure(kExtentScratchWords + 2ull * max_reqs));
        // a request long enough for the sectioned cut walk travels in a slot of its own (admits),
        // so one buffer's sections bound its speculative-walk scratch (pipeline_need)
        if (const uint32_t sec = resolve_section_len(max_req, e->prm.max_len, e->sec_log2)) {
            const uint64_t nsec = (max_req + sec - 1) / sec;
            HIP_TRY(w.spec_starts.ensure(nsec * (sec / (e->first_off + 1) + 2)));
            HIP_TRY(w.spec_cnt.ensure(nsec));
            HIP_TRY(w.spec_next.ensure(nsec));
            HIP_TRY(w.join.ensure(nsec * kJoinWords + 1));
        }
        HIP_TRY(hipEventCreateWithFlags(&d->kdone, hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&d->ws.free_ev, hipEventDisableTiming));
        // touch the pinned staging once here, not inside some caller's first request
        memset(s.in, 0, slot_bytes);
        memset(d->pin_out, 0, d->pin_out_n);
        return SDFS_CDC_OK;
    }

    // result image: counts[n] | starts[n*dcap] | lens[n*dcap] | flags[16] | digests | hash digests
    static uint64_t image_bytes(uint64_t n, uint64_t nout, uint64_t nh) {
        return ((n * 4 + nout * 8 + 64 + 15) & ~15ull) + nout * 32 + nh * 32 + 64;
    }

    // getChunks requests whose cut walk runs in sections (buffers of 4 MiB and more) travel alone
    bool is_long(uint64_t len) const { return resolve_section_len(len, e->prm.max_len, e->sec_log2) != 0; }

    bool admits(const QSlot& s, const QReq& r) {
        if (r.kind != QReq::kChunks) return true;
        if (!s.chunks.empty() && (is_long(r.len) || is_long(s.max_chunk_len))) return false;
        const uint64_t dcap = slot_cap_for(e->prm, std::max<uint64_t>(std::max<uint64_t>(s.max_chunk_len, r.len), 1));
        return (s.chunks.size() + 1) * dcap <= out_entries;
    }

    void release(QSlot& s) {
        auto* d = static_cast<QSlotDev*>(s.dev);
        (void)hipSetDevice(e->prm.device);
        if (d) {
            if (d->st) (void)hipStreamSynchronize(d->st);
            if (d->kdone) (void)hipEventDestroy(d->kdone);
            if (d->pin_meta) (void)hipHostFree(d->pin_meta);
            if (d->pin_out) (void)hipHostFree(d->pin_out);
            for (auto* b : {&d->total, &d->meta32}) b->release();
            d->dimg.release();
            d->ws.release_all();
            if (d->ws.free_ev) (void)hipEventDestroy(d->ws.free_ev);
            d->meta64.release();
            d->data.release();
            delete d;
        }
        if (s.in) (void)hipHostFree(s.in);
        s.in = nullptr;
        s.cap = 0;
        s.dev = nullptr;
    }

    // Runs on the queue's dispatcher thread: the error message goes with the slot to the callers.
    int launch(QSlot& s, int lane) {
        std::lock_guard<std::mutex> lk(e->mu);
        auto* d = static_cast<QSlotDev*>(s.dev);
        d->err.clear();
        hipStream_t st = e->qs[lane];  // lane < Config::lanes: created by queue_ready
        d->st = st;
        const int rc = launch_impl(s, d, st);
        if (rc) {
            d->err = g_last_error;
            (void)hipStreamSynchronize(st);  // nothing of a failed batch stays in flight
        }
        return rc;
    }

    // H2D of the slot's bytes and metadata, the CDC pipeline over its getChunks buffers, the
    // fingerprints of its getHash extents, D2H of the result image; all on one of the engine's
    // two queue streams (two batches in flight overlap on the device).  Caller holds e->mu.
    int launch_impl(QSlot& s, QSlotDev* d, hipStream_t st) {
        HIP_TRY(hipSetDevice(e->prm.device));
        const uint32_t n = (uint32_t)s.chunks.size(), nh = (uint32_t)s.hashes.size();
        const uint32_t dcap = n ? slot_cap_for(e->prm, std::max<uint64_t>(s.max_chunk_len, 1)) : 0;
        const uint64_t nout = (uint64_t)n * dcap;
        if (nout > out_entries || n > max_reqs || nh > max_reqs)
            return fail(SDFS_CDC_EHIP, "internal: queue slot over its result capacity");
        d->n = n;
        d->nh = nh;
        d->dcap = dcap;
        d->digests_at = (n * 4ull + nout * 8 + 64 + 15) & ~15ull;
        d->hdig_at = d->digests_at + nout * 32;
        d->img_bytes = d->hdig_at + 32ull * nh;
        int rc = SDFS_CDC_OK;
        uint64_t* m64 = reinterpret_cast<uint64_t*>(d->pin_meta);
        uint32_t* m32 = reinterpret_cast<uint32_t*>(m64 + 2ull * max_reqs);
        for (uint32_t i = 0; i < n; i++) {
            m64[i] = s.chunks[i]->off;
            m32[i] = (uint32_t)s.chunks[i]->len;
        }
        for (uint32_t j = 0; j < nh; j++) {
            m64[max_reqs + j] = s.hashes[j]->off;
            m32[max_reqs + j] = (uint32_t)s.hashes[j]->len;
        }
        if (s.lo) HIP_TRY(hipMemcpyAsync(d->data.p, s.in, s.lo, hipMemcpyHostToDevice, st));
        if (s.hi < s.cap) HIP_TRY(hipMemcpyAsync(d->data.p + s.hi, s.in + s.hi, s.cap - s.hi, hipMemcpyHostToDevice, st));
        // offsets/lengths only where a kernel reads them: the chunk requests' of a ragged pass (a
        // uniform pass of CHUNK_LENGTH buffers, the common case, needs none) and the getHash
        // extents' (two small copies instead of two 24 KiB ones on every pass)
        const bool uniform_pass = s.uniform_len && (s.uniform_len & 63) == 0;
        if (n && !uniform_pass) {
            HIP_TRY(hipMemcpyAsync(d->meta64.p, m64, 8ull * n, hipMemcpyHostToDevice, st));
            HIP_TRY(hipMemcpyAsync(d->meta32.p, m32, 4ull * n, hipMemcpyHostToDevice, st));
        }
        if (nh) {
            HIP_TRY(hipMemcpyAsync(d->meta64.p + max_reqs, m64 + max_reqs, 8ull * nh, hipMemcpyHostToDevice, st));
            HIP_TRY(hipMemcpyAsync(d->meta32.p + max_reqs, m32 + max_reqs, 4ull * nh, hipMemcpyHostToDevice, st));
        }
        uint32_t* dc = reinterpret_cast<uint32_t*>(d->dimg.p);
        uint32_t* dflag = dc + n + 2 * nout;
        if (n) {
            sdfs_cdc_dev_out out{};
            out.counts = dc;
            out.starts = dc + n;
            out.lens = dc + n + nout;
            out.digests = d->dimg.p + d->digests_at;
            out.cap = dcap;
            out.total = d->total.p;
            // every CHUNK_LENGTH flush buffer (the common case) takes the uniform layout and the
            // fused cut walk; mixed lengths (write-accelerator runs) the ragged one
            const uint32_t ul = uniform_pass ? s.uniform_len : 0;
            // Early completion: the header goes to the pinned image before the fingerprint, the
            // digests straight into it, and each buffer's ready word is set when its last chunk
            // is stored (HashArgs::done_ctr); the completer's poll wakes that caller then.
            EarlyDone ed;
            d->early = e->q_early;
            if (d->early) {
                out.digests = d->pin_out + d->digests_at;
                ed.hdr_src = d->dimg.p;
                ed.hdr_dst = d->pin_out;
                ed.hdr_bytes = d->digests_at;
                ed.ready = reinterpret_cast<uint32_t*>(d->pin_out + d->ready_at);
                ed.seq = (uint32_t)s.seq;
            }
            rc = device_run(e, d->data.p, s.lo, ul ? nullptr : d->meta64.p, ul ? nullptr : d->meta32.p, n, ul, 0,
                            &out, st, s.max_chunk_len, nullptr, &d->ws, dflag, d->early ? &ed : nullptr);
            if (rc) return rc;
        }
        if (nh) {
            rc = hash_extents(e, d->data.p, d->meta64.p + max_reqs, d->meta32.p + max_reqs, nullptr, nh,
                              d->dimg.p + d->hdig_at, st, &d->ws);
            if (rc) return rc;
        }
        if (n && d->early)  // header and digests are in the pinned image already: only getHash's
            HIP_TRY(launch_copy_out(d->dimg.p + d->hdig_at, d->pin_out + d->hdig_at, d->img_bytes - d->hdig_at, st));
        else
            HIP_TRY(launch_copy_out(d->dimg.p, d->pin_out, d->img_bytes, st));
        HIP_TRY(hipEventRecord(d->kdone, st));
        return SDFS_CDC_OK;
    }

    // Runs on the queue's completer thread.
    int wait(QSlot& s) {
        auto* d = static_cast<QSlotDev*>(s.dev);
        const int rc = wait_impl(d);
        if (rc && d->err.empty()) d->err = g_last_error;
        return rc;
    }

    // Runs on the queue's completer thread (host_queue.h Backend::poll): a chunk request is final
    // once its ready word holds this pass's number (the kernel set it after a system-scope fence
    // behind the buffer's last digest; its header was in the image before the fingerprint ran),
    // unless the walk flagged a slot overflow, which the batch's end reports.
    int poll(QSlot& s, uint8_t* ready, bool* finished) {
        auto* d = static_cast<QSlotDev*>(s.dev);
        if (d->early && d->n) {
            const volatile uint32_t* rd = reinterpret_cast<const volatile uint32_t*>(d->pin_out + d->ready_at);
            const volatile uint32_t* pflag = reinterpret_cast<const volatile uint32_t*>(d->pin_out) + d->n + 2ull * d->n * d->dcap;
            const uint32_t seq = (uint32_t)s.seq;
            for (uint32_t i = 0; i < d->n; i++)
                if (!ready[i] && rd[i] == seq) {
                    std::atomic_thread_fence(std::memory_order_acquire);
                    if (*pflag == 0) ready[i] = 1;
                }
        }
        const hipError_t q = hipEventQuery(d->kdone);
        if (q == hipErrorNotReady && d->early && d->n) {
            *finished = false;
            return SDFS_CDC_OK;
        }
        *finished = true;  // done, failed, or nothing to complete early: finish as wait does
        return wait(s);
    }

    // Kernels (the last one wrote the pinned result image) done -> done.
    int wait_impl(QSlotDev* d) {
        HIP_TRY(hipSetDevice(e->prm.device));
        HIP_TRY(hipEventSynchronize(d->kdone));
        if (d->n) {
            const uint32_t* pflag = reinterpret_cast<const uint32_t*>(d->pin_out) + d->n + 2ull * d->n * d->dcap;
            if (*pflag) return fail(SDFS_CDC_EHIP, "internal: chunk slot overflow");
        }
        return SDFS_CDC_OK;
    }
};

namespace {

// Starts the queue on first use.  Slot staging: 2 x CHUNK_LENGTH, at least 32 MiB (128 flush
// buffers of 256 KiB; 40 MiB backup buffers get 80 MiB slots), at most 512 MiB.
bool queue_ready(DevEngine* e) {
    std::lock_guard<std::mutex> lk(e->q_init);
    if (e->q_state) return e->q_state > 0;
    const uint64_t slot = std::min<uint64_t>(std::max<uint64_t>(32ull << 20, 2ull * e->prm.chunk_length), 512ull << 20);
    // result image: room for every 64-byte-aligned request's worst-case chunk list at the
    // shortest chunk length, plus two slots of tail per request
    const uint64_t shortest = std::max<uint64_t>(1, std::min<uint64_t>(e->first_off + 1, e->prm.max_len));
    CoalescingQueue<QueueBackend>::Config c;
    c.lanes = kQueueLanes;
#ifdef SDFS_TUNING
    if (const char* v = getenv("SDFS_Q_INFLIGHT")) c.lanes = std::max(1, std::min(atoi(v), kQueueInflight));
    if (const char* v = getenv("SDFS_Q_LINGER_US")) c.linger_us = (uint32_t)atoi(v);
    if (const char* v = getenv("SDFS_Q_SHARE_DIV")) c.share_div = (uint32_t)std::max(1, atoi(v));
#endif
    c.nslots = c.lanes + kQueueSpareSlots;
    c.max_reqs = 1024;
    c.max_req_bytes = slot / 2;
    {
        // Queue lanes, created with the queue (an engine that never sees a single-buffer call holds
        // no lane streams): each lane's passes are a long serial SHA-256 chain on a few CUs, so
        // lanes must run side by side.  Streams beyond GPU_MAX_HW_QUEUES share hardware queues, and
        // two lanes on one queue run their passes one after the other (the bench's process, where
        // torch's streams came first: lanes on queues 3,4,4,3, 1.6 instead of 2.9 GiB/s at 8
        // callers, profiles/r05/queue/).  A stream with a CU mask gets a hardware queue of its own;
        // the mask is every CU.  (Such a stream synchronises with the legacy null stream, which the
        // engine never uses.)
        if (hipSetDevice(e->prm.device) != hipSuccess) return false;
        std::vector<uint32_t> mask((e->num_cus + 31) / 32, 0xFFFFFFFFu);
        for (int l = 0; l < c.lanes; l++)
            if (!e->qs[l] && hipExtStreamCreateWithCUMask(&e->qs[l], (uint32_t)mask.size(), mask.data()) != hipSuccess) {
                e->qs[l] = nullptr;
                e->q_state = -1;  // the direct path serves every call
                return false;
            }
    }
    e->qb.reset(new QueueBackend{e, slot, 1024, slot / 2, slot / shortest + 2ull * 1024});
    e->q.reset(new CoalescingQueue<QueueBackend>(*e->qb, c));
    if (e->q->start() != 0) {  // pinned/device allocation failed: the direct path serves every call
        e->q.reset();
        e->qb.reset();
        e->q_state = -1;
        return false;
    }
    // first work on a stream sets up its hardware queue (milliseconds): do it for every lane now
    for (hipStream_t st : e->qs)
        if (st && (hipMemsetAsync(e->zero_page.p, 0, 256, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess))
            (void)hipGetLastError();
    e->q_state = 1;
    return true;
}

// A queued call's outcome: the batch's failure (its message becomes this thread's last error),
// a queue-level refusal, or the caller's own status.
int queue_result(int rc, const QSlot* s) {
    if (rc == kQueueStopped) return fail(SDFS_CDC_EINVAL, "engine is shutting down");
    if (rc == kQueueTooBig) return fail(SDFS_CDC_EINVAL, "request larger than a queue slot");
    if (rc && s && s->dev) {
        const auto* d = static_cast<const QSlotDev*>(s->dev);
        g_last_error = d->err.empty() ? "batch failed" : d->err;
    }
    return rc;
}

}  // namespace

// ---------------------------------------------------------------------------------------------
// One device (DevEngine): what a handle's call runs on once the set has picked the device.
// ---------------------------------------------------------------------------------------------
namespace {

int dev_create(const sdfs_cdc_params* p, int ordinal, std::unique_ptr<DevEngine>* out) {
    HIP_TRY(hipSetDevice(ordinal));
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, ordinal));
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(SDFS_CDC_ENODEV, "device %d is %s, this build targets gfx950", ordinal, prop.gcnArchName);
    std::unique_ptr<DevEngine> e(new DevEngine());
    e->prm = *p;
    e->prm.device = ordinal;
    e->degree = poly_degree(p->poly);
    if (p->pred_kind == SDFS_CDC_PRED_DIV) {
        // fp >= 0, so fp % 2^k == R < 2^k is the bitmask detector (fp & (2^k - 1)) == R: run the
        // mask kernels for it; any other divisor (or R >= D, never true) takes the f64 form
        const uint64_t dv = p->pred_div;
        if ((dv & (dv - 1)) == 0 && p->pred_rem < dv) {
            e->prm.pred_mask = dv - 1;
            e->prm.pred_value = p->pred_rem;
        } else {
            e->pred_div = true;
        }
    }
    e->num_cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    e->first_off = p->min_cmp == SDFS_CDC_MIN_GT ? p->min_len : (p->min_len ? p->min_len - 1 : 0);
    e->digest_len = p->hash_algo == SDFS_CDC_SHA256 ? 32 : (p->hash_algo == SDFS_CDC_SHA256_160 ? 20 : 16);
    if (p->flags & SDFS_CDC_FLAG_DIRECT) e->q_state = -1;
    // bins over SHA block counts: maxLen chunk = (max_len + 8)/64 + 1 blocks
    const uint32_t maxblocks = (p->max_len + 8) / 64 + 1;
    e->bin_shift = 0;
    while ((maxblocks >> e->bin_shift) >= (uint32_t)kMaxBins) e->bin_shift++;
    e->nbins = (maxblocks >> e->bin_shift) + 1;
    bool ok = hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) == hipSuccess &&
              hipStreamCreateWithFlags(&e->s_h2d, hipStreamNonBlocking) == hipSuccess;
    for (auto& sl : e->hs)
        ok = ok && hipEventCreateWithFlags(&sl.h2d, hipEventDisableTiming) == hipSuccess &&
             hipEventCreateWithFlags(&sl.done, hipEventDisableTiming) == hipSuccess;
    for (auto& w : e->ws) ok = ok && hipEventCreateWithFlags(&w.free_ev, hipEventDisableTiming) == hipSuccess;
    if (!ok) return fail(SDFS_CDC_EHIP, "stream/event creation failed");
#ifdef SDFS_TUNING
    // measurement-only overrides (tuning library; the product library reads no environment)
    if (const char* v = getenv("SDFS_COPY_THREADS")) e->copy_threads = std::max(1, std::min(atoi(v), 64));
    if (const char* v = getenv("SDFS_SCAN_VARIANT")) e->scan_variant = atoi(v);
    if (const char* v = getenv("SDFS_SEG_LEN")) e->seg_len = (uint32_t)atoi(v);
    if (const char* v = getenv("SDFS_HASH_VARIANT")) e->hash_variant = atoi(v);
    if (const char* v = getenv("SDFS_HASH_WG_PER_CU")) e->hash_wg_per_cu = std::max(1, atoi(v));
    if (const char* v = getenv("SDFS_HASH_SPLIT")) e->hash_split = atoi(v) != 0;
    if (const char* v = getenv("SDFS_SMALL_SEG")) e->small_seg = atoi(v) != 0;
    if (const char* v = getenv("SDFS_TINY_SCAN")) e->tiny_scan = atoi(v) != 0;
    if (const char* v = getenv("SDFS_Q_EARLY")) e->q_early = atoi(v) != 0;
    if (const char* v = getenv("SDFS_TINY_SEG_LEN")) {
        const int n = atoi(v);
        if (n >= 64 && n % 64 == 0) e->tiny_seg_len = (uint32_t)n;
    }
    if (const char* v = getenv("SDFS_SMALL_SEG_LEN")) {
        const uint32_t n = (uint32_t)atoi(v);
        if (n >= 256 && n % 256 == 0) e->small_seg_len = n;
    }
    if (const char* v = getenv("SDFS_LONG_SPLIT")) e->long_split = atoi(v) != 0;
    if (const char* v = getenv("SDFS_PAR_STITCH")) e->par_stitch = atoi(v) != 0;
    if (const char* v = getenv("SDFS_PIECE_WALK")) e->piece_walk = atoi(v) != 0;
    if (const char* v = getenv("SDFS_SKIP_WALK")) e->skip_walk = (uint32_t)std::max(0, std::min(atoi(v), 3));
    if (const char* v = getenv("SDFS_LIST_WALK")) e->list_walk = atoi(v) != 0;
    if (const char* v = getenv("SDFS_SCAN_DYN")) e->scan_dyn = atoi(v) != 0;
    if (const char* v = getenv("SDFS_SEC_LOG2")) e->sec_log2 = (uint32_t)std::max(16, std::min(atoi(v), 24));
    if (const char* v = getenv("SDFS_SCAN_PRIO")) e->scan_prio = atoi(v) != 0;
    if (e->scan_prio) {
        int lo = 0, hi = 0;
        if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess ||
            hipStreamCreateWithPriority(&e->s_scan, hipStreamNonBlocking, hi) != hipSuccess ||
            hipEventCreateWithFlags(&e->ev_fork, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&e->ev_join, hipEventDisableTiming) != hipSuccess)
            return fail(SDFS_CDC_EHIP, "scan-priority stream creation failed");
    }
    if (const char* v = getenv("SDFS_FRONT_SERIAL")) e->front_serial = atoi(v) != 0;
    if (const char* v = getenv("SDFS_FUSED_PROBE")) e->fused_probe = atoi(v);
    if (const char* v = getenv("SDFS_SPLIT_PACKED")) e->split_packed = atoi(v) != 0;
    if (const char* v = getenv("SDFS_SPLIT_SPREAD")) e->split_spread = atoi(v) != 0;
    if (const char* v = getenv("SDFS_SPLIT_BYBUF")) e->split_bybuf = atoi(v) != 0;
    if (const char* v = getenv("SDFS_SPLIT_MASKED")) e->split_masked = atoi(v) != 0;
    if (const char* v = getenv("SDFS_SMALL_BALLOT")) e->small_ballot = atoi(v) != 0;
    if (const char* v = getenv("SDFS_SCAN_MAX_BLOCK"))
        e->scan_max_block = (uint32_t)std::max(256, std::min(atoi(v), kScanThreads)) / 256 * 256;
#endif
    if (e->front_serial && hipEventCreateWithFlags(&e->ev_front, hipEventDisableTiming) != hipSuccess)
        return fail(SDFS_CDC_EHIP, "event creation failed");
    e->scan_info = scan_variant_info(e->scan_variant);
    if (e->scan_info.copies == 0 || e->seg_len == 0 || (e->seg_len % e->scan_info.blk) != 0)
        return fail(SDFS_CDC_EINVAL, "bad scan variant/segment length");
    if (e->pred_div && (e->scan_variant != 0 || !e->scan_info.mirror))
        return fail(SDFS_CDC_EINVAL, "the divisor predicate runs on the production scan only");
    std::vector<uint8_t> img = build_table_image(p->poly, p->window, e->scan_info.copies, e->scan_info.mirror != 0,
                                                 e->scan_info.pop_swap != 0);
    // on the engine's own non-blocking stream: the queue lanes are blocking streams (CU-masked),
    // so anything on the legacy null stream would wait for their passes in flight
    if (e->zero_page.ensure(256) != hipSuccess || hipMemsetAsync(e->zero_page.p, 0, 256, e->stream) != hipSuccess ||
        e->tab_image.ensure(img.size()) != hipSuccess ||
        hipMemcpyAsync(e->tab_image.p, img.data(), img.size(), hipMemcpyHostToDevice, e->stream) != hipSuccess ||
        hipStreamSynchronize(e->stream) != hipSuccess)
        return fail(SDFS_CDC_ENOMEM, "table upload failed");
    *out = std::move(e);
    return SDFS_CDC_OK;
}

}  // namespace

DevEngine::~DevEngine() {
    DevEngine* e = this;
    if (e->q) e->q->shutdown();  // drains what was placed, joins the queue threads
    e->q.reset();
    e->qb.reset();
    std::lock_guard<std::mutex> lk(e->mu);
    (void)hipSetDevice(e->prm.device);
    for (hipStream_t s : {e->stream, e->s_h2d, e->s_scan})
        if (s) (void)hipStreamSynchronize(s);
    for (hipStream_t s : e->qs)
        if (s) (void)hipStreamSynchronize(s);
    e->tab_image.release();
    e->zero_page.release();
    for (auto& w : e->ws) {
        w.release_all();
        if (w.free_ev) (void)hipEventDestroy(w.free_ev);
    }
    e->h_data.release();
    e->o_starts.release();
    e->o_digests.release();
    e->x_data.release();
    e->x_offs.release();
    e->x_lens.release();
    e->x_digests.release();
    if (e->pin_data) (void)hipHostFree(e->pin_data);
    for (auto& sl : e->hs) {
        if (sl.pin_in) (void)hipHostFree(sl.pin_in);
        if (sl.pin_out) (void)hipHostFree(sl.pin_out);
        for (auto* b : {&sl.counts, &sl.starts, &sl.clens, &sl.total}) b->release();
        sl.data.release();
        sl.offs.release();
        sl.lens.release();
        sl.digests.release();
        if (sl.h2d) (void)hipEventDestroy(sl.h2d);
        if (sl.done) (void)hipEventDestroy(sl.done);
    }
    e->pool.reset();
    for (auto& run : e->ev_runs)
        for (auto& ev : run.ev)
            if (ev) (void)hipEventDestroy(ev);
    for (hipStream_t s : {e->stream, e->s_h2d, e->s_scan})
        if (s) (void)hipStreamDestroy(s);
    for (hipEvent_t ev : {e->ev_fork, e->ev_join, e->ev_front})
        if (ev) (void)hipEventDestroy(ev);
    for (hipStream_t s : e->qs)
        if (s) (void)hipStreamDestroy(s);
}

namespace {

int dev_run_device(DevEngine* e, const uint8_t* d_data, uint32_t nbuf, uint32_t uniform_len, uint64_t buffer_id_base,
                   const sdfs_cdc_dev_out* out, hipStream_t s) {
    std::lock_guard<std::mutex> lk(e->mu);
    HIP_TRY(hipSetDevice(e->prm.device));
    return device_run(e, d_data, 0, nullptr, nullptr, nbuf, uniform_len, buffer_id_base, out, s, 0, nullptr);
}

int dev_run_device_ragged(DevEngine* e, const uint8_t* d_data, uint64_t data_bytes, const uint64_t* d_offs,
                          const uint32_t* d_lens, uint32_t nbuf, uint64_t buffer_id_base, const sdfs_cdc_dev_out* out,
                          hipStream_t s) {
    std::lock_guard<std::mutex> lk(e->mu);
    HIP_TRY(hipSetDevice(e->prm.device));
    // the longest buffer is not known on the host: a few buffers sharing data_bytes are treated as
    // long (LDS-staged cut walk), many as their mean length
    const uint64_t max_len_hint = nbuf <= 4u * (uint32_t)e->num_cus ? data_bytes : data_bytes / (nbuf ? nbuf : 1);
    return device_run(e, d_data, data_bytes, d_offs, d_lens, nbuf, 0, buffer_id_base, out, s, max_len_hint, nullptr);
}

int dev_set_timing_mask(DevEngine* e, int nruns, uint32_t stage_mask) {
    std::lock_guard<std::mutex> lk(e->mu);
    e->timing_mask = stage_mask;
    HIP_TRY(hipSetDevice(e->prm.device));
    while ((int)e->ev_runs.size() < nruns) {
        DevEngine::TimedRun r;
        r.ev.assign(kEvPerRun, nullptr);
        for (auto& ev : r.ev) HIP_TRY(hipEventCreate(&ev));
        e->ev_runs.push_back(std::move(r));
    }
    e->timing_slots = nruns;
    e->runs_recorded = 0;
    return SDFS_CDC_OK;
}

int dev_kernel_times(DevEngine* e, const char** names, float* ms, int n) {
    std::lock_guard<std::mutex> lk(e->mu);
    HIP_TRY(hipSetDevice(e->prm.device));
    if (e->timing_slots == 0 || e->runs_recorded == 0) return 0;
    const uint64_t nr = std::min<uint64_t>(e->runs_recorded, (uint64_t)e->timing_slots);
    double sum[kNumTimed] = {};
    for (uint64_t r = 0; r < nr; r++) {
        auto& run = e->ev_runs[(e->runs_recorded - 1 - r) % e->timing_slots];
        for (size_t i = 0; i < run.kid.size(); i++) {
            HIP_TRY(hipEventSynchronize(run.ev[2 * i + 1]));
            float t = 0;
            HIP_TRY(hipEventElapsedTime(&t, run.ev[2 * i], run.ev[2 * i + 1]));
            sum[run.kid[i]] += t;
        }
    }
    int k = 0;
    for (int i = 0; i < kNumTimed && k < n; i++, k++) {
        if (names) names[k] = kKernelNames[i];
        if (ms) ms[k] = (float)(sum[i] / nr);
    }
    return k;
}

int dev_get_chunks_batch(DevEngine* e, const uint8_t* base, const uint64_t* offs, const uint32_t* lens, uint32_t nbuf,
                         uint32_t* counts, uint32_t* starts, uint32_t* lens_out, uint8_t* digests, uint32_t cap) {
    std::lock_guard<std::mutex> lk(e->mu);
    HIP_TRY(hipSetDevice(e->prm.device));
    return host_batch(e, base, offs, lens, nbuf, counts, starts, lens_out, digests, cap);
}

// getChunks of one buffer whose `len` bytes `fill` writes (into the queue's pinned staging when
// the queue takes the request, else into a temporary buffer for the direct path).
template <class Fill>
int dev_get_chunks(DevEngine* e, uint32_t len, Fill&& fill, uint32_t* starts, uint32_t* lens, uint8_t* digests,
                   uint32_t cap, uint32_t* count) {
    if (queue_ready(e) && e->q->accepts(len)) {
        QReq r;
        r.kind = QReq::kChunks;
        r.len = len;
        const uint32_t dl = e->digest_len;
        const int rc = e->q->run_fill(r, fill, [&](const QSlot& s, const QReq& q, int status) -> int {
            if (status) return queue_result(status, &s);
            const auto* d = static_cast<const QSlotDev*>(s.dev);
            const uint32_t* pc = reinterpret_cast<const uint32_t*>(d->pin_out);
            const uint32_t c = pc[q.idx];
            if (c > cap) return fail(SDFS_CDC_ECAP, "buffer has %u chunks > cap %u", c, cap);
            const uint64_t so = (uint64_t)q.idx * d->dcap, nout = (uint64_t)d->n * d->dcap;
            memcpy(starts, pc + d->n + so, c * 4ull);
            memcpy(lens, pc + d->n + nout + so, c * 4ull);
            if (digests) {
                const uint8_t* pd = d->pin_out + d->digests_at + so * 32;
                for (uint32_t k = 0; k < c; k++) memcpy(digests + (uint64_t)k * dl, pd + k * 32ull, dl);
            }
            *count = c;
            return SDFS_CDC_OK;
        });
        return rc == kQueueStopped || rc == kQueueTooBig ? queue_result(rc, nullptr) : rc;
    }
    std::unique_ptr<uint8_t[]> tmp(new (std::nothrow) uint8_t[len]);
    if (!tmp) return fail(SDFS_CDC_ENOMEM, "getChunks: %u bytes of host memory", len);
    const int frc = fill(tmp.get());
    if (frc) return frc;
    const uint64_t off = 0;
    std::lock_guard<std::mutex> lk(e->mu);
    HIP_TRY(hipSetDevice(e->prm.device));
    return host_batch(e, tmp.get(), &off, &len, 1, count, starts, lens, digests, cap);
}

int dev_get_hash(DevEngine* e, const uint8_t* data, uint64_t len, uint8_t* digest) {
    if (queue_ready(e) && e->q->accepts(len)) {
        QReq r;
        r.kind = QReq::kHash;
        r.src = data;
        r.len = len;
        const uint32_t dl = e->digest_len;
        const int rc = e->q->run(r, [&](const QSlot& s, const QReq& q, int status) -> int {
            if (status) return queue_result(status, &s);
            const auto* d = static_cast<const QSlotDev*>(s.dev);
            memcpy(digest, d->pin_out + d->hdig_at + 32ull * q.idx, dl);
            return SDFS_CDC_OK;
        });
        return rc == kQueueStopped || rc == kQueueTooBig ? queue_result(rc, nullptr) : rc;
    }
    std::lock_guard<std::mutex> lk(e->mu);
    HIP_TRY(hipSetDevice(e->prm.device));
    return get_hash_direct(e, data, len, digest);
}

int dev_get_hash_batch(DevEngine* e, const uint8_t* base, const uint64_t* offs, const uint32_t* lens, uint32_t n,
                       uint8_t* digests) {
    std::lock_guard<std::mutex> lk(e->mu);
    HIP_TRY(hipSetDevice(e->prm.device));
    hipStream_t s = e->stream;
    // pack the chunks 16-byte aligned into pinned staging, one H2D
    std::vector<uint64_t> po(n);
    uint64_t bytes = 0;
    for (uint32_t i = 0; i < n; i++) {
        po[i] = bytes;
        bytes += (lens[i] + 15ull) & ~15ull;
    }
    int rc = pinned_ensure(&e->pin_data, &e->pin_data_n, bytes + 64);
    if (rc) return rc;
    for (uint32_t i = 0; i < n; i++) memcpy(e->pin_data + po[i], base + offs[i], lens[i]);
    HIP_TRY(e->x_data.ensure(bytes + 64));
    HIP_TRY(e->x_offs.ensure(n));
    HIP_TRY(e->x_lens.ensure(n));
    HIP_TRY(e->x_digests.ensure(32ull * n));
    HIP_TRY(hipMemcpyAsync(e->x_data.p, e->pin_data, bytes, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(e->x_offs.p, po.data(), 8ull * n, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(e->x_lens.p, lens, 4ull * n, hipMemcpyHostToDevice, s));
    rc = hash_extents(e, e->x_data.p, e->x_offs.p, e->x_lens.p, nullptr, n, e->x_digests.p, s);
    if (rc) {
        (void)hipStreamSynchronize(s);
        return rc;
    }
    std::vector<uint8_t> dg(32ull * n);
    HIP_TRY(hipMemcpyAsync(dg.data(), e->x_digests.p, 32ull * n, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    const uint32_t dl = (uint32_t)e->digest_len;
    for (uint32_t i = 0; i < n; i++) memcpy(digests + (uint64_t)dl * i, dg.data() + 32ull * i, dl);
    return SDFS_CDC_OK;
}

// ---------------------------------------------------------------------------------------------
// Handles and shared sets (engine_share.h): the C-ABI below.
// ---------------------------------------------------------------------------------------------
typedef Registry<DevEngine> Reg;
typedef Handle<DevEngine> H;
typedef SharedSet<DevEngine> Set;

Reg& reg() {
    static Reg* r = new Reg();  // never destroyed: no engine teardown runs after the HIP runtime's exit
    return *r;
}

// The gfx950 ordinals a parameter block names: device_mask (bit i = ordinal i) when set, else
// `device` (>= 0), else (-1) every gfx950 device.
int device_set(const sdfs_cdc_params* p, std::vector<int>* ords) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        (void)hipGetLastError();
        return fail(SDFS_CDC_ENODEV, "no HIP device");
    }
    ords->clear();
    if (p->device_mask) {
        for (int i = 0; i < 64; i++)
            if ((p->device_mask >> i) & 1) {
                if (i >= ndev) return fail(SDFS_CDC_ENODEV, "device_mask names device %d of %d", i, ndev);
                ords->push_back(i);
            }
        return SDFS_CDC_OK;
    }
    if (p->device >= 0) {
        if (p->device >= ndev) return fail(SDFS_CDC_ENODEV, "device %d of %d", p->device, ndev);
        ords->push_back(p->device);
        return SDFS_CDC_OK;
    }
    if (p->device != -1) return fail(SDFS_CDC_EINVAL, "device %d (-1 = every gfx950 device)", p->device);
    for (int i = 0; i < ndev; i++) {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, i) == hipSuccess && strncmp(prop.gcnArchName, "gfx950", 6) == 0)
            ords->push_back(i);
    }
    if (ords->empty()) return fail(SDFS_CDC_ENODEV, "no gfx950 device among %d", ndev);
    return SDFS_CDC_OK;
}

// Engines are shared between handles whose parameters (other than the device fields) and device
// sets are equal.
std::string share_key(const sdfs_cdc_params* p, const std::vector<int>& ords) {
    char buf[384];
    snprintf(buf, sizeof(buf), "%llx/%u/%u/%u/%u/%llx/%llx/%u/%u/%x/%llx/%u/%llx/%llx|",
             (unsigned long long)p->poly, p->window, p->min_len, p->max_len, p->chunk_length,
             (unsigned long long)p->pred_mask, (unsigned long long)p->pred_value, p->min_cmp, p->hash_algo, p->flags,
             (unsigned long long)p->max_batch_bytes, p->pred_kind, (unsigned long long)p->pred_div,
             (unsigned long long)p->pred_rem);
    std::string k(buf);
    for (int o : ords) k += std::to_string(o) + ",";
#ifdef SDFS_TUNING
    // measurement build: engines created under different SDFS_* settings (A/B in one process,
    // scripts/ab.py) must not share
    for (char** ev = ::environ; ev && *ev; ev++)
        if (strncmp(*ev, "SDFS_", 5) == 0) k += std::string("|") + *ev;
#endif
    return k;
}

#define USE_OR_FAIL(u, e)                                                            \
    Reg::Use u(reg(), e);                                                            \
    if (!u.ok()) return fail(SDFS_CDC_EINVAL, "not a live engine handle");

// The set's device holding device pointer p (set order index); a set of one takes it as is.
int dev_of_ptr(Set& s, const void* p, size_t* idx) {
    *idx = 0;
    if (s.ndev() == 1) return SDFS_CDC_OK;
    hipPointerAttribute_t a;
    if (!p || hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return fail(SDFS_CDC_EINVAL, "not a device pointer: %p", p);
    }
    for (size_t i = 0; i < s.ndev(); i++)
        if (s.ordinals[i] == a.device) {
            *idx = i;
            return SDFS_CDC_OK;
        }
    return fail(SDFS_CDC_EINVAL, "pointer %p is on device %d, outside this engine's device set", p, a.device);
}

// ---- in-process RCCL all-gather of the fingerprint tables ----
// RCCL is opened on first use (dlopen), so the library loads, and serves every other call,
// without it; the exchange itself fails loudly when it is missing.
struct RcclApi {
    typedef int (*init_all_t)(void**, int, const int*);
    typedef int (*all_gather_t)(const void*, void*, size_t, int, void*, hipStream_t);
    typedef int (*group_t)(void);
    typedef int (*destroy_t)(void*);
    typedef const char* (*errstr_t)(int);
    init_all_t init_all = nullptr;
    all_gather_t all_gather = nullptr;
    group_t group_start = nullptr, group_end = nullptr;
    destroy_t destroy = nullptr;
    errstr_t errstr = nullptr;
};
constexpr int kNcclUint8 = 1, kNcclUint32 = 3;  // ncclDataType_t (rccl.h)

const RcclApi* rccl_api() {
    static RcclApi api;
    static std::once_flag once;
    static bool ok = false;
    std::call_once(once, [] {
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
        api.init_all = (RcclApi::init_all_t)dlsym(h, "ncclCommInitAll");
        api.all_gather = (RcclApi::all_gather_t)dlsym(h, "ncclAllGather");
        api.group_start = (RcclApi::group_t)dlsym(h, "ncclGroupStart");
        api.group_end = (RcclApi::group_t)dlsym(h, "ncclGroupEnd");
        api.destroy = (RcclApi::destroy_t)dlsym(h, "ncclCommDestroy");
        api.errstr = (RcclApi::errstr_t)dlsym(h, "ncclGetErrorString");
        ok = api.init_all && api.all_gather && api.group_start && api.group_end && api.destroy && api.errstr;
    });
    return ok ? &api : nullptr;
}

// Per set: one communicator per device (ncclCommInitAll over the set's ordinals) and a small
// device buffer per device for the gathered counts.
struct Coll {
    std::vector<void*> comms;
    std::vector<uint32_t*> d_counts;  // [ndev] u32 on each device
    uint32_t* h_counts = nullptr;     // pinned [ndev]
    std::vector<int> ords;
    ~Coll() {
        const RcclApi* api = rccl_api();
        for (size_t i = 0; i < comms.size(); i++)
            if (comms[i] && api) api->destroy(comms[i]);
        for (size_t i = 0; i < d_counts.size(); i++)
            if (d_counts[i]) {
                (void)hipSetDevice(ords[i]);
                (void)hipFree(d_counts[i]);
            }
        if (h_counts) (void)hipHostFree(h_counts);
    }
};

#define NCCL_TRY(api, expr)                                                                         \
    do {                                                                                            \
        const int _r = (expr);                                                                      \
        if (_r != 0) return fail(SDFS_CDC_EHIP, "%s failed: %s", #expr, (api)->errstr(_r));          \
    } while (0)

// One all-gather per device of the set inside one RCCL group.  ncclGroupEnd runs on every path
// once ncclGroupStart succeeded, so a failing device never leaves the group open on this thread.
// Every device is selected once BEFORE the group opens: a hipSetDevice failure is not an RCCL
// error, so inside the group it would let ncclGroupEnd launch the all-gathers of the devices
// before it, whose kernels would then wait for peers that were never enqueued.  Failures RCCL
// itself reports (an ncclAllGather that fails inside the group) are the group's to abort.
template <class Issue>
int grouped_all_gather(const RcclApi* api, Set& s, Issue&& issue) {
    for (int i = 0; i < (int)s.ndev(); i++) {
        const hipError_t he = hipSetDevice(s.ordinals[i]);
        if (he != hipSuccess) {
            (void)hipGetLastError();
            return fail(SDFS_CDC_EHIP, "hipSetDevice(%d) failed before the all-gather group: %s", s.ordinals[i],
                        hipGetErrorString(he));
        }
    }
    const int g = api->group_start();
    if (g) return fail(SDFS_CDC_EHIP, "ncclGroupStart failed: %s", api->errstr(g));
    int rc = SDFS_CDC_OK;
    for (int i = 0; i < (int)s.ndev() && rc == SDFS_CDC_OK; i++) {
        const hipError_t he = hipSetDevice(s.ordinals[i]);
        if (he != hipSuccess) {
            rc = fail(SDFS_CDC_EHIP, "hipSetDevice(%d) failed: %s", s.ordinals[i], hipGetErrorString(he));
            break;
        }
        const int r = issue(i);
        if (r) rc = fail(SDFS_CDC_EHIP, "ncclAllGather on device %d failed: %s", s.ordinals[i], api->errstr(r));
    }
    const int e = api->group_end();
    if (rc) return rc;
    if (e) return fail(SDFS_CDC_EHIP, "ncclGroupEnd failed: %s", api->errstr(e));
    return SDFS_CDC_OK;
}

int coll_ready(Set& s, Coll** out) {
    std::lock_guard<std::mutex> lk(s.coll_mu);
    if (s.coll) {
        *out = static_cast<Coll*>(s.coll.get());
        return SDFS_CDC_OK;
    }
    const RcclApi* api = rccl_api();
    if (!api) return fail(SDFS_CDC_ENODEV, "RCCL (librccl.so.1) not loadable: %s", dlerror());
    std::shared_ptr<Coll> c(new Coll());
    const int n = (int)s.ndev();
    c->ords = s.ordinals;
    c->comms.assign(n, nullptr);
    c->d_counts.assign(n, nullptr);
    NCCL_TRY(api, api->init_all(c->comms.data(), n, s.ordinals.data()));
    for (int i = 0; i < n; i++) {
        HIP_TRY(hipSetDevice(s.ordinals[i]));
        HIP_TRY(hipMalloc(reinterpret_cast<void**>(&c->d_counts[i]), 4ull * n));
    }
    HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&c->h_counts), 4ull * n, hipHostMallocDefault));
    s.coll = c;
    *out = c.get();
    return SDFS_CDC_OK;
}

}  // namespace

extern "C" {

int sdfs_cdc_abi_version(void) { return SDFS_CDC_ABI_VERSION; }

const char* sdfs_cdc_last_error(void) { return g_last_error.c_str(); }

int sdfs_cdc_params_default(sdfs_cdc_params* p, int backup_volume) {
    if (!p) return fail(SDFS_CDC_EINVAL, "null params");
    memset(p, 0, sizeof(*p));
    p->poly = 10923124345206883ull;                        // VariableSha256HashEngine.java:41
    p->window = 48;                                        // HashFunctionPool.java:51
    p->min_len = 4 * 1024 - 1;                             // Main.java:189
    p->max_len = backup_volume ? 128 * 1024 : 32 * 1024;   // VolumeConfigWriter.java:96,301
    p->chunk_length = backup_volume ? 40960u * 1024 : 256u * 1024;  // VolumeConfigWriter.java:63,304
    p->pred_mask = 0xFFF;                                  // SURVEY.md A.3 (knob; parity unpinned)
    p->pred_value = 0;
    p->min_cmp = SDFS_CDC_MIN_GT;
    p->hash_algo = SDFS_CDC_SHA256;                        // VolumeConfigWriter.java:109
    p->device = 0;
    p->max_batch_bytes = 0;
    p->device_mask = 0;
    return SDFS_CDC_OK;
}

int sdfs_cdc_create(const sdfs_cdc_params* p, sdfs_cdc_engine** out) {
    if (!out) return fail(SDFS_CDC_EINVAL, "null out");
    *out = nullptr;
    int rc = validate(p);
    if (rc) return rc;
    std::vector<int> ords;
    rc = device_set(p, &ords);
    if (rc) return rc;
    void* h = nullptr;
    rc = reg().create(share_key(p, ords), ords,
                      [p](int ord, std::unique_ptr<DevEngine>* d) { return dev_create(p, ord, d); }, &h);
    if (rc) return rc;
    *out = reinterpret_cast<sdfs_cdc_engine*>(h);
    return SDFS_CDC_OK;
}

int sdfs_cdc_destroy(sdfs_cdc_engine* e) {
    if (!e) return SDFS_CDC_OK;
    if (!reg().destroy(e)) return fail(SDFS_CDC_EINVAL, "not a live engine handle");
    return SDFS_CDC_OK;
}

int sdfs_cdc_device_count(const sdfs_cdc_engine* e) {
    USE_OR_FAIL(u, e);
    return (int)u.set().ndev();
}

int sdfs_cdc_device_ordinal(const sdfs_cdc_engine* e, int i) {
    USE_OR_FAIL(u, e);
    if (i < 0 || (size_t)i >= u.set().ndev()) return fail(SDFS_CDC_EINVAL, "device index %d", i);
    return u.set().ordinals[i];
}

int sdfs_cdc_share_count(const sdfs_cdc_engine* e) {
    USE_OR_FAIL(u, e);
    return reg().refs_of(u.set());
}

int sdfs_cdc_is_variable_length(const sdfs_cdc_engine* e) {
    USE_OR_FAIL(u, e);
    return 1;
}
int sdfs_cdc_get_max_len(const sdfs_cdc_engine* e) {
    Reg::Use u(reg(), e);
    return u.ok() ? (int)u.set().devs[0]->prm.chunk_length : -1;
}
int sdfs_cdc_get_min_len(const sdfs_cdc_engine* e) {
    Reg::Use u(reg(), e);
    return u.ok() ? (int)u.set().devs[0]->prm.min_len : -1;
}
int sdfs_cdc_set_seed(sdfs_cdc_engine* e, int) {
    USE_OR_FAIL(u, e);
    return SDFS_CDC_OK;
}
int sdfs_cdc_digest_len(const sdfs_cdc_engine* e) {
    Reg::Use u(reg(), e);
    return u.ok() ? (int)u.set().devs[0]->digest_len : -1;
}
uint32_t sdfs_cdc_slot_cap(const sdfs_cdc_engine* e, uint64_t buf_len) {
    Reg::Use u(reg(), e);
    return u.ok() ? slot_cap_for(u.set().devs[0]->prm, buf_len) : 0;
}

int sdfs_cdc_run_device(sdfs_cdc_engine* e, const uint8_t* d_data, const uint64_t* d_offs, const uint32_t* d_lens,
                        uint32_t nbuf, uint32_t uniform_len, uint64_t buffer_id_base, const sdfs_cdc_dev_out* out,
                        void* stream) {
    USE_OR_FAIL(u, e);
    if (!uniform_len)
        return fail(SDFS_CDC_EINVAL, "sdfs_cdc_run_device: ragged layouts need sdfs_cdc_run_device_ragged");
    (void)d_offs;
    (void)d_lens;
    size_t i;
    const int rc = dev_of_ptr(u.set(), d_data, &i);
    if (rc) return rc;
    return dev_run_device(u.set().devs[i].get(), d_data, nbuf, uniform_len, buffer_id_base, out,
                          reinterpret_cast<hipStream_t>(stream));
}

int sdfs_cdc_run_device_ragged(sdfs_cdc_engine* e, const uint8_t* d_data, uint64_t data_bytes, const uint64_t* d_offs,
                               const uint32_t* d_lens, uint32_t nbuf, uint64_t buffer_id_base,
                               const sdfs_cdc_dev_out* out, void* stream) {
    USE_OR_FAIL(u, e);
    size_t i;
    const int rc = dev_of_ptr(u.set(), d_data, &i);
    if (rc) return rc;
    return dev_run_device_ragged(u.set().devs[i].get(), d_data, data_bytes, d_offs, d_lens, nbuf, buffer_id_base, out,
                                 reinterpret_cast<hipStream_t>(stream));
}

int sdfs_cdc_set_timing(sdfs_cdc_engine* e, int nruns) { return sdfs_cdc_set_timing_mask(e, nruns, 0xFFFFFFFFu); }

int sdfs_cdc_set_timing_mask(sdfs_cdc_engine* e, int nruns, uint32_t stage_mask) {
    USE_OR_FAIL(u, e);
    if (nruns < 0 || nruns > 4096) return fail(SDFS_CDC_EINVAL, "timing slots %d", nruns);
    for (auto& d : u.set().devs) {
        const int rc = dev_set_timing_mask(d.get(), nruns, stage_mask);
        if (rc) return rc;
    }
    return SDFS_CDC_OK;
}

int sdfs_cdc_kernel_times_on(sdfs_cdc_engine* e, int dev_index, const char** names, float* ms, int n) {
    USE_OR_FAIL(u, e);
    if (dev_index < 0 || (size_t)dev_index >= u.set().ndev()) return fail(SDFS_CDC_EINVAL, "device index %d", dev_index);
    return dev_kernel_times(u.set().devs[dev_index].get(), names, ms, n);
}

int sdfs_cdc_kernel_times(sdfs_cdc_engine* e, const char** names, float* ms, int n) {
    return sdfs_cdc_kernel_times_on(e, 0, names, ms, n);
}

int sdfs_cdc_get_chunks_batch(sdfs_cdc_engine* e, const uint8_t* base, const uint64_t* offs, const uint32_t* lens,
                              uint32_t nbuf, uint32_t* counts, uint32_t* starts, uint32_t* lens_out,
                              uint8_t* digests, uint32_t cap) {
    USE_OR_FAIL(u, e);
    if (nbuf && (!base || !offs || !lens || !counts || !starts || !lens_out))
        return fail(SDFS_CDC_EINVAL, "null argument");
    Set& s = u.set();
    // Contiguous shares of the buffers, one per device, run concurrently (every buffer is chunked
    // from fresh state, so a share is an independent batch); at least kShareMin buffers per device.
    constexpr uint32_t kShareMin = 64;
    const uint32_t dl = s.devs[0]->digest_len;
    std::vector<std::string> errs(s.ndev());
    size_t bad = 0;
    const int rc = Reg::run_shares(
        s, nbuf, kShareMin,
        [&](size_t d, uint32_t b0, uint32_t b1) {
            const uint64_t o = (uint64_t)b0 * cap;
            const int r = dev_get_chunks_batch(s.devs[d].get(), base, offs + b0, lens + b0, b1 - b0, counts + b0,
                                               starts + o, lens_out + o, digests ? digests + o * dl : nullptr, cap);
            if (r) errs[d] = g_last_error;  // per-thread message, kept for the caller's thread
            return r;
        },
        &bad);
    if (rc) return fail(rc, "device %d: %s", s.ordinals[bad], errs[bad].c_str());
    return SDFS_CDC_OK;
}

int sdfs_cdc_get_chunks_fill(sdfs_cdc_engine* e, uint64_t stream_key, uint32_t len, sdfs_cdc_fill_fn fill, void* ctx,
                             uint32_t* starts, uint32_t* lens, uint8_t* digests, uint32_t cap, uint32_t* count) {
    if (!count) return fail(SDFS_CDC_EINVAL, "null argument");
    *count = 0;
    USE_OR_FAIL(u, e);
    if (len == 0) return SDFS_CDC_OK;  // an empty byte[] yields no Finger
    if (!fill || !starts || !lens) return fail(SDFS_CDC_EINVAL, "null buffer");
    Set& s = u.set();
    const size_t i = Reg::pick(s, stream_key != SDFS_CDC_NO_STREAM, stream_key);
    Reg::Load ld(s, i);
    int frc = 0;
    const int rc = dev_get_chunks(
        s.devs[i].get(), len,
        [&](uint8_t* dst) {
            frc = fill(ctx, dst, len);
            if (!frc) return 0;
            memset(dst, 0, len);  // the batch still scans this request's bytes: defined ones
            return (int)SDFS_CDC_EINVAL;
        },
        starts, lens, digests, cap, count);
    if (frc) {
        *count = 0;
        return fail(SDFS_CDC_EINVAL, "getChunks: fill callback failed (%d)", frc);
    }
    return rc;
}

static int copy_fill(void* ctx, uint8_t* dst, uint32_t len) {
    memcpy(dst, ctx, len);
    return 0;
}

int sdfs_cdc_get_chunks_stream(sdfs_cdc_engine* e, uint64_t stream_key, const uint8_t* buf, uint32_t len,
                               uint32_t* starts, uint32_t* lens, uint8_t* digests, uint32_t cap, uint32_t* count) {
    if (len && !buf) return fail(SDFS_CDC_EINVAL, "null buffer");
    return sdfs_cdc_get_chunks_fill(e, stream_key, len, copy_fill, const_cast<uint8_t*>(buf), starts, lens, digests,
                                    cap, count);
}

int sdfs_cdc_get_chunks(sdfs_cdc_engine* e, const uint8_t* buf, uint32_t len, uint32_t* starts, uint32_t* lens,
                        uint8_t* digests, uint32_t cap, uint32_t* count) {
    return sdfs_cdc_get_chunks_stream(e, SDFS_CDC_NO_STREAM, buf, len, starts, lens, digests, cap, count);
}

int sdfs_cdc_get_hash(sdfs_cdc_engine* e, const uint8_t* data, uint64_t len, uint8_t* digest) {
    if (!digest || (len && !data)) return fail(SDFS_CDC_EINVAL, "null argument");
    if (len > 0xFFFFFFFFull) return fail(SDFS_CDC_EINVAL, "getHash input > 4 GiB");
    USE_OR_FAIL(u, e);
    Set& s = u.set();
    const size_t i = Reg::pick(s, false, 0);
    Reg::Load ld(s, i);
    return dev_get_hash(s.devs[i].get(), data, len, digest);
}

int sdfs_cdc_queue_stats(sdfs_cdc_engine* e, uint64_t* batches, uint64_t* requests) {
    USE_OR_FAIL(u, e);
    uint64_t b = 0, r = 0;
    for (auto& d : u.set().devs) {
        std::lock_guard<std::mutex> lk(d->q_init);
        if (d->q) {
            b += d->q->batches();
            r += d->q->requests();
        }
    }
    if (batches) *batches = b;
    if (requests) *requests = r;
    return SDFS_CDC_OK;
}

int sdfs_cdc_queue_early(sdfs_cdc_engine* e, uint64_t* early) {
    USE_OR_FAIL(u, e);
    uint64_t n = 0;
    for (auto& d : u.set().devs) {
        std::lock_guard<std::mutex> lk(d->q_init);
        if (d->q) n += d->q->early();
    }
    if (early) *early = n;
    return SDFS_CDC_OK;
}

int sdfs_cdc_queue_timing(sdfs_cdc_engine* e, double* fill_us, double* copy_us, double* device_us) {
    USE_OR_FAIL(u, e);
    double f = 0, c = 0, dv = 0, wsum = 0;
    for (auto& d : u.set().devs) {
        std::lock_guard<std::mutex> lk(d->q_init);
        if (!d->q) continue;
        double a, b, x;
        d->q->timing(&a, &b, &x);
        const double w = (double)d->q->batches();
        f += a * w;
        c += b * w;
        dv += x * w;
        wsum += w;
    }
    if (wsum > 0) f /= wsum, c /= wsum, dv /= wsum;
    if (fill_us) *fill_us = f;
    if (copy_us) *copy_us = c;
    if (device_us) *device_us = dv;
    return SDFS_CDC_OK;
}

int sdfs_cdc_host_register(void* p, uint64_t n) {
    if (!p || !n) return fail(SDFS_CDC_EINVAL, "null or empty region");
    HIP_TRY(hipHostRegister(p, n, hipHostRegisterPortable));  // pinned for every device of a set
    return SDFS_CDC_OK;
}

int sdfs_cdc_host_unregister(void* p) {
    if (!p) return fail(SDFS_CDC_EINVAL, "null region");
    HIP_TRY(hipHostUnregister(p));
    return SDFS_CDC_OK;
}

int sdfs_cdc_hash_device(sdfs_cdc_engine* e, const uint8_t* d_data, const uint64_t* d_offs, const uint32_t* d_lens,
                         const uint32_t* d_count, uint64_t n_max, uint8_t* d_digests, void* stream) {
    USE_OR_FAIL(u, e);
    if (n_max && (!d_data || !d_offs || !d_lens || !d_digests)) return fail(SDFS_CDC_EINVAL, "null argument");
    size_t i = 0;
    if (n_max) {
        const int rc = dev_of_ptr(u.set(), d_data, &i);
        if (rc) return rc;
    }
    DevEngine* d = u.set().devs[i].get();
    std::lock_guard<std::mutex> lk(d->mu);
    HIP_TRY(hipSetDevice(d->prm.device));
    return hash_extents(d, d_data, d_offs, d_lens, d_count, n_max, d_digests, reinterpret_cast<hipStream_t>(stream));
}

int sdfs_cdc_get_hash_batch(sdfs_cdc_engine* e, const uint8_t* base, const uint64_t* offs, const uint32_t* lens,
                            uint32_t n, uint8_t* digests) {
    USE_OR_FAIL(u, e);
    if (n == 0) return SDFS_CDC_OK;
    if (!base || !offs || !lens || !digests) return fail(SDFS_CDC_EINVAL, "null argument");
    Set& s = u.set();
    const size_t i = Reg::pick(s, false, 0);
    Reg::Load ld(s, i);
    return dev_get_hash_batch(s.devs[i].get(), base, offs, lens, n, digests);
}

int sdfs_cdc_synth_device(sdfs_cdc_engine* e, uint8_t* d_out, uint64_t n, uint64_t seed, uint64_t stream,
                          uint64_t offset, void* stream_handle) {
    USE_OR_FAIL(u, e);
    size_t i;
    const int rc = dev_of_ptr(u.set(), d_out, &i);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(u.set().ordinals[i]));
    hipStream_t s = reinterpret_cast<hipStream_t>(stream_handle);  // NULL = the HIP null stream
    HIP_TRY(launch_synth(d_out, n, seed, stream, offset, s));
    return SDFS_CDC_OK;
}

int sdfs_cdc_stream_sync(sdfs_cdc_engine* e) {
    USE_OR_FAIL(u, e);
    for (auto& d : u.set().devs) {
        HIP_TRY(hipSetDevice(d->prm.device));
        HIP_TRY(hipStreamSynchronize(d->stream));
    }
    return SDFS_CDC_OK;
}

int sdfs_cdc_allgather_records(sdfs_cdc_engine* e, uint8_t* const* records, const uint64_t* records_cap,
                               const uint32_t* const* d_totals, uint8_t* const* gathered, uint64_t gathered_cap,
                               uint32_t* counts, uint64_t* stride, void* const* streams) {
    USE_OR_FAIL(u, e);
    if (!records || !records_cap || !d_totals || !gathered || !counts || !stride)
        return fail(SDFS_CDC_EINVAL, "null argument");
    Set& s = u.set();
    const int n = (int)s.ndev();
    for (int i = 0; i < n; i++)
        if (!records[i] || !d_totals[i] || !gathered[i]) return fail(SDFS_CDC_EINVAL, "null table of device %d", i);
    Coll* c = nullptr;
    int rc = coll_ready(s, &c);
    if (rc) return rc;
    const RcclApi* api = rccl_api();
    auto st = [&](int i) { return streams ? reinterpret_cast<hipStream_t>(streams[i]) : (hipStream_t) nullptr; };
    std::lock_guard<std::mutex> lk(s.coll_mu);  // one exchange of the set at a time (shared count buffers)
    // 1. counts: one u32 per device, gathered on every device; device 0's copy to the host
    rc = grouped_all_gather(api, s, [&](int i) {
        return api->all_gather(d_totals[i], c->d_counts[i], 1, kNcclUint32, c->comms[i], st(i));
    });
    if (rc) return rc;
    HIP_TRY(hipSetDevice(s.ordinals[0]));
    HIP_TRY(hipMemcpyAsync(c->h_counts, c->d_counts[0], 4ull * n, hipMemcpyDeviceToHost, st(0)));
    HIP_TRY(hipStreamSynchronize(st(0)));
    uint64_t m = 0;
    for (int i = 0; i < n; i++) {
        counts[i] = c->h_counts[i];
        m = std::max<uint64_t>(m, counts[i]);
    }
    for (int i = 0; i < n; i++)
        if (records_cap[i] < m)
            return fail(SDFS_CDC_ECAP, "device %d holds %llu records, the largest table has %llu", i,
                        (unsigned long long)records_cap[i], (unsigned long long)m);
    if ((uint64_t)n * m > gathered_cap)
        return fail(SDFS_CDC_ECAP, "gathered table of %llu records > capacity %llu", (unsigned long long)((uint64_t)n * m),
                    (unsigned long long)gathered_cap);
    *stride = m;
    if (m == 0) return SDFS_CDC_OK;
    // 2. the tables, padded to the largest count: device j's records at gathered[i] + j*m*48
    return grouped_all_gather(api, s, [&](int i) {
        return api->all_gather(records[i], gathered[i], m * SDFS_CDC_RECORD_BYTES, kNcclUint8, c->comms[i], st(i));
    });
}

#ifdef SDFS_TUNING
// measurement only (tuning library): where fingerprint variant 50 writes its per-wave stamps
// (8 u64 per 64 tasks; device memory the caller owns, or null)
int sdfs_cdc_tuning_set_stamps(void* dev_ptr) {
    g_stamps = static_cast<uint64_t*>(dev_ptr);
    return SDFS_CDC_OK;
}
#endif

}  // extern "C"
