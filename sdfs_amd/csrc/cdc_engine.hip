// cdc_engine.hip — host side of the C-ABI (include/sdfs_cdc.h): engine lifecycle, device
// workspace, the device-resident pipeline, and the host-buffer paths (getChunks / getHash /
// batched getChunks) with pinned staging.  Drop-in for org.opendedup.hashing.AbstractHashEngine
// (AbstractHashEngine.java:24-39) as implemented by VariableSha256HashEngine /
// VariableMD5HashEngine (VariableSha256HashEngine.java:41-121, VariableMD5HashEngine.java:37-108).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/sdfs_cdc.h"
#include "cdc_internal.h"

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

// shared with the other C-ABI translation units (dedup_index.hip)
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

// Rolling-hash tables (same definition as the jar's precompute), laid out as the
// scan kernel's LDS image with `copies` lane-private copies (cdc_internal.h).
std::vector<uint8_t> build_table_image(uint64_t poly, uint32_t window, int copies) {
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
    hipError_t ensure(size_t want) {
        if (want <= n && p) return hipSuccess;
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

// timed stages (kernel_times order); "pipeline" = device time from the first enqueue to the last
// kernel of the run on the caller's stream (the stages overlap when the run is sub-batched)
constexpr int kNumTimed = 7;
const char* kKernelNames[kNumTimed] = {"prep", "cdc_scan", "cdc_resolve", "cdc_prefix", "cdc_scatter",
                                       "chunk_hash", "pipeline"};
enum { K_PREP = 0, K_SCAN, K_RESOLVE, K_PREFIX, K_SCATTER, K_HASH, K_PIPE };
constexpr int kMaxParts = 16;
constexpr int kEvPerRun = 2 * (kMaxParts * 5 + 2);

// One slot of the double-buffered host path (host_batch): pinned staging in and out, the
// device copy of the packed batch and its output slots.  While the GPU chunks the batch in one
// slot, the host packs the next batch into the other and unpacks the previous one's results.
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

// Pageable caller buffers -> pinned staging, split over a small persistent thread pool (the
// host memcpy, not PCIe, bounds the host path when it runs on one thread).
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
        drain(p);  // the calling thread copies too
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

}  // namespace

struct sdfs_cdc_engine {
    sdfs_cdc_params prm{};
    int degree = 0;
    int num_cus = 256;
    uint32_t seg_len = 4096;  // bytes of one buffer per lane (multiple of the variant's block)
    int scan_variant = 0;
    int hash_variant = 0;
    int hash_wg_per_cu = 2;  // persistent hash variant: 256-thread workgroups per CU
    ScanVariantInfo scan_info{};
    uint32_t first_off = 0;
    uint32_t bin_shift = 0, nbins = 1;
    uint32_t digest_len = 32;
    hipStream_t stream = nullptr;
    std::mutex mu;  // one engine context: calls are serialised (DESIGN.md "Host edge")

    DevBuf<uint8_t> tab_image;
    DevBuf<uint8_t> zero_page;
    // workspace for run_device
    DevBuf<uint32_t> bitmap;
    DevBuf<uint64_t> seg_prefix;
    DevBuf<uint32_t> small;  // hist[kMaxBins] | cursor[kMaxBins] | overflow[1]
    DevBuf<uint32_t> rec_base;
    DevBuf<uint32_t> tasks;
    DevBuf<uint32_t> spec_starts, spec_cnt, spec_next;  // sectioned cut walk of very long buffers
    // getHash device buffers and pinned staging
    DevBuf<uint8_t> h_data;
    DevBuf<uint32_t> o_starts;
    DevBuf<uint8_t> o_digests;
    DevBuf<uint32_t> x_scratch;  // extent ordering: hist | cursor | total, then starts | tasks
    DevBuf<uint8_t> x_data;      // host-batch staging of getHash in bulk
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

    // sub-batch pipeline: scan of part k+1 on s_scan overlaps resolve..hash of part k on s_post.
    // Measured NEGATIVE on MI355X (4 GiB step: 1 part 4.84 ms, 2 parts 7.0, 4 parts 9.7, 8 parts
    // 17.4: the persistent 128 KiB-LDS scan workgroups and the hash workgroups starve each other
    // in the dispatcher), so the default is 1 part; kept for experiments.
    int parts = 1;
    uint64_t part_min_bytes = 512ull << 20;
    hipStream_t s_scan = nullptr, s_post = nullptr;
    hipEvent_t ev_in = nullptr, ev_done = nullptr;
    hipEvent_t ev_scan[kMaxParts] = {};
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
    if (p->pred_mask >> d) return fail(SDFS_CDC_EINVAL, "pred_mask has bits above the fp degree");
    return SDFS_CDC_OK;
}

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

uint32_t slot_cap_for(const sdfs_cdc_params& p, uint64_t len) {
    const uint64_t shortest_cut = p.min_cmp == SDFS_CDC_MIN_GT ? (uint64_t)p.min_len + 1 : std::max<uint64_t>(p.min_len, 1);
    const uint64_t shortest = std::min<uint64_t>(shortest_cut, p.max_len);
    return (uint32_t)(len / shortest + 2);
}

// Records a start event for stage `kid` on stream `st` (timing runs only); returns the pair index.
int t_begin(sdfs_cdc_engine* e, int kid, hipStream_t st) {
    if (!e->run || !((e->timing_mask >> kid) & 1u)) return -1;
    const int i = (int)e->run->kid.size();
    if (2 * i + 1 >= kEvPerRun) return -1;
    e->run->kid.push_back(kid);
    (void)hipEventRecord(e->run->ev[2 * i], st);
    return i;
}
void t_end(sdfs_cdc_engine* e, int i, hipStream_t st) {
    if (e->run && i >= 0) (void)hipEventRecord(e->run->ev[2 * i + 1], st);
}

// The device pipeline, enqueued behind everything already on `s` and completing on `s`.  Large
// uniform batches are split into `parts` sub-batches: the scan of part k+1 (engine stream
// s_scan) overlaps resolve/prefix/scatter/hash of part k (s_post), so the latency-bound scan and
// the VALU-bound hash share the CUs (DESIGN.md "Pipeline").  Caller holds e->mu.
int run_pipeline(sdfs_cdc_engine* e, const uint8_t* d_data, uint64_t data_bytes, const uint64_t* d_offs,
                 const uint32_t* d_lens, uint32_t nbuf, uint32_t uniform_len, uint64_t buffer_id_base,
                 const sdfs_cdc_dev_out* out, hipStream_t s, uint64_t max_buf_len = 0) {
    if (!out || !out->counts || !out->starts || !out->lens || !out->digests || !out->total)
        return fail(SDFS_CDC_EINVAL, "incomplete sdfs_cdc_dev_out");
    if (uniform_len && (uniform_len & 63)) return fail(SDFS_CDC_EINVAL, "uniform_len must be a multiple of 64");
    if (!uniform_len && (!d_offs || !d_lens)) return fail(SDFS_CDC_EINVAL, "offs/lens required without uniform_len");
    if ((reinterpret_cast<uintptr_t>(d_data) & 63) != 0) return fail(SDFS_CDC_EINVAL, "d_data must be 64-byte aligned");
    if (uniform_len) data_bytes = (uint64_t)nbuf * uniform_len;
    if (uniform_len && out->cap < slot_cap_for(e->prm, uniform_len))
        return fail(SDFS_CDC_ECAP, "cap %u < slot_cap %u", out->cap, slot_cap_for(e->prm, uniform_len));

    e->run = nullptr;
    if (e->timing_slots > 0) {
        e->run = &e->ev_runs[e->runs_recorded % e->timing_slots];
        e->run->kid.clear();
    }
    const int tpipe = t_begin(e, K_PIPE, s);
    if (nbuf == 0) {
        HIP_TRY(hipMemsetAsync(out->total, 0, 4, s));
        t_end(e, tpipe, s);
        if (e->run) e->runs_recorded++;
        return SDFS_CDC_OK;
    }

    // sub-batch split (uniform layout only): parts of whole buffers, each >= part_min_bytes
    uint32_t parts = 1;
    if (uniform_len && e->parts > 1) {
        const uint64_t by_size = data_bytes / std::max<uint64_t>(e->part_min_bytes, 1);
        parts = (uint32_t)std::min<uint64_t>({(uint64_t)e->parts, by_size, (uint64_t)nbuf, (uint64_t)kMaxParts});
        parts = std::max<uint32_t>(parts, 1);
    }

    // workspace
    const uint64_t nwords = ((data_bytes + 63) / 64) * 2 + 2;
    HIP_TRY(e->bitmap.ensure(nwords));
    constexpr uint32_t kSmall = 2 * kMaxBins + 8;  // hist | cursor | overflow, total, base_in, base_out ..
    HIP_TRY(e->small.ensure((uint64_t)kSmall * parts + 8));
    HIP_TRY(e->rec_base.ensure(nbuf));
    const uint64_t nslots = (uint64_t)nbuf * out->cap;
    HIP_TRY(e->tasks.ensure(nslots));
    uint32_t* running = e->small.p + (uint64_t)kSmall * parts;  // running record base per part
    hipStream_t sscan = parts > 1 ? e->s_scan : s;
    hipStream_t spost = parts > 1 ? e->s_post : s;
    if (parts > 1) {
        HIP_TRY(hipEventRecord(e->ev_in, s));
        HIP_TRY(hipStreamWaitEvent(sscan, e->ev_in, 0));
        HIP_TRY(hipStreamWaitEvent(spost, e->ev_in, 0));
    }
    {
        const int t = t_begin(e, K_PREP, spost);
        HIP_TRY(hipMemsetAsync(e->small.p, 0, ((uint64_t)kSmall * parts + 8) * sizeof(uint32_t), spost));
        if (!uniform_len) {
            HIP_TRY(e->seg_prefix.ensure((uint64_t)nbuf + 1));
            HIP_TRY(launch_seg_prefix(d_lens, nbuf, e->seg_len, e->seg_prefix.p, spost));
        }
        t_end(e, t, spost);
    }
    if (!uniform_len && sscan != spost) return fail(SDFS_CDC_EINVAL, "internal: ragged batches are not split");

    const bool pred64 = (e->prm.pred_mask >> 32) != 0;
    for (uint32_t p = 0; p < parts; p++) {
        const uint32_t b0 = (uint32_t)((uint64_t)nbuf * p / parts);
        const uint32_t b1 = (uint32_t)((uint64_t)nbuf * (p + 1) / parts);
        const uint32_t nb = b1 - b0;
        const uint64_t byte0 = uniform_len ? (uint64_t)b0 * uniform_len : 0;
        const uint8_t* data_p = d_data + byte0;
        uint32_t* bitmap_p = e->bitmap.p + (byte0 >> 5);
        uint32_t* small_p = e->small.p + (uint64_t)kSmall * p;
        uint32_t* hist = small_p;
        uint32_t* cursor = small_p + kMaxBins;
        uint32_t* part_total = small_p + 2 * kMaxBins + 1;
        const uint64_t slot0 = (uint64_t)b0 * out->cap;

        // ---- scan (s_scan)
        ScanArgs sa{};
        sa.data = data_p;
        sa.offs = d_offs;
        sa.lens = d_lens;
        sa.bitmap = bitmap_p;
        sa.nbuf = nb;
        sa.uniform_len = uniform_len;
        sa.seg_len = e->seg_len;
        sa.jshift = (uint32_t)(e->degree - 40);
        sa.mask_lo = (uint32_t)e->prm.pred_mask;
        sa.mask_hi = (uint32_t)(e->prm.pred_mask >> 32);
        sa.val_lo = (uint32_t)e->prm.pred_value;
        sa.val_hi = (uint32_t)(e->prm.pred_value >> 32);
        sa.tab_image = e->tab_image.p;
        sa.zero_page = e->zero_page.p;
        uint64_t seg_bound;
        if (uniform_len) {
            const uint64_t spb = (uniform_len + e->seg_len - 1) / e->seg_len;
            sa.total_segs = spb * nb;
            seg_bound = sa.total_segs;
        } else {
            sa.seg_prefix = e->seg_prefix.p;
            seg_bound = data_bytes / e->seg_len + nb;
        }
        ResolveArgs ra{};
        ra.bitmap = bitmap_p;
        ra.offs = d_offs;
        ra.lens = d_lens;
        ra.nbuf = nb;
        ra.uniform_len = uniform_len;
        ra.first_off = e->first_off;
        ra.max_len = e->prm.max_len;
        ra.cap = out->cap;
        ra.bin_shift = e->bin_shift;
        ra.nbins = e->nbins;
        ra.counts = out->counts + b0;
        ra.starts = out->starts + slot0;
        ra.clens = out->lens + slot0;
        ra.hist = hist;
        ra.overflow = e->small.p + 2 * kMaxBins;  // part 0's word: one flag for the whole run
        ra.max_buf_len = uniform_len ? uniform_len : max_buf_len;
        ra.sec_len = resolve_section_len(ra.max_buf_len, e->prm.max_len);
        if (ra.sec_len) {
            ra.nsec = (uint32_t)((ra.max_buf_len + ra.sec_len - 1) / ra.sec_len);
            ra.spec_cap = ra.sec_len / (e->first_off + 1) + 2;
            const uint64_t items = (uint64_t)nb * ra.nsec;
            HIP_TRY(e->spec_starts.ensure(items * ra.spec_cap));
            HIP_TRY(e->spec_cnt.ensure(items));
            HIP_TRY(e->spec_next.ensure(items));
            ra.spec_starts = e->spec_starts.p;
            ra.spec_cnt = e->spec_cnt.p;
            ra.spec_next = e->spec_next.p;
        }
        // one wave = one buffer: the fused scan variant resolves inside the scan kernel
        // (single stream only: the histogram it feeds is cleared on the post stream)
        const bool fused = e->scan_info.fuse && parts == 1 && uniform_len && e->scan_info.chains == 1 &&
                           (uint64_t)uniform_len == 64ull * e->seg_len && e->seg_len < 0xFFFFu;
        sa.fuse_resolve = fused ? 1u : 0u;
        sa.res = ra;
        const uint64_t per_block = (uint64_t)kScanThreads * e->scan_info.chains;
        uint64_t grid = (seg_bound + per_block - 1) / per_block;
        grid = std::min<uint64_t>(grid, (uint64_t)e->num_cus * e->scan_info.wg_per_cu);
        grid = std::max<uint64_t>(grid, 1);
        {
            const int t = t_begin(e, K_SCAN, sscan);
            HIP_TRY(launch_scan(sa, (int)e->prm.window, pred64, e->scan_variant, (int)grid, sscan));
            t_end(e, t, sscan);
        }
        if (parts > 1) {
            HIP_TRY(hipEventRecord(e->ev_scan[p], sscan));
            HIP_TRY(hipStreamWaitEvent(spost, e->ev_scan[p], 0));
        }

        // ---- resolve, prefix, scatter, hash (s_post)
        if (!fused) {
            const int t = t_begin(e, K_RESOLVE, spost);
            HIP_TRY(launch_resolve(ra, spost));
            t_end(e, t, spost);
        }
        PrefixArgs pa{};
        pa.counts = out->counts + b0;
        pa.nbuf = nb;
        pa.hist = hist;
        pa.nbins = e->nbins;
        pa.cursor = cursor;
        pa.rec_base = e->rec_base.p + b0;
        pa.total = part_total;
        pa.base_in = p ? running + p : nullptr;
        pa.base_out = running + p + 1;
        pa.grand_total = p + 1 == parts ? out->total : nullptr;
        {
            const int t = t_begin(e, K_PREFIX, spost);
            HIP_TRY(launch_prefix(pa, spost));
            t_end(e, t, spost);
        }
        ScatterArgs ca{};
        ca.counts = out->counts + b0;
        ca.clens = out->lens + slot0;
        ca.nbuf = nb;
        ca.cap = out->cap;
        ca.bin_shift = e->bin_shift;
        ca.nbins = e->nbins;
        ca.cursor = cursor;
        ca.tasks = e->tasks.p + slot0;
        {
            const int t = t_begin(e, K_SCATTER, spost);
            HIP_TRY(launch_scatter(ca, spost));
            t_end(e, t, spost);
        }
        HashArgs ha{};
    ha.zero_page = e->zero_page.p;
        ha.data = data_p;
        ha.offs = d_offs;
        ha.uniform_len = uniform_len;
        ha.tasks = e->tasks.p + slot0;
        ha.total = part_total;
        ha.starts = out->starts + slot0;
        ha.clens = out->lens + slot0;
        ha.rec_base = e->rec_base.p + b0;
        ha.cap = out->cap;
        ha.digests = out->digests + slot0 * 32;
        ha.records = out->records;
        ha.records_cap = out->records_cap;
        ha.buffer_id_base = buffer_id_base + b0;
        ha.algo = e->prm.hash_algo;
        ha.wave_ctr = small_p + 2 * kMaxBins + 2;  // zeroed with the rest of `small` above
        ha.persist_grid = (uint32_t)(e->num_cus * e->hash_wg_per_cu);
        {
            const int t = t_begin(e, K_HASH, spost);
            HIP_TRY(launch_hash(ha, (uint64_t)nb * out->cap, e->hash_variant, spost));
            t_end(e, t, spost);
        }
    }
    if (parts > 1) {
        HIP_TRY(hipEventRecord(e->ev_done, spost));
        HIP_TRY(hipStreamWaitEvent(s, e->ev_done, 0));
    }
    t_end(e, tpipe, s);
    if (e->run) e->runs_recorded++;
    return SDFS_CDC_OK;
}

// Results of the batch in slot `sl` (synchronises on it) -> the caller's arrays.
int drain_slot(sdfs_cdc_engine* e, HostSlot& sl, uint32_t* counts, uint32_t* starts, uint32_t* lens_out,
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
int host_batch_impl(sdfs_cdc_engine* e, const uint8_t* base, const uint64_t* offs, const uint32_t* lens,
                    uint32_t nbuf, uint32_t* counts, uint32_t* starts, uint32_t* lens_out, uint8_t* digests,
                    uint32_t cap) {
    // 256 MiB per slot: smaller batches leave most CUs idle and pay the per-batch fixed costs
    // (64 MiB: 26.5 GiB/s end to end, 256 MiB: 45.9 GiB/s from pinned memory; scripts/h2d_probe.py)
    const uint64_t staging = e->prm.max_batch_bytes ? e->prm.max_batch_bytes : (256ull << 20);
    if (!e->pool && e->copy_threads > 1) e->pool.reset(new CopyPool(e->copy_threads - 1));
    hipStream_t s = e->stream;
    std::vector<CopyPiece> pieces;
    uint32_t b0 = 0, k = 0;
    // is the caller's input pinned host memory (both ends of the span)?
    bool host_pinned = false;
    {
        uint64_t lo = UINT64_MAX, hi = 0;
        for (uint32_t i = 0; i < nbuf; i++) {
            lo = std::min<uint64_t>(lo, offs[i]);
            hi = std::max<uint64_t>(hi, offs[i] + lens[i]);
        }
        hipPointerAttribute_t a0, a1;
        if (hi > lo && hipPointerGetAttributes(&a0, base + lo) == hipSuccess &&
            hipPointerGetAttributes(&a1, base + hi - 1) == hipSuccess)
            host_pinned = a0.type == hipMemoryTypeHost && a1.type == hipMemoryTypeHost;
        (void)hipGetLastError();  // pageable memory reports an error here: clear it
    }
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
        // Pinned (hipHostMalloc'd or hipHostRegister'ed) input whose buffers sit back to back at
        // 64-byte multiples: copy it to the GPU straight from the caller's memory (no staging).
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
        rc = run_pipeline(e, sl.data.p, bytes, sl.offs.p, sl.lens.p, n, 0, 0, &out, s, maxlen);
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
        // the run-wide overflow flag, read before the next batch's pipeline clears it
        HIP_TRY(hipMemcpyAsync(povf, e->small.p + 2 * kMaxBins, 4, hipMemcpyDeviceToHost, s));
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

int host_batch(sdfs_cdc_engine* e, const uint8_t* base, const uint64_t* offs, const uint32_t* lens, uint32_t nbuf,
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
    return SDFS_CDC_OK;
}

int sdfs_cdc_create(const sdfs_cdc_params* p, sdfs_cdc_engine** out) {
    if (!out) return fail(SDFS_CDC_EINVAL, "null out");
    *out = nullptr;
    int rc = validate(p);
    if (rc) return rc;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(SDFS_CDC_ENODEV, "no HIP device");
    if (p->device < 0 || p->device >= ndev) return fail(SDFS_CDC_ENODEV, "device %d of %d", p->device, ndev);
    HIP_TRY(hipSetDevice(p->device));
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, p->device));
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(SDFS_CDC_ENODEV, "device %d is %s, this build targets gfx950", p->device, prop.gcnArchName);
    auto* e = new sdfs_cdc_engine();
    e->prm = *p;
    e->degree = poly_degree(p->poly);
    e->num_cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    e->first_off = p->min_cmp == SDFS_CDC_MIN_GT ? p->min_len : (p->min_len ? p->min_len - 1 : 0);
    e->digest_len = p->hash_algo == SDFS_CDC_SHA256 ? 32 : (p->hash_algo == SDFS_CDC_SHA256_160 ? 20 : 16);
    // bins over SHA block counts: maxLen chunk = (max_len + 8)/64 + 1 blocks
    const uint32_t maxblocks = (p->max_len + 8) / 64 + 1;
    e->bin_shift = 0;
    while ((maxblocks >> e->bin_shift) >= (uint32_t)kMaxBins) e->bin_shift++;
    e->nbins = (maxblocks >> e->bin_shift) + 1;
    if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&e->s_scan, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&e->s_post, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&e->ev_in, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&e->ev_done, hipEventDisableTiming) != hipSuccess ||
        hipStreamCreateWithFlags(&e->s_h2d, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&e->hs[0].h2d, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&e->hs[0].done, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&e->hs[1].h2d, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&e->hs[1].done, hipEventDisableTiming) != hipSuccess) {
        sdfs_cdc_destroy(e);
        return fail(SDFS_CDC_EHIP, "stream/event creation failed");
    }
    if (const char* v = getenv("SDFS_COPY_THREADS")) e->copy_threads = std::max(1, std::min(atoi(v), 64));
    for (auto& ev : e->ev_scan)
        if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
            sdfs_cdc_destroy(e);
            return fail(SDFS_CDC_EHIP, "event creation failed");
        }
    if (const char* v = getenv("SDFS_PIPE_PARTS")) e->parts = std::max(1, std::min(atoi(v), kMaxParts));
    // tuning overrides for experiments (DESIGN.md "Scan variants"); production uses variant 0
    if (const char* v = getenv("SDFS_SCAN_VARIANT")) e->scan_variant = atoi(v);
    if (const char* v = getenv("SDFS_SEG_LEN")) e->seg_len = (uint32_t)atoi(v);
    if (const char* v = getenv("SDFS_HASH_VARIANT")) e->hash_variant = atoi(v);
    if (const char* v = getenv("SDFS_HASH_WG_PER_CU")) e->hash_wg_per_cu = std::max(1, atoi(v));
    e->scan_info = scan_variant_info(e->scan_variant);
    if (e->scan_info.copies == 0 || e->seg_len == 0 || (e->seg_len % e->scan_info.blk) != 0) {
        sdfs_cdc_destroy(e);
        return fail(SDFS_CDC_EINVAL, "bad scan variant/segment length");
    }
    std::vector<uint8_t> img = build_table_image(p->poly, p->window, e->scan_info.copies);
    if (e->zero_page.ensure(256) != hipSuccess || hipMemset(e->zero_page.p, 0, 256) != hipSuccess ||
        e->tab_image.ensure(img.size()) != hipSuccess ||
        hipMemcpy(e->tab_image.p, img.data(), img.size(), hipMemcpyHostToDevice) != hipSuccess) {
        sdfs_cdc_destroy(e);
        return fail(SDFS_CDC_ENOMEM, "table upload failed");
    }
    *out = e;
    return SDFS_CDC_OK;
}

int sdfs_cdc_destroy(sdfs_cdc_engine* e) {
    if (!e) return SDFS_CDC_OK;
    {
        std::lock_guard<std::mutex> lk(e->mu);
        (void)hipSetDevice(e->prm.device);
        if (e->stream) (void)hipStreamSynchronize(e->stream);
        e->tab_image.release();
        e->zero_page.release();
        e->bitmap.release();
        e->seg_prefix.release();
        e->small.release();
        e->rec_base.release();
        e->tasks.release();
        e->spec_starts.release();
        e->spec_cnt.release();
        e->spec_next.release();
        e->h_data.release();
        e->o_starts.release();
        e->o_digests.release();
        e->x_scratch.release();
        e->x_data.release();
        e->x_offs.release();
        e->x_lens.release();
        e->x_digests.release();
        if (e->pin_data) (void)hipHostFree(e->pin_data);
        if (e->s_h2d) (void)hipStreamSynchronize(e->s_h2d);
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
        if (e->s_scan) (void)hipStreamSynchronize(e->s_scan);
        if (e->s_post) (void)hipStreamSynchronize(e->s_post);
        for (auto& run : e->ev_runs)
            for (auto& ev : run.ev)
                if (ev) (void)hipEventDestroy(ev);
        for (auto& ev : e->ev_scan)
            if (ev) (void)hipEventDestroy(ev);
        if (e->ev_in) (void)hipEventDestroy(e->ev_in);
        if (e->ev_done) (void)hipEventDestroy(e->ev_done);
        if (e->stream) (void)hipStreamDestroy(e->stream);
        if (e->s_scan) (void)hipStreamDestroy(e->s_scan);
        if (e->s_post) (void)hipStreamDestroy(e->s_post);
        if (e->s_h2d) (void)hipStreamDestroy(e->s_h2d);
    }
    delete e;
    return SDFS_CDC_OK;
}

int sdfs_cdc_is_variable_length(const sdfs_cdc_engine*) { return 1; }
int sdfs_cdc_get_max_len(const sdfs_cdc_engine* e) { return e ? (int)e->prm.chunk_length : -1; }
int sdfs_cdc_get_min_len(const sdfs_cdc_engine* e) { return e ? (int)e->prm.min_len : -1; }
int sdfs_cdc_set_seed(sdfs_cdc_engine*, int) { return SDFS_CDC_OK; }
int sdfs_cdc_digest_len(const sdfs_cdc_engine* e) { return e ? (int)e->digest_len : -1; }
uint32_t sdfs_cdc_slot_cap(const sdfs_cdc_engine* e, uint64_t buf_len) { return e ? slot_cap_for(e->prm, buf_len) : 0; }

int sdfs_cdc_run_device(sdfs_cdc_engine* e, const uint8_t* d_data, const uint64_t* d_offs, const uint32_t* d_lens,
                        uint32_t nbuf, uint32_t uniform_len, uint64_t buffer_id_base, const sdfs_cdc_dev_out* out,
                        void* stream) {
    if (!e) return fail(SDFS_CDC_EINVAL, "null engine");
    if (!uniform_len)
        return fail(SDFS_CDC_EINVAL, "sdfs_cdc_run_device: ragged layouts need sdfs_cdc_run_device_ragged");
    std::lock_guard<std::mutex> lk(e->mu);
    HIP_TRY(hipSetDevice(e->prm.device));
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);  // NULL = the HIP null stream
    return run_pipeline(e, d_data, 0, d_offs, d_lens, nbuf, uniform_len, buffer_id_base, out, s);
}

int sdfs_cdc_run_device_ragged(sdfs_cdc_engine* e, const uint8_t* d_data, uint64_t data_bytes, const uint64_t* d_offs,
                               const uint32_t* d_lens, uint32_t nbuf, uint64_t buffer_id_base,
                               const sdfs_cdc_dev_out* out, void* stream) {
    if (!e) return fail(SDFS_CDC_EINVAL, "null engine");
    std::lock_guard<std::mutex> lk(e->mu);
    HIP_TRY(hipSetDevice(e->prm.device));
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);  // NULL = the HIP null stream
    // the longest buffer is not known on the host: a few buffers sharing data_bytes are treated as
    // long (LDS-staged cut walk), many as their mean length
    const uint64_t max_len_hint = nbuf <= 4u * (uint32_t)e->num_cus ? data_bytes : data_bytes / (nbuf ? nbuf : 1);
    return run_pipeline(e, d_data, data_bytes, d_offs, d_lens, nbuf, 0, buffer_id_base, out, s, max_len_hint);
}

int sdfs_cdc_set_timing(sdfs_cdc_engine* e, int nruns) { return sdfs_cdc_set_timing_mask(e, nruns, 0xFFFFFFFFu); }

int sdfs_cdc_set_timing_mask(sdfs_cdc_engine* e, int nruns, uint32_t stage_mask) {
    if (!e) return fail(SDFS_CDC_EINVAL, "null engine");
    if (nruns < 0 || nruns > 4096) return fail(SDFS_CDC_EINVAL, "timing slots %d", nruns);
    std::lock_guard<std::mutex> lk(e->mu);
    e->timing_mask = stage_mask;
    HIP_TRY(hipSetDevice(e->prm.device));
    while ((int)e->ev_runs.size() < nruns) {
        sdfs_cdc_engine::TimedRun r;
        r.ev.assign(kEvPerRun, nullptr);
        for (auto& ev : r.ev) HIP_TRY(hipEventCreate(&ev));
        e->ev_runs.push_back(std::move(r));
    }
    e->timing_slots = nruns;
    e->runs_recorded = 0;
    return SDFS_CDC_OK;
}

int sdfs_cdc_kernel_times(sdfs_cdc_engine* e, const char** names, float* ms, int n) {
    if (!e) return fail(SDFS_CDC_EINVAL, "null engine");
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

int sdfs_cdc_set_pipeline(sdfs_cdc_engine* e, int parts, uint64_t part_min_bytes) {
    if (!e) return fail(SDFS_CDC_EINVAL, "null engine");
    if (parts < 1 || parts > kMaxParts) return fail(SDFS_CDC_EINVAL, "parts %d outside [1,%d]", parts, kMaxParts);
    std::lock_guard<std::mutex> lk(e->mu);
    e->parts = parts;
    e->part_min_bytes = part_min_bytes;
    return SDFS_CDC_OK;
}

int sdfs_cdc_get_chunks_batch(sdfs_cdc_engine* e, const uint8_t* base, const uint64_t* offs, const uint32_t* lens,
                              uint32_t nbuf, uint32_t* counts, uint32_t* starts, uint32_t* lens_out,
                              uint8_t* digests, uint32_t cap) {
    if (!e) return fail(SDFS_CDC_EINVAL, "null engine");
    if (nbuf && (!base || !offs || !lens || !counts || !starts || !lens_out))
        return fail(SDFS_CDC_EINVAL, "null argument");
    std::lock_guard<std::mutex> lk(e->mu);
    HIP_TRY(hipSetDevice(e->prm.device));
    return host_batch(e, base, offs, lens, nbuf, counts, starts, lens_out, digests, cap);
}

int sdfs_cdc_get_chunks(sdfs_cdc_engine* e, const uint8_t* buf, uint32_t len, uint32_t* starts, uint32_t* lens,
                        uint8_t* digests, uint32_t cap, uint32_t* count) {
    if (!e || !count) return fail(SDFS_CDC_EINVAL, "null argument");
    *count = 0;
    if (len == 0) return SDFS_CDC_OK;  // an empty byte[] yields no Finger
    if (!buf) return fail(SDFS_CDC_EINVAL, "null buffer");
    const uint64_t off = 0;
    std::lock_guard<std::mutex> lk(e->mu);
    HIP_TRY(hipSetDevice(e->prm.device));
    return host_batch(e, buf, &off, &len, 1, count, starts, lens, digests, cap);
}

int sdfs_cdc_get_hash(sdfs_cdc_engine* e, const uint8_t* data, uint64_t len, uint8_t* digest) {
    if (!e || !digest || (len && !data)) return fail(SDFS_CDC_EINVAL, "null argument");
    if (len > 0xFFFFFFFFull) return fail(SDFS_CDC_EINVAL, "getHash input > 4 GiB");
    std::lock_guard<std::mutex> lk(e->mu);
    HIP_TRY(hipSetDevice(e->prm.device));
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

namespace {
// fingerprints of n extents on the engine (caller holds e->mu and has set the device)
int hash_extents(sdfs_cdc_engine* e, const uint8_t* d_data, const uint64_t* d_offs, const uint32_t* d_lens,
                 const uint32_t* d_count, uint64_t n_max, uint8_t* d_digests, hipStream_t s) {
    if (n_max == 0) return SDFS_CDC_OK;
    if (n_max > 0xFFFFFFFFull) return fail(SDFS_CDC_EINVAL, "more than 2^32 extents");
    HIP_TRY(e->x_scratch.ensure(kExtentScratchWords + 2 * n_max));
    uint32_t* sc = e->x_scratch.p;
    ExtentArgs xa{d_lens, d_count, n_max, sc + kExtentScratchWords, sc + kExtentScratchWords + n_max,
                  sc + 1024, sc, sc + 512};
    HIP_TRY(launch_extent_order(xa, s));
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
    HIP_TRY(launch_hash(ha, n_max, 0, s));
    return SDFS_CDC_OK;
}
}  // namespace

int sdfs_cdc_host_register(void* p, uint64_t n) {
    if (!p || !n) return fail(SDFS_CDC_EINVAL, "null or empty region");
    HIP_TRY(hipHostRegister(p, n, hipHostRegisterDefault));
    return SDFS_CDC_OK;
}

int sdfs_cdc_host_unregister(void* p) {
    if (!p) return fail(SDFS_CDC_EINVAL, "null region");
    HIP_TRY(hipHostUnregister(p));
    return SDFS_CDC_OK;
}

int sdfs_cdc_hash_device(sdfs_cdc_engine* e, const uint8_t* d_data, const uint64_t* d_offs, const uint32_t* d_lens,
                         const uint32_t* d_count, uint64_t n_max, uint8_t* d_digests, void* stream) {
    if (!e) return fail(SDFS_CDC_EINVAL, "null engine");
    if (n_max && (!d_data || !d_offs || !d_lens || !d_digests)) return fail(SDFS_CDC_EINVAL, "null argument");
    std::lock_guard<std::mutex> lk(e->mu);
    HIP_TRY(hipSetDevice(e->prm.device));
    return hash_extents(e, d_data, d_offs, d_lens, d_count, n_max, d_digests, reinterpret_cast<hipStream_t>(stream));
}

int sdfs_cdc_get_hash_batch(sdfs_cdc_engine* e, const uint8_t* base, const uint64_t* offs, const uint32_t* lens,
                            uint32_t n, uint8_t* digests) {
    if (!e) return fail(SDFS_CDC_EINVAL, "null engine");
    if (n == 0) return SDFS_CDC_OK;
    if (!base || !offs || !lens || !digests) return fail(SDFS_CDC_EINVAL, "null argument");
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

int sdfs_cdc_synth_device(sdfs_cdc_engine* e, uint8_t* d_out, uint64_t n, uint64_t seed, uint64_t stream,
                          uint64_t offset, void* stream_handle) {
    if (!e) return fail(SDFS_CDC_EINVAL, "null engine");
    HIP_TRY(hipSetDevice(e->prm.device));
    hipStream_t s = reinterpret_cast<hipStream_t>(stream_handle);  // NULL = the HIP null stream
    HIP_TRY(launch_synth(d_out, n, seed, stream, offset, s));
    return SDFS_CDC_OK;
}

int sdfs_cdc_stream_sync(sdfs_cdc_engine* e) {
    if (!e) return fail(SDFS_CDC_EINVAL, "null engine");
    HIP_TRY(hipSetDevice(e->prm.device));
    HIP_TRY(hipStreamSynchronize(e->stream));
    return SDFS_CDC_OK;
}

}  // extern "C"
